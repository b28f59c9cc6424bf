#!/bin/bash
# Side by side (u8 / u16 planes, P2 > 15) vs strips for small launches of
# D = 32 / 128 / 256 at liveDisparity's P1/P2.  Usage: bash tools/gpu_r06_sched2.sh TAG
set -o pipefail
TAG=${1:?TAG}; cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
for D in 32 128 256; do
  for f in 1 2 3; do
    for s in 0 2; do
      MVSV_PATH_SCHEDULE=$s timeout -k 10 60 python tools/stage_times.py --frames $f --ndisp $D --bs 9 --p1 648 --p2 2592 >> $O/sched2.jsonl || exit 1
    done
  done
done
for f in 1 2 3; do
  for s in 0 2; do
    MVSV_PATH_SCHEDULE=$s timeout -k 10 60 python tools/stage_times.py --frames $f --ndisp 64 --bs 9 --p1 648 --p2 2592 --mode 1 >> $O/sched2.jsonl || exit 1
  done
done
python - <<PY
import json
for l in open("$O/sched2.jsonl"):
    d=json.loads(l); print(d["ndisp"], d["mode"], d["frames"], d["env"].get("MVSV_PATH_SCHEDULE"), d["ms_per_call"], d["stages"].get("path_aggregation"), d["stages"].get("final_wta_lr"))
PY
