#!/bin/bash
# Packed strip width A/B for batches (MVSV_STRIP_WAVES: 0 auto, wide, narrow):
# liveDisparity default (D 64: 15 / 8) and config 5 (D 256: 7 / 4) at 4 and 8 frames.
set -o pipefail
TAG=${1:?TAG}; cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
for r in 1 2; do
  for w in 0 15 8; do
    for f in 4 8; do
      MVSV_STRIP_WAVES=$w timeout -k 10 60 python tools/stage_times.py --frames $f --ndisp 64 --bs 9 --p1 648 --p2 2592 | sed "s/^/$w /" >> $O/ab.txt || exit 1
    done
  done
  for w in 0 7 4; do
    for f in 4 8; do
      MVSV_STRIP_WAVES=$w timeout -k 10 60 python tools/stage_times.py --frames $f | sed "s/^/$w /" >> $O/ab.txt || exit 1
    done
  done
done
python - <<PY
import json
for l in open("$O/ab.txt"):
    v, j = l.split(" ", 1); d = json.loads(j)
    print(v, d["ndisp"], d["frames"], d["ms_per_call"], d["stages"].get("path_aggregation"), d["stages"].get("path_strips"))
PY
