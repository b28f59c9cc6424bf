#!/bin/bash
# L->R lines beside / after the packed strips for batches (MVSV_LINES_AUX -1 auto,
# 0 after, 1 beside launched first, 2 beside launched after): liveDisparity
# default and config 5 at 4 and 8 frames.  Usage: bash tools/gpu_r06_aux.sh TAG
set -o pipefail
TAG=${1:?TAG}; cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
for r in 1 2; do
for a in -1 1 2; do
  for f in 4 8; do
    MVSV_LINES_AUX=$a timeout -k 10 60 python tools/stage_times.py --frames $f --ndisp 64 --bs 9 --p1 648 --p2 2592 | sed "s/^/$a /" >> $O/ab.txt || exit 1
    MVSV_LINES_AUX=$a timeout -k 10 60 python tools/stage_times.py --frames $f | sed "s/^/$a /" >> $O/ab.txt || exit 1
  done
done
done
python - <<PY
import json
for l in open("$O/ab.txt"):
    v, j = l.split(" ", 1); d = json.loads(j)
    print(v, d["ndisp"], d["frames"], d["ms_per_call"], d["stages"].get("path_aggregation"))
PY
