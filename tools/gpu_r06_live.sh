#!/bin/bash
# liveDisparity default create(0, 64, 9, 648, 2592) at 1280x960: path schedule
# A/B (auto / strips / side by side, u16 planes).  Usage: bash tools/gpu_r06_live.sh TAG
set -o pipefail
TAG=${1:?TAG}; cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
for f in 1 2 4 8; do
  for s in 0 1 2; do
    MVSV_PATH_SCHEDULE=$s timeout -k 10 60 python tools/stage_times.py --frames $f --ndisp 64 --bs 9 --p1 648 --p2 2592 >> $O/live_sched.jsonl || exit 1
  done
done
cat $O/live_sched.jsonl
