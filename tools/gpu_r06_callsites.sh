#!/bin/bash
# Stage times and a kernel trace of the reference's other call sites:
# captureDisparity create(0, 16, 5, 200, 800) at 640x480 and liveDisparity's
# default create(0, 64, 9, 648, 2592) at 1280x960.  Usage: bash tools/gpu_r06_callsites.sh TAG
set -o pipefail
TAG=${1:?TAG}; cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
for f in 1 8; do
  timeout -k 10 60 python tools/stage_times.py --frames $f --width 640 --height 480 --ndisp 16 --bs 5 --p1 200 --p2 800 >> $O/stages.jsonl || exit 1
  timeout -k 10 60 python tools/stage_times.py --frames $f --ndisp 64 --bs 9 --p1 648 --p2 2592 >> $O/stages.jsonl || exit 1
done
cat $O/stages.jsonl
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/cap -o run -- python3 tools/stage_times.py --frames 1 --width 640 --height 480 --ndisp 16 --bs 5 --p1 200 --p2 800 --steps 5 > $O/cap.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/live -o run -- python3 tools/stage_times.py --frames 1 --ndisp 64 --bs 9 --p1 648 --p2 2592 --steps 5 > $O/live.log 2>&1 || exit 1
find $O -name '*kernel_stats.csv' | while read f; do echo "== $f"; cut -d, -f1-4 "$f" | head -20; done
