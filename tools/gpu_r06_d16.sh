#!/bin/bash
# D = 16 on the 8-lane kernels: parity tests, then the call-site stage times
# and the liveDisparity path-schedule A/B.  Usage: bash tools/gpu_r06_d16.sh TAG
set -o pipefail
TAG=${1:?TAG}; cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_d16.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for f in 1 8; do
  for s in 0 1; do
    MVSV_PATH_SCHEDULE=$s timeout -k 10 60 python tools/stage_times.py --frames $f --width 640 --height 480 --ndisp 16 --bs 5 --p1 200 --p2 800 >> $O/stages.jsonl || exit 1
  done
done
bash tools/gpu_r06_live.sh $TAG
