#!/bin/bash
# Config-5 A/B (liveDisparity parameters, 1280x960, D 256): one frame and 8
# frames per launch (tools/c5_frame.py), this build vs variants/prev.so,
# after the GPU tests that cover config 5 and the u16-plane schedules.
set -o pipefail
TAG=${1:-c5ab}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for i in 1 2; do
  for v in new prev; do
    unset MVSV_LIBRARY
    [ $v = prev ] && export MVSV_LIBRARY=$R/variants/prev.so
    { timeout -k 10 120 python tools/c5_frame.py && timeout -k 10 120 python tools/c5_frame.py --frames 8; } 2>/dev/null | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$v', d['frames'], d['ms_per_call'], {k: round(x, 3) for k, x in d['stages_ms'].items()})" >> $O/c5_ab.txt || { echo "c5 $v failed"; exit 1; }
  done
done
unset MVSV_LIBRARY
cat $O/c5_ab.txt
bash tools/gpu_ab_libs.sh $TAG "new prev"
