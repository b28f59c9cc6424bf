#!/bin/bash
# StereoBM session: the BM GPU tests, then bm_time.py on this build and on the
# round-3 library (variants/r03.so), alternating, then the tile-height sweep.
set -o pipefail
TAG=${1:-bm}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_bm_lanes.py tests -m gpu -k "bm or BM" -x -q --timeout 300 --timeout-method thread > $O/bm_tests.log 2>&1 || { echo "bm tests failed"; tail -40 $O/bm_tests.log; exit 1; }
tail -2 $O/bm_tests.log
for i in 1 2; do
  MVSV_LIBRARY=$R/variants/r03.so timeout -k 10 120 python tools/bm_time.py --auto 2>&1 | sed 's/^auto /r03  /' >> $O/bm_ab.txt || { echo "bm_time r03 failed"; exit 1; }
  timeout -k 10 120 python tools/bm_time.py --auto >> $O/bm_ab.txt 2>&1 || { echo "bm_time failed"; exit 1; }
done
cat $O/bm_ab.txt
timeout -k 10 300 python tools/bm_time.py > $O/bm_time.txt 2>&1 || { echo "bm sweep failed"; exit 1; }
cat $O/bm_time.txt
echo "bm ok"
