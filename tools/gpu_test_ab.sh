#!/bin/bash
# Full GPU test suite on this build, then the library A/B (tools/gpu_ab_libs.sh).
# Usage (on the box): bash tools/gpu_test_ab.sh TAG "new prev"
set -o pipefail
TAG=${1:-tab}; VARS=${2:-"new prev"}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash tools/gpu_ab_libs.sh $TAG "$VARS"
