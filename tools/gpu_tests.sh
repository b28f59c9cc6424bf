#!/bin/bash
# GPU parity tests only (+ optional -k filter).  Usage (on the box): bash tools/gpu_tests.sh TAG [pytest args]
set -o pipefail
T=${1:-tests}; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/$T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/$T/tests.log | head -30; tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -3 gpurun_out/$T/tests.log
