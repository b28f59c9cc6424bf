#!/bin/bash
# Quick GPU check: parity tests + bench (no CPU baseline).  Usage: bash tools/quick.sh TAG [bench args]
set -o pipefail
T=${1:-quick}; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo "bench failed"; tail -20 gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json
