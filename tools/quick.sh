#!/bin/bash
# Quick GPU check: a subset of the parity tests (-k filter) + bench without the CPU baseline.
# Usage (on the box): bash tools/quick.sh TAG "KFILTER" [bench args]
set -o pipefail
T=${1:-quick}; K=${2:-sgbm}; shift 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/$T/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo "bench failed"; tail -20 gpurun_out/$T/bench.err; exit 1; }
python -c "import json,sys; d=json.load(open('gpurun_out/$T/bench.json')); print(d['value'], d['ms_per_step'], d['stages_ms_per_step'])"
