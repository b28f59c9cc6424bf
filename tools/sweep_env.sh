#!/bin/bash
# Sweep one environment knob over values on the bench workload; prints value + stage times.
# Usage: bash tools/sweep_env.sh VAR "v1 v2 ..." [bench args]
set -o pipefail
VAR=$1; VALS=$2; shift 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
for v in $VALS; do
  env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 "$@" > gpurun_out/sweep/$VAR.$v.json 2> gpurun_out/sweep/$VAR.$v.err || { echo "bench $v failed"; tail -5 gpurun_out/sweep/$VAR.$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sweep/$VAR.$v.json')); print('$VAR=$v', d['value'], d['ms_per_step'], d['stages_ms_per_step'])"
done
