#!/bin/bash
# A/B of in-tree library variants (variants/*.so) on the default bench workload.
# Usage (on the box, via gpurun): bash tools/ab.sh TAG [extra bench args]
set -o pipefail
T=${1:-ab}; shift
mkdir -p gpurun_out/$T
for v in variants/*.so; do
  n=$(basename $v .so)
  MVSV_LIBRARY=$PWD/$v timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/$T/$n.json 2> gpurun_out/$T/$n.err || { echo "bench $n failed"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$T/$n.json')); print('$n', d['value'], d['ms_per_step'], d.get('stages_ms_per_step'))"
done
