#!/bin/bash
# A/B of environment-selected kernel variants on the bench workload (same box,
# alternating runs).  Usage (on the box): bash tools/ab_env.sh TAG ROUNDS "ENV_A" "ENV_B" [bench args]
# e.g. bash tools/ab_env.sh ab1 3 "" "MVSV_STRIP_WAVES=8"
set -o pipefail
T=$1; N=$2; A=$3; B=$4; shift 4
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$T
for i in $(seq 1 $N); do
  for v in A B; do
    if [ $v = A ]; then E="$A"; else E="$B"; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/$T/bench_${v}_$i.json 2> gpurun_out/$T/bench_${v}_$i.err || { echo "bench $v failed"; tail -20 gpurun_out/$T/bench_${v}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/$T/bench_${v}_$i.json')); print('$v', '$E', d['value'], d['ms_per_step'], {k: round(x, 3) for k, x in d['stages_ms_per_step'].items()})"
  done
done
