#!/bin/bash
# A/B of library builds on the bench workload (one batch in flight, stage times),
# alternating rounds on one box.  v = default or the name of variants/NAME.so.
# Usage (on the box): bash tools/ab_lib.sh OUTDIR ROUNDS v1 v2 ... [-- bench args]
O=gpurun_out/$1; N=$2; shift 2
V=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done; [ "$1" = "--" ] && shift
mkdir -p $O
for i in $(seq 1 $N); do
  for v in "${V[@]}"; do
    if [ $v = default ]; then unset MVSV_LIBRARY; else export MVSV_LIBRARY=$PWD/variants/$v.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 --inflight 1 --profile-steps 5 "$@" 2>$O/err_$v.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], {k: round(x, 3) for k, x in d['stages_ms_per_step'].items()})" >> $O/out.txt || { tail -5 $O/err_$v.txt; exit 1; }
  done
done
cat $O/out.txt
