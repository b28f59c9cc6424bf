#!/bin/bash
# Same-box A/B of library variants (variants/NAME.so; "new" = the in-tree build):
# bench stage times, one batch in flight, two alternating rounds.
# Usage (on the box): bash tools/gpu_ab_libs.sh TAG "new prev"
set -o pipefail
TAG=${1:-ab}; VARS=${2:-new}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp; cd $R
for i in 1 2; do
  for v in $VARS; do
    unset MVSV_LIBRARY
    [ $v != new ] && export MVSV_LIBRARY=$R/variants/$v.so
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 --inflight 1 --profile-steps 10 --no-configs 2>$O/ab_err_$v.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], {k: round(x, 3) for k, x in d['stages_ms_per_step'].items()})" >> $O/ab.txt || { tail -5 $O/ab_err_$v.txt; exit 1; }
  done
done
unset MVSV_LIBRARY
cat $O/ab.txt
