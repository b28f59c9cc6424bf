#!/bin/bash
# Post-filter session: speckle / median GPU tests, then the bench's stage times
# for this build and the previous commit's library (variants/prev.so), alternating.
set -o pipefail
TAG=${1:-post}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -k "speckle or median or post or config5 or stream" -x -q --timeout 300 --timeout-method thread > $O/post_tests.log 2>&1 || { echo "post tests failed"; tail -40 $O/post_tests.log; exit 1; }
tail -2 $O/post_tests.log
for i in 1 2; do
  for v in prev new; do
    unset MVSV_LIBRARY
    [ $v = prev ] && export MVSV_LIBRARY=$R/variants/prev.so
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 --inflight 1 --profile-steps 10 --no-configs 2>$O/ab_err_$v.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], {k: round(x, 3) for k, x in d['stages_ms_per_step'].items()})" >> $O/ab.txt || { tail -5 $O/ab_err_$v.txt; exit 1; }
  done
done
unset MVSV_LIBRARY
cat $O/ab.txt
echo "post ok"
