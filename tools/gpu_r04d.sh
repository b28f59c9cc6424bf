#!/bin/bash
# Round 4, strip-launch session: new tests, full GPU suite, same-box A/B of the
# round-3 library vs this build with the L->R lines on the aux stream (aux2) and
# narrow strips (nar, nar2), PMC traffic, bench, kernel-trace stats.
set -o pipefail
TAG=${1:-r04d}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp; cd $R
WL=sgbm_1280x960_d128_8path_batch8
timeout -k 10 600 python -u -m pytest tests/test_gpu_cost_residual.py tests/test_gpu_strip_width.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/new_tests.log 2>&1 || { echo "new tests failed"; tail -40 $O/new_tests.log; exit 1; }
tail -2 $O/new_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for i in 1 2; do
  for v in r03 new aux2 nar nar2; do
    unset MVSV_LIBRARY MVSV_COST_RESIDUAL MVSV_LINES_AUX MVSV_STRIP_WAVES
    case $v in r03) export MVSV_LIBRARY=$R/variants/r03.so;; res0) export MVSV_COST_RESIDUAL=0;; aux1) export MVSV_LINES_AUX=1;; aux2) export MVSV_LINES_AUX=2;; nar) export MVSV_STRIP_WAVES=8;; nar2) export MVSV_STRIP_WAVES=8 MVSV_LINES_AUX=2;; esac
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 --inflight 1 --profile-steps 10 --no-configs 2>$O/ab_err_$v.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], {k: round(x, 3) for k, x in d['stages_ms_per_step'].items()})" >> $O/ab.txt || { tail -5 $O/ab_err_$v.txt; exit 1; }
  done
done
unset MVSV_LIBRARY MVSV_COST_RESIDUAL MVSV_LINES_AUX MVSV_STRIP_WAVES
cat $O/ab.txt
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 --inflight 1 --profile-steps 2 --no-configs > $O/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 --inflight 1 --profile-steps 2 --no-configs > $O/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
cd $R
python tools/pmc_traffic.py $(find $O/pmc_fetch -name '*counter_collection.csv' | head -1) $(find $O/pmc_write -name '*counter_collection.csv' | head -1) $WL $O/pmc_traffic.json > $O/pmc_traffic.txt || { echo "pmc summary failed"; exit 1; }
cat $O/pmc_traffic.txt | tail -20
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 10 --inflight 1 --profile-steps 10 --no-configs > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
echo "round ok"
