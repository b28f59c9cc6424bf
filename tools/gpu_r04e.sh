#!/bin/bash
# Round 4 session on the cost-residual build: SAD-family rate ubench, new tests,
# full GPU suite, same-box A/B (round-3 library vs this build, lines on / off the
# aux stream), PMC traffic (FETCH_SIZE / WRITE_SIZE passes), bench, kernel-trace
# stats, config-5 frame probe, batches-in-flight sweep.  Usage: bash tools/gpu_r04e.sh TAG
set -o pipefail
TAG=${1:-r04e}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp; cd $R
WL=sgbm_1280x960_d128_8path_batch8
[ -x tools/ubench/sad_rate ] && { timeout -k 10 60 tools/ubench/sad_rate > $O/sad_rate.txt 2>&1 || { echo "sad_rate failed"; exit 1; }; cat $O/sad_rate.txt; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_cost_residual.py tests/test_gpu_strip_width.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/new_tests.log 2>&1 || { echo "new tests failed"; tail -40 $O/new_tests.log; exit 1; }
tail -2 $O/new_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for i in 1 2; do
  for v in r03 new aux0; do
    unset MVSV_LIBRARY MVSV_COST_RESIDUAL MVSV_LINES_AUX MVSV_STRIP_WAVES
    case $v in r03) export MVSV_LIBRARY=$R/variants/r03.so;; res0) export MVSV_COST_RESIDUAL=0;; aux1) export MVSV_LINES_AUX=1;; aux2) export MVSV_LINES_AUX=2;; nar) export MVSV_STRIP_WAVES=8;; nar2) export MVSV_STRIP_WAVES=8 MVSV_LINES_AUX=2;; aux0) export MVSV_LINES_AUX=0;; esac
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
cd $R
timeout -k 10 120 python tools/c5_frame.py > $O/c5_frame.jsonl 2>/dev/null && timeout -k 10 120 python tools/c5_frame.py --frames 8 >> $O/c5_frame.jsonl 2>/dev/null || { echo "config-5 frame probe failed"; exit 1; }
cat $O/c5_frame.jsonl
for n in 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-configs --inflight $n --steps 40 --profile-steps 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('inflight', $n, d['value'], d['ms_per_step'])" >> $O/inflight.txt || { echo "inflight sweep failed"; exit 1; }
done
cat $O/inflight.txt
echo "round ok"
