#!/bin/bash
# One parameterised GPU-box session (replaces the round-specific gpu_r04*.sh
# scripts).  Usage (on the box, via gpurun):
#   bash tools/gpu_session.sh TAG [--tests FILES|all] [--ab "name:ENV=V,ENV=V name2:..."]
#        [--rounds N] [--pmc] [--bench] [--trace]
# --tests  pytest -m gpu on the given files (space separated, quoted) or the whole suite
# --ab     same-box A/B of bench.py (one batch in flight, stage times) per variant;
#          a variant's ENV list may set MVSV_LIBRARY=variants/x.so (relative to the repo)
#          or any MVSV_* knob; "new" with no list is the build as is
# --pmc    FETCH_SIZE / WRITE_SIZE passes -> pmc_traffic.json
# --bench  the default bench.py line
# --trace  rocprofv3 --kernel-trace --stats of a short one-in-flight bench
set -o pipefail
TAG=${1:?TAG}
shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
WL=sgbm_1280x960_d128_8path_batch8
TESTS="" AB="" ROUNDS=2 PMC=0 BENCH=0 TRACE=0
while [ $# -gt 0 ]; do
  case $1 in
    --tests) TESTS=$2; shift 2;;
    --ab) AB=$2; shift 2;;
    --rounds) ROUNDS=$2; shift 2;;
    --pmc) PMC=1; shift;;
    --bench) BENCH=1; shift;;
    --trace) TRACE=1; shift;;
    *) echo "unknown option $1"; exit 2;;
  esac
done
if [ -n "$TESTS" ]; then
  [ "$TESTS" = all ] && TESTS=tests
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
if [ -n "$AB" ]; then
  for i in $(seq 1 $ROUNDS); do
    for spec in $AB; do
      name=${spec%%:*}
      envs=""
      [ "$spec" != "$name" ] && envs=${spec#*:}
      (
        for kv in ${envs//,/ }; do
          k=${kv%%=*}; v=${kv#*=}
          [ "$k" = MVSV_LIBRARY ] && v=$R/$v
          export "$k=$v"
        done
        timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 --inflight 1 --profile-steps 10 --no-configs 2>$O/ab_err_$name.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['value'], d['ms_per_step'], {k: round(x, 3) for k, x in d['stages_ms_per_step'].items()})" >> $O/ab.txt
      ) || { echo "A/B variant $name failed"; tail -5 $O/ab_err_$name.txt; exit 1; }
    done
  done
  cat $O/ab.txt
fi
if [ $PMC = 1 ]; then
  cd /tmp
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 --inflight 1 --profile-steps 2 --no-configs > $O/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 --inflight 1 --profile-steps 2 --no-configs > $O/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
  cd $R
  python tools/pmc_traffic.py $(find $O/pmc_fetch -name '*counter_collection.csv' | head -1) $(find $O/pmc_write -name '*counter_collection.csv' | head -1) $WL $O/pmc_traffic.json > $O/pmc_traffic.txt || { echo "pmc summary failed"; exit 1; }
  tail -20 $O/pmc_traffic.txt
fi
if [ $BENCH = 1 ]; then
  timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
  cat $O/bench.json
fi
if [ $TRACE = 1 ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktrace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 10 --warmup 2 --inflight 1 --no-configs > $O/ktrace.log 2>&1 || { echo "kernel trace failed"; exit 1; }
  cd $R
  f=$(find $O/ktrace -name '*kernel_stats.csv' | head -1)
  [ -n "$f" ] && cp $f $O/kernel_stats.csv && head -12 $O/kernel_stats.csv
fi
exit 0
