#!/bin/bash
# Round-6 closing session on the final sources: the -m gpu suite, smoke, SQ/GRBM
# counter passes -> profiles/r06/sq_summary.json, PMC passes (FETCH_SIZE and
# WRITE_SIZE in separate runs) -> profiles/r06/pmc_traffic.json, the default bench
# line (reads both), the forced-gather one-rank launch, kernel-trace stats.
# Usage (on the box, via gpurun): bash tools/gpu_r06_final.sh TAG [--no-tests]
set -o pipefail
TAG=${1:-final}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
P=$R/profiles/r06
mkdir -p $O $P
export TMPDIR=/tmp
cd $R
WL=sgbm_1280x960_d128_8path_batch8
if [ "$2" != "--no-tests" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
bash tools/gpu_census.sh $TAG/census || exit 1
fi
bash tools/sq_counters.sh $TAG/sq || exit 1
python tools/sq_summary.py $O/sq $WL $O/sq_summary.json > $O/sq_summary.txt && cp $O/sq_summary.json $P/sq_summary.json || { echo "sq summary failed"; exit 1; }
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 --inflight 1 --profile-steps 2 --no-configs > $O/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 --inflight 1 --profile-steps 2 --no-configs > $O/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
cd $R
python tools/pmc_traffic.py $(find $O/pmc_fetch -name '*counter_collection.csv' | head -1) $(find $O/pmc_write -name '*counter_collection.csv' | head -1) $WL $O/pmc_traffic.json > $O/pmc_traffic.txt && cp $O/pmc_traffic.json $P/pmc_traffic.json || { echo "pmc summary failed"; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json | cut -c1-600
timeout -k 10 600 python bench.py --force-gather --no-cpu-baseline --no-configs > $O/bench_force_gather.json 2> $O/bench_fg.err || { echo "force-gather bench failed"; tail -20 $O/bench_fg.err; exit 1; }
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 10 --inflight 1 --no-configs > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
cd $R
f=$(find $O/trace -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp $f $O/kernel_stats.csv
echo "final ok"
