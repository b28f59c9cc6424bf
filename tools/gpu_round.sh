#!/bin/bash
# One GPU-box session: tests, smoke, bench, config-5 stream bench, kernel-trace stats,
# PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs).
# Usage (on the box, via gpurun): bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; exit 1; }
cat $O/bench.json
timeout -k 10 300 python tools/bench_stream.py > $O/stream_config5.json 2> $O/stream.err || { echo "stream bench failed"; exit 1; }
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python $R/bench.py --no-cpu-baseline --steps 10 > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
echo "round ok"
