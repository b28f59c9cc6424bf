set -o pipefail
T=${1:-c6}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/$T/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo "bench failed"; exit 1; }
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$T/trace -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/$T/trace.log 2>&1 || { echo "trace failed"; exit 1; }
echo ok
