set -o pipefail
T=${1:-c3}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -m pytest tests -q -m gpu -x -k "sgbm" > gpurun_out/$T/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo "bench failed"; exit 1; }
bash tools/sq_counters.sh $T/sq
