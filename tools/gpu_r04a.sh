set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04a; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 10 --inflight 1 > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
echo "round ok"
