set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bitslice.py -m gpu -x -q --timeout 300 --timeout-method thread -k "speckle or config or bench_batch or random" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab_libs.sh r06m/libs "new prev" || exit 1
