#!/bin/bash
# One library variant against the in-tree build on one box: the full GPU test
# suite on the variant (MVSV_LIBRARY) and a parity sweep, then alternating bench
# stage times (tools/gpu_ab_libs.sh) and config-5 frame times (tools/c5_frame.py).
# The C++ tests (tests/test_cpp_*.py) link libmvsv by name: they run on the in-tree build only.
# Usage (on the box): bash tools/gpu_variant_ab.sh TAG VARIANT
set -o pipefail
TAG=${1:-vab}; V=${2:?variant name}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp; cd $R
[ -f variants/$V.so ] || { echo "no variants/$V.so"; exit 1; }
MVSV_LIBRARY=$R/variants/$V.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --ignore-glob 'tests/test_cpp_*.py' > $O/gpu_tests_$V.log 2>&1 || { echo "tests failed on $V"; tail -40 $O/gpu_tests_$V.log; exit 1; }
tail -2 $O/gpu_tests_$V.log
MVSV_LIBRARY=$R/variants/$V.so timeout -k 10 600 python -u tools/parity_sweep.py --sgbm 300 --bm 150 --large 16 --seed 8 > $O/parity_sweep_$V.txt 2>&1 || { echo "sweep failed on $V"; grep -v "^checked" $O/parity_sweep_$V.txt | tail -20; exit 1; }
tail -1 $O/parity_sweep_$V.txt
bash tools/gpu_ab_libs.sh $TAG "new $V" || exit 1
for i in 1 2; do
  for v in new $V; do
    unset MVSV_LIBRARY
    [ $v != new ] && export MVSV_LIBRARY=$R/variants/$v.so
    { timeout -k 10 120 python tools/c5_frame.py && timeout -k 10 120 python tools/c5_frame.py --frames 8; } 2>/dev/null | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$v', d['frames'], d['ms_per_call'], {k: round(x, 3) for k, x in d['stages_ms'].items()})" >> $O/c5_ab.txt || { echo "c5 $v failed"; exit 1; }
  done
done
unset MVSV_LIBRARY
cat $O/c5_ab.txt
