#!/bin/bash
# Speckle local stage with pointer jumping over run starts vs HEAD's per-pixel
# root walks (variants/prevpost.so): speckle / full-size GPU tests on the new
# build, then post-filter stage times alternating.  Usage: bash tools/gpu_r06_speckle2.sh TAG
set -o pipefail
TAG=${1:?TAG}; cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_bitslice.py tests/test_gpu_d16.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
for v in default prevpost; do
  if [ $v = default ]; then unset MVSV_LIBRARY; else export MVSV_LIBRARY=$PWD/variants/$v.so; fi
  timeout -k 10 60 python tools/stage_times.py --frames 8 --ndisp 128 --mind 1 --bs 13 --p1 0 --p2 0 --mode 1 --speckle-window 150 --speckle-range 2 | sed "s/^/$v /" >> $O/ab.txt || exit 1
done
done
python - <<PY
import json
for l in open("$O/ab.txt"):
    v, j = l.split(" ", 1); d = json.loads(j)
    print(v, d["ms_per_call"], d["stages"].get("post_filters"))
PY
