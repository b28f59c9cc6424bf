#!/bin/bash
# Final kernel: S[best -+ 1] parked by their lanes (default) vs the per-step LDS
# vector (variants/noring.so): GPU tests on the default, then stage times of the
# final16 configurations, alternating.  Usage: bash tools/gpu_r06_ring.sh TAG
set -o pipefail
TAG=${1:?TAG}; cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || bash tools/gpu_census.sh $TAG/census || exit 1
[ -n "$SKIP_TESTS" ] || tail -2 $O/gpu_tests.log
for r in 1 2; do
for v in default noring; do
  if [ $v = default ]; then unset MVSV_LIBRARY; else export MVSV_LIBRARY=$PWD/variants/$v.so; fi
  for f in 1 8; do
    timeout -k 10 60 python tools/stage_times.py --frames $f --width 640 --height 480 --ndisp 16 --bs 5 --p1 200 --p2 800 | sed "s/^/$v /" >> $O/ab.txt || exit 1
    timeout -k 10 60 python tools/stage_times.py --frames $f --ndisp 64 --bs 9 --p1 648 --p2 2592 | sed "s/^/$v /" >> $O/ab.txt || exit 1
    timeout -k 10 60 python tools/stage_times.py --frames $f | sed "s/^/$v /" >> $O/ab.txt || exit 1
  done
done
done
python - <<PY
import json
for l in open("$O/ab.txt"):
    v, j = l.split(" ", 1); d = json.loads(j)
    print(v, d["ndisp"], d["frames"], d["ms_per_call"], d["stages"].get("final_wta_lr"))
PY
