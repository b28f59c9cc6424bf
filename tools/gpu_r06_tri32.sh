#!/bin/bash
# D = 256 narrow strips on 32 lanes per column: the D = 256 parity tests first,
# then the whole GPU suite, then config-5 stage times A/B (MVSV_TRI32 = 1 / 0).
# Usage: bash tools/gpu_r06_tri32.sh TAG
set -o pipefail
TAG=${1:?TAG}; cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "256 or wide_disparity or accumulator" > $O/t256.log 2>&1 || { tail -30 $O/t256.log; exit 1; }
tail -1 $O/t256.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in 1 2; do
for v in 1 0; do
  for f in 1 2 3; do
    MVSV_TRI32=$v timeout -k 10 60 python tools/stage_times.py --frames $f | sed "s/^/$v /" >> $O/ab.txt || exit 1
  done
done
done
python - <<PY
import json
for l in open("$O/ab.txt"):
    v, j = l.split(" ", 1); d = json.loads(j)
    print(v, d["frames"], d["ms_per_call"], d["stages"].get("path_strips"), d["stages"].get("path_lines"), d["stages"].get("final_wta_lr"))
PY
