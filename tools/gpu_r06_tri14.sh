#!/bin/bash
# D = 256 32-lane strips: 8 (default) vs 14 compute waves (MVSV_TRI32=2).
set -o pipefail
TAG=${1:?TAG}; cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
MVSV_TRI32=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "256 or wide_disparity or accumulator" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2 3; do
  for v in 1 2; do
    for f in 1 2; do
      MVSV_TRI32=$v timeout -k 10 60 python tools/stage_times.py --frames $f | sed "s/^/$v /" >> $O/ab.txt || exit 1
    done
  done
done
python - <<PY
import json
for l in open("$O/ab.txt"):
    v, j = l.split(" ", 1); d = json.loads(j)
    print(v, d["frames"], d["ms_per_call"], d["stages"].get("path_strips"))
PY
