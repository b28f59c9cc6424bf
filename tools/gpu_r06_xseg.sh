#!/bin/bash
# One strip chain's neighbours on one XCD (MVSV_TRI_XSEG=1) vs blockIdx /
# ticket order: D = 256 parity with the knob on, then config-5 one-frame times.
# Usage: bash tools/gpu_r06_xseg.sh TAG
set -o pipefail
TAG=${1:?TAG}; cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
MVSV_TRI_XSEG=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "256 or wide_disparity or accumulator or call_sites" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2 3; do
for v in 1 0; do
  MVSV_TRI_XSEG=$v timeout -k 10 60 python tools/stage_times.py --frames 1 | sed "s/^/$v /" >> $O/ab.txt || exit 1
  MVSV_TRI_XSEG=$v MVSV_TRI32=0 timeout -k 10 60 python tools/stage_times.py --frames 1 | sed "s/^/${v}n /" >> $O/ab.txt || exit 1
done
done
python - <<PY
import json
for l in open("$O/ab.txt"):
    v, j = l.split(" ", 1); d = json.loads(j)
    print(v, d["frames"], d["ms_per_call"], d["stages"].get("path_strips"), d["stages"].get("final_wta_lr"))
PY
