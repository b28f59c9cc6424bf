#!/bin/bash
# Split side-by-side WTA (MVSV_FINAL_SPLIT=1) vs the fused R->L + WTA final
# kernel: the D = 16 / call-site tests and the whole parity file, then the call
# sites' stage times A/B.  Usage: bash tools/gpu_r06_split.sh TAG
set -o pipefail
TAG=${1:?TAG}; cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_d16.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for v in 1 0; do
  for f in 1 2 8; do
    MVSV_FINAL_SPLIT=$v timeout -k 10 60 python tools/stage_times.py --frames $f --width 640 --height 480 --ndisp 16 --bs 5 --p1 200 --p2 800 | sed "s/^/$v /" >> $O/ab.txt || exit 1
  done
  for f in 1 2; do
    MVSV_FINAL_SPLIT=$v timeout -k 10 60 python tools/stage_times.py --frames $f --ndisp 64 --bs 9 --p1 648 --p2 2592 | sed "s/^/$v /" >> $O/ab.txt || exit 1
  done
  for D in 32 128; do
    MVSV_FINAL_SPLIT=$v timeout -k 10 60 python tools/stage_times.py --frames 1 --ndisp $D --bs 9 --p1 648 --p2 2592 | sed "s/^/$v /" >> $O/ab.txt || exit 1
  done
  MVSV_FINAL_SPLIT=$v timeout -k 10 60 python tools/stage_times.py --frames 1 --ndisp 64 --bs 9 --p1 648 --p2 2592 --mode 1 | sed "s/^/$v /" >> $O/ab.txt || exit 1
done
done
python - <<PY
import json
for l in open("$O/ab.txt"):
    v, j = l.split(" ", 1); d = json.loads(j)
    print(v, d["ndisp"], d["mode"], d["frames"], d["ms_per_call"], d["stages"].get("path_aggregation"), d["stages"].get("final_wta_lr"))
PY
