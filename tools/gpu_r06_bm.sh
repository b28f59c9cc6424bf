#!/bin/bash
# StereoBM column-group width (MVSV_BM_COLS 16 / 32): the BM parity tests under
# both widths, then configs 1 / 2 timings alternating.  Usage: bash tools/gpu_r06_bm.sh TAG
set -o pipefail
TAG=${1:?TAG}; cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
for c in 32 16; do
  MVSV_BM_COLS=$c timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "bm" > $O/t$c.log 2>&1 || { tail -30 $O/t$c.log; exit 1; }
  tail -1 $O/t$c.log
done
for r in 1 2 3; do
  for c in 32 16; do
    MVSV_BM_COLS=$c timeout -k 10 120 python tools/bm_time.py --auto | sed "s/^auto /c$c /" >> $O/ab.txt || exit 1
  done
done
cat $O/ab.txt
