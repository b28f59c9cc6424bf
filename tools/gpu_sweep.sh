#!/bin/bash
# Randomized parity sweep on the box (tools/parity_sweep.py), output under gpurun_out/TAG.
set -o pipefail
TAG=${1:-sweep}; SEED=${2:-5}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 1000 python -u tools/parity_sweep.py --sgbm 300 --bm 150 --large 16 --seed $SEED 2>&1 | tee $O/parity_sweep_seed$SEED.txt | grep -v "^checked" ; rc=${PIPESTATUS[0]}
tail -1 $O/parity_sweep_seed$SEED.txt
exit $rc
