#!/bin/bash
# Round-6 randomized parity sweep (both SGBM modes in the bit-sliced regime).
set -o pipefail
SEED=${1:-61}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06sweep2; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 900 python -u tools/parity_sweep.py --sgbm 150 --bm 100 --large 8 --bits 300 --bits-large 24 --seed $SEED > $O/parity_sweep_seed$SEED.txt 2>&1; rc=$?
grep -v "^checked" $O/parity_sweep_seed$SEED.txt | tail -5
exit $rc
