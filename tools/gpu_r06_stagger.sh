#!/bin/bash
# Cross-batch stagger A/B (two batches in flight), plus the strip LDS pad that
# lets a cost block share a CU with a strip block.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_env.sh r06r/a 2 "MVSV_STAGGER=0" "MVSV_STAGGER=1" --no-configs --steps 40 --warmup 5 --profile-steps 10 || exit 1
bash tools/ab_env.sh r06r/b 1 "MVSV_STAGGER=1 MVSV_BS_LDSPAD=86016" "MVSV_STAGGER=1 MVSV_BS_GROUPS=2" --no-configs --steps 40 --warmup 5 --profile-steps 10 || exit 1
