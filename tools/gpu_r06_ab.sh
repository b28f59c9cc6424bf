#!/bin/bash
# Round-6 A/B session: strip LDS padding (cost-block co-residence) with two
# batches in flight, then library variants (stage times, one batch in flight).
# Usage (on the box): bash tools/gpu_r06_ab.sh TAG "lib variants" ["ENV_A" "ENV_B"]
set -o pipefail
TAG=${1:?TAG}; LIBS=${2:-new}; EA=${3:-}; EB=${4:-}
cd $GRAFT_REPO_ROOT
if [ -n "$EA$EB" ]; then
  bash tools/ab_env.sh $TAG/env 2 "$EA" "$EB" --no-configs --steps 40 --warmup 5 --profile-steps 10 || exit 1
fi
bash tools/gpu_ab_libs.sh $TAG/libs "$LIBS" || exit 1
