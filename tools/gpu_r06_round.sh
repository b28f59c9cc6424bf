#!/bin/bash
# Round-6 GPU session: the -m gpu suite, then optional A/B steps.
# Usage (on the box): bash tools/gpu_r06_round.sh TAG [tests|notests] ["lib variants"] ["ENV_A" "ENV_B"]
set -o pipefail
TAG=${1:?TAG}; T=${2:-tests}; LIBS=${3:-}; EA=${4:-}; EB=${5:-}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
if [ "$T" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
if [ -n "$EA$EB" ]; then
  bash tools/ab_env.sh $TAG/env 2 "$EA" "$EB" --no-configs --steps 40 --warmup 5 --profile-steps 10 || exit 1
fi
if [ -n "$LIBS" ]; then
  bash tools/gpu_ab_libs.sh $TAG/libs "$LIBS" || exit 1
fi
