#!/bin/bash
# Round-6 quick GPU check: given test files (or "all"), then the config table.
# Usage (on the box): bash tools/gpu_r06_quick.sh TAG "tests/x.py tests/y.py"|all [configs]
set -o pipefail
TAG=${1:?TAG}; T=${2:-all}; CF=${3:-}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
[ "$T" = all ] && T=tests
timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
if [ -n "$CF" ]; then
  timeout -k 10 300 python tools/bench_configs.py --steps 30 --warmup 5 > $O/configs.jsonl 2> $O/configs.err || { tail -5 $O/configs.err; exit 1; }
  python -c "
import json
for l in open('$O/configs.jsonl'): d=json.loads(l); print(d['config'], d['frames_per_step'], d['median_ms_per_step'], d['mpix_s'])"
fi
