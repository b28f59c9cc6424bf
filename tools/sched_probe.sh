#!/bin/bash
# Path schedule A/B: auto vs strips forced, small and batch launches (bench.py workload).
set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "--frames 1 --width 640 --height 480" "--frames 2 --width 640 --height 480" "--frames 4 --width 640 --height 480" "--frames 1" "--frames 2"; do
  for ps in 0 1; do
    MVSV_PATH_SCHEDULE=$ps timeout -k 10 120 python bench.py --no-cpu-baseline $cfg 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); s=d['stages_ms_per_step']; print('$cfg sched=$ps', d['median_ms_per_step'], s.get('path_aggregation'), s.get('final_wta_lr'))" || exit 1
  done
done
