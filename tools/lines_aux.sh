#!/bin/bash
# L->R lines beside / after the strips: auto (-1) vs forced after (0), small and batch launches.
set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "--frames 1 --width 640 --height 480" "--frames 1" "--frames 2" "--frames 8"; do
  for la in -1 0; do
    MVSV_LINES_AUX=$la timeout -k 10 120 python bench.py --no-cpu-baseline $cfg 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); s=d['stages_ms_per_step']; print('$cfg aux=$la', d['median_ms_per_step'], s['path_aggregation'], s['path_strips'], s['path_lines'])" || exit 1
  done
done
