#!/bin/bash
# Single-frame strip-width sweep over variants/n*.so (narrow strip widths).
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in variants/n*.so; do
  for cfg in "--frames 1 --width 640 --height 480" "--frames 1" "--frames 4"; do
    MVSV_LIBRARY=$PWD/$v timeout -k 10 120 python bench.py --no-cpu-baseline $cfg 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); s=d['stages_ms_per_step']; print('$v $cfg', d['median_ms_per_step'], s['path_strips'])" || exit 1
  done
done
