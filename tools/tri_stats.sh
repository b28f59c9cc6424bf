#!/bin/bash
# Strip-kernel timeline statistics (MVSV_TRI_STATS) over a short bench run.
set -o pipefail
cd $GRAFT_REPO_ROOT
MVSV_TRI_STATS=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/tri_stats.json 2> gpurun_out/tri_stats.err
