#!/bin/bash
# Cost-kernel tile height A/B (MVSV_COST_TY, 0 = chosen) for config 5 one / two frames.
set -o pipefail
TAG=${1:?TAG}; cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
for r in 1 2; do
  for ty in 0 8 12 16 24 32 48 64; do
    for f in 1 2; do
      MVSV_COST_TY=$ty timeout -k 10 60 python tools/stage_times.py --frames $f | sed "s/^/$ty /" >> $O/ab.txt || exit 1
    done
  done
done
python - <<PY
import json
for l in open("$O/ab.txt"):
    v, j = l.split(" ", 1); d = json.loads(j)
    print(v, d["frames"], d["ms_per_call"], d["stages"].get("cost_volume"))
PY
