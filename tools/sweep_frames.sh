#!/bin/bash
# Per-stage times per frame vs frames per launch: a stage whose per-frame time
# falls as the batch grows is latency-bound at the smaller batch.
# Usage (on the box, via gpurun): bash tools/sweep_frames.sh "2 4 8 16"
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/frames
for f in $1; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --frames $f > gpurun_out/frames/f$f.json 2> gpurun_out/frames/f$f.err || { echo "bench $f failed"; tail -5 gpurun_out/frames/f$f.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/frames/f$f.json')); print('frames=$f', d['value'], d['ms_per_step'], {k: round(v/$f, 4) for k, v in d['stages_ms_per_step'].items()})"
done
