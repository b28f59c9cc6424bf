#!/bin/bash
# Config-5 stream: sustained fps vs frames per launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/stream
for db in "3 1" "4 2" "16 8" "24 12" "32 16"; do
  set -- $db
  timeout -k 10 200 python tools/bench_stream.py --frames 240 --depth $1 --batch $2 > gpurun_out/stream/d$1b$2.json 2> gpurun_out/stream/d$1b$2.err || { echo "stream $db failed"; tail -5 gpurun_out/stream/d$1b$2.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/stream/d$1b$2.json')); print('depth $1 batch $2', d['stream_fps'], d['stream_ms_per_frame'], d['obstacle_tiles_found'])"
done
