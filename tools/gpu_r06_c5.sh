#!/bin/bash
# Config-5 frame timings (1, 2, 8 frames) and the default bench line with the
# config table (incl. the config-5 stream).  Usage: bash tools/gpu_r06_c5.sh TAG
set -o pipefail
TAG=${1:?TAG}; cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
for f in 1 2 3 8; do timeout -k 10 60 python tools/stage_times.py --frames $f >> $O/c5_stages.jsonl || exit 1; done
cat $O/c5_stages.jsonl
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - <<PY
import json
d=json.load(open("$O/bench.json"))
print(d["value"], d["ms_per_step"], d.get("single_batch_ms"))
for k,v in d.get("configs",{}).items(): print(k, {kk: v.get(kk) for kk in ("median_ms","mpix_s","stream_fps","parity_frame0")})
PY
