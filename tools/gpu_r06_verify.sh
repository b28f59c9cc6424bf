#!/bin/bash
# Whole GPU suite, then the call sites' stage times.  Usage: bash tools/gpu_r06_verify.sh TAG
set -o pipefail
TAG=${1:?TAG}; cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
for f in 1 2 4 8; do
  timeout -k 10 60 python tools/stage_times.py --frames $f --ndisp 64 --bs 9 --p1 648 --p2 2592 >> $O/stages.jsonl || exit 1
  timeout -k 10 60 python tools/stage_times.py --frames $f --width 640 --height 480 --ndisp 16 --bs 5 --p1 200 --p2 800 >> $O/stages.jsonl || exit 1
done
python - <<PY
import json
for l in open("$O/stages.jsonl"):
    d=json.loads(l); print(d["ndisp"], d["mode"], d["frames"], d["ms_per_call"], d["stages"].get("path_aggregation"), d["stages"].get("final_wta_lr"))
PY
