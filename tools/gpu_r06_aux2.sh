#!/bin/bash
# After the lines-beside-strips rule for D <= 64 batches: GPU suite, a parity
# sweep with full-size batches, liveDisparity default stage times.
set -o pipefail
TAG=${1:?TAG}; cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 900 python -u tools/parity_sweep.py --sgbm 200 --bm 50 --large 60 --bits 50 --bits-large 8 --seed 79 > $O/parity_sweep_seed79.txt 2>&1 || { tail -5 $O/parity_sweep_seed79.txt; exit 1; }
tail -1 $O/parity_sweep_seed79.txt
for f in 1 2 4 8; do
  timeout -k 10 60 python tools/stage_times.py --frames $f --ndisp 64 --bs 9 --p1 648 --p2 2592 >> $O/stages.jsonl || exit 1
done
python - <<PY
import json
for l in open("$O/stages.jsonl"):
    d=json.loads(l); print(d["ndisp"], d["frames"], d["ms_per_call"], d["stages"].get("path_aggregation"))
PY
