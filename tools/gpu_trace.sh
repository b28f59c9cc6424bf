#!/bin/bash
# rocprofv3 kernel trace + stats of a short one-in-flight bench (or bench args given).
# Usage (on the box): bash tools/gpu_trace.sh TAG [bench args...]
set -o pipefail
TAG=${1:?TAG}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
ARGS=${@:-"--no-cpu-baseline --no-configs --steps 10 --warmup 3 --inflight 1 --profile-steps 2"}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/bench.py $ARGS > $O/bench.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
python3 - <<PY
import csv, glob
f = glob.glob("$O/kt/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:100]}")
PY
