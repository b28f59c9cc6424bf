#!/bin/bash
# rocprofv3 kernel traces of every config in tools/dispatch_census.py.
# Usage (on the box): bash tools/gpu_census.sh TAG
set -o pipefail
TAG=${1:?TAG}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in c1 c2 c3m0 c3m1 c4 c4m0 c5 live64 capture; do
  timeout -k 10 120 rocprofv3 --kernel-trace -d $O/$c -o run --output-format csv -- python3 $R/tools/dispatch_census.py $c > $O/$c.log 2>&1 || { echo "census $c failed"; tail -5 $O/$c.log; exit 1; }
done
python3 $R/tools/dispatch_census.py --collect $O $O/census.json
