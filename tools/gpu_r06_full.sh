#!/bin/bash
# Round-6 session: the whole -m gpu suite, the default bench line, SQ counters.
# Usage (on the box): bash tools/gpu_r06_full.sh TAG [sq]
set -o pipefail
TAG=${1:?TAG}; SQ=${2:-}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print(d['value'], d['ms_per_step'], d.get('single_batch_ms'), json.dumps(d.get('roofline'))[:300])"
if [ -n "$SQ" ]; then
  bash tools/sq_counters.sh $TAG/sq || exit 1
  python tools/sq_summary.py $O/sq > $O/sq_summary.txt 2>&1 || { tail -5 $O/sq_summary.txt; exit 1; }
  grep -i "speckle\|cost2\|strip\|rlwta\|lines4\|median" $O/sq_summary.txt | cut -c1-200
fi
