#!/bin/bash
# SQ (shader) counter passes over a short bench run, one rocprofv3 --pmc pass each.
# Usage (on the box, via gpurun): bash tools/sq_counters.sh TAG [program args...]
# (default program: a 2-step bench.py run)
set -o pipefail
TAG=${1:-sq}
shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
if [ $# -gt 0 ]; then CMD=("$@"); else CMD=(python $R/bench.py --no-cpu-baseline --steps 2 --warmup 1); fi
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $O/p1 -o run --output-format csv -- "${CMD[@]}" > $O/p1.log 2>&1 || { echo "p1 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $O/p2 -o run --output-format csv -- "${CMD[@]}" > $O/p2.log 2>&1 || { echo "p2 failed"; exit 1; }
echo "sq ok"
