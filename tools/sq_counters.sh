#!/bin/bash
# SQ (shader) + GRBM counter passes over a short bench run, one rocprofv3 --pmc
# pass each (at most 8 SQ and 2 GRBM counters per pass), then the per-stage
# summary (tools/sq_summary.py -> sq_summary.json, tied to the kernel sources).
# Usage (on the box, via gpurun): bash tools/sq_counters.sh TAG [program args...]
# (default program: a 2-step bench.py run at the bench workload)
set -o pipefail
TAG=${1:-sq}
shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
if [ $# -gt 0 ]; then CMD=("$@"); else CMD=(python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 --inflight 1 --profile-steps 2 --no-configs); fi
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $P1 -d $O/p1 -o run --output-format csv -- "${CMD[@]}" > $O/p1.log 2>&1 || { echo "p1 failed"; tail -5 $O/p1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc $P2 -d $O/p2 -o run --output-format csv -- "${CMD[@]}" > $O/p2.log 2>&1 || { echo "p2 failed"; tail -5 $O/p2.log; exit 1; }
echo "sq ok"
