#!/bin/bash
# One GPU-box session: tests, smoke, the VALU issue-rate ubench (+ its counter
# calibration), SQ/GRBM counter passes -> sq_summary.json, PMC passes
# (FETCH_SIZE and WRITE_SIZE in separate runs) -> pmc_traffic.json, the bench
# (reads both), the forced-gather one-rank launch, per-config table, config-5
# stream bench, config-5 frame probe + strip traces, dispatch-placement probe,
# kernel-trace stats.
# Usage (on the box, via gpurun): bash tools/gpu_round.sh TAG [--no-tests]
set -o pipefail
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
P=$R/profiles/r04
mkdir -p $O $P
export TMPDIR=/tmp
cd $R
WL=sgbm_1280x960_d128_8path_batch8
if [ "$2" != "--no-tests" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
fi
timeout -k 10 300 ./tools/ubench/valu_rate > $O/valu_rate.txt 2>&1 || { echo "ubench failed"; exit 1; }
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/ubench_pmc -o run --output-format csv -- $R/tools/ubench/valu_rate 4 > $O/ubench_pmc.log 2>&1 || { echo "ubench pmc failed"; exit 1; }
cd $R
bash tools/sq_counters.sh $TAG/sq || exit 1
python tools/sq_summary.py $O/sq $WL $O/sq_summary.json > $O/sq_summary.txt && cp $O/sq_summary.json $P/sq_summary.json || { echo "sq summary failed"; exit 1; }
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 --inflight 1 --profile-steps 2 --no-configs > $O/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 --inflight 1 --profile-steps 2 --no-configs > $O/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
cd $R
python tools/pmc_traffic.py $(find $O/pmc_fetch -name '*counter_collection.csv' | head -1) $(find $O/pmc_write -name '*counter_collection.csv' | head -1) $WL $O/pmc_traffic.json > /dev/null && cp $O/pmc_traffic.json $P/pmc_traffic.json || { echo "pmc summary failed"; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 python bench.py --force-gather --no-cpu-baseline > $O/bench_force_gather.json 2> $O/bench_fg.err || { echo "force-gather bench failed"; tail -20 $O/bench_fg.err; exit 1; }
timeout -k 10 600 python tools/bench_configs.py > $O/configs.jsonl 2> $O/configs.err || { echo "config table failed"; tail -20 $O/configs.err; exit 1; }
timeout -k 10 300 python tools/bench_stream.py > $O/stream_config5.json 2> $O/stream.err || { echo "stream bench failed"; exit 1; }
timeout -k 10 120 python tools/c5_frame.py > $O/c5_frame.jsonl 2>/dev/null && timeout -k 10 120 python tools/c5_frame.py --frames 2 >> $O/c5_frame.jsonl 2>/dev/null || { echo "config-5 frame probe failed"; exit 1; }
MVSV_TRI_TRACE=$O/tri_trace_c5.bin timeout -k 10 120 python tools/c5_frame.py > /dev/null 2>&1 && python tools/tri_trace.py $O/tri_trace_c5.bin > $O/tri_trace_c5.txt || { echo "c5 strip trace failed"; exit 1; }
MVSV_TRI_TRACE=$O/tri_trace_b8.bin timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1 --warmup 0 --inflight 1 --profile-steps 0 --no-configs > /dev/null 2>&1 && python tools/tri_trace.py $O/tri_trace_b8.bin > $O/tri_trace_b8.txt || { echo "batch strip trace failed"; exit 1; }
timeout -k 10 60 ./tools/ubench/xcc_map 576 20 > $O/xcc_map.txt 2>&1 || { echo "xcc probe failed"; exit 1; }
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 10 --inflight 1 --no-configs > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
echo "round ok"
