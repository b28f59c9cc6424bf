#!/bin/bash
# Copy the summaries of one tools/gpu_round.sh session (gpurun_out/TAG) into
# profiles/r04/TAG (tracked) and refresh the top-level counter summaries that
# bench.py reads (profiles/r04/{sq_summary,pmc_traffic}.json).
# Usage (here, after the gpurun call): bash tools/collect_profiles.sh TAG
set -e
T=$1
R=$(cd "$(dirname "$0")/.." && pwd)
S=$R/gpurun_out/$T
D=$R/profiles/r04/$T
mkdir -p $D
cp $S/bench.json $S/configs.jsonl $S/stream_config5.json $S/valu_rate.txt $S/sq_summary.txt \
   $S/sq_summary.json $S/pmc_traffic.json $D/
[ -f $S/bench_force_gather.json ] && grep '^{' $S/bench_force_gather.json > $D/bench_force_gather.json
[ -f $S/smoke.log ] && cp $S/smoke.log $D/
for f in c5_frame.jsonl tri_trace_c5.txt tri_trace_b8.txt xcc_map.txt; do [ -f $S/$f ] && cp $S/$f $D/; done
[ -f $S/gpu_tests.log ] && grep -E "PASSED|FAILED|ERROR|passed|failed" $S/gpu_tests.log > $D/gpu_tests_summary.txt || true
cp $(find $S/trace -name '*kernel_stats.csv' | head -1) $D/kernel_stats.csv
cp $(find $S/pmc_fetch -name '*counter_collection.csv' | head -1) $D/pmc_fetch_counter_collection.csv
cp $(find $S/pmc_write -name '*counter_collection.csv' | head -1) $D/pmc_write_counter_collection.csv
cp $(find $S/sq/p1 -name '*counter_collection.csv' | head -1) $D/sq_p1_counter_collection.csv
cp $(find $S/sq/p2 -name '*counter_collection.csv' | head -1) $D/sq_p2_counter_collection.csv
cp $(find $S/ubench_pmc -name '*counter_collection.csv' | head -1) $D/ubench_pmc_counter_collection.csv
cp $D/sq_summary.json $D/pmc_traffic.json $R/profiles/r04/
echo "profiles/r04/$T:"; ls $D
