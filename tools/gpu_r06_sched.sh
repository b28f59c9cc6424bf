#!/bin/bash
# Scheduling A/Bs with two batches in flight (round 6): the L->R lines beside /
# after the 3-group strips, 2 vs 3 batches in flight, 5-path strip groups.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r06p; mkdir -p $O
bash tools/ab_env.sh r06p/serial 2 "MVSV_BS_SERIAL=0" "MVSV_BS_SERIAL=1" --no-configs --steps 40 --warmup 5 --profile-steps 10 || exit 1
for inf in 2 3; do timeout -k 10 200 python bench.py --no-cpu-baseline --no-configs --steps 40 --warmup 5 --profile-steps 10 --inflight $inf > $O/inf$inf.json 2>/dev/null || exit 1; python -c "import json; d=json.load(open('$O/inf$inf.json')); print('inflight $inf', d['value'], d['ms_per_step'])"; done
C4="--frames 8 --width 1280 --height 960 --ndisp 128 --mind 1 --bs 13 --p1 0 --p2 0"
for g in 2 3; do MVSV_BS_GROUPS=$g timeout -k 10 60 python tools/stage_times.py $C4 --mode 0 | python -c "import json,sys; d=json.load(sys.stdin); print('mode0 groups $g', d['ms_per_call'], d['stages'])" || exit 1; done
for g in 2 3; do for inf in 2; do MVSV_BS_GROUPS=$g timeout -k 10 200 python bench.py --mode 0 --no-cpu-baseline --no-configs --steps 40 --warmup 5 --profile-steps 10 > $O/m0g$g.json 2>/dev/null || exit 1; python -c "import json; d=json.load(open('$O/m0g$g.json')); print('bench mode 0 groups $g', d['value'], d['ms_per_step'])"; done; done
