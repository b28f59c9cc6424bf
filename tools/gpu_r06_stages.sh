set -o pipefail
O=gpurun_out/r06b; mkdir -p $O
C3="--frames 1 --width 640 --height 480 --ndisp 128 --mind 1 --bs 13 --p1 0 --p2 0"
C4="--frames 8 --width 1280 --height 960 --ndisp 128 --mind 1 --bs 13 --p1 0 --p2 0"
for m in 0 1; do timeout -k 10 60 python tools/stage_times.py $C3 --mode $m --steps 50 >> $O/stages.jsonl || exit 1; done
for g in 1 2 4; do MVSV_BS_GROUPS=$g timeout -k 10 60 python tools/stage_times.py $C4 --mode 0 >> $O/stages.jsonl || exit 1; done
MVSV_BS_SERIAL=1 timeout -k 10 60 python tools/stage_times.py $C4 --mode 0 >> $O/stages.jsonl || exit 1
timeout -k 10 60 python tools/stage_times.py $C4 --mode 1 >> $O/stages.jsonl || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/stage_times.py $C3 --mode 0 --steps 20 > /dev/null 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt4 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/stage_times.py $C4 --mode 0 --steps 10 > /dev/null 2>&1 || exit 1
cat $GRAFT_REPO_ROOT/$O/stages.jsonl
