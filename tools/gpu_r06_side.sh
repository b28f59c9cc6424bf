set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r06e; mkdir -p $O
C4="--frames 8 --width 1280 --height 960 --ndisp 128 --mind 1 --bs 13 --p1 0 --p2 0"
C3="--frames 8 --width 640 --height 480 --ndisp 128 --mind 1 --bs 13 --p1 0 --p2 0"
for m in 0 1; do
 for s in 1 2; do
  MVSV_PATH_SCHEDULE=$s timeout -k 10 60 python tools/stage_times.py $C4 --mode $m >> $O/side.jsonl || exit 1
  MVSV_PATH_SCHEDULE=$s timeout -k 10 60 python tools/stage_times.py $C3 --mode $m >> $O/side.jsonl || exit 1
 done
done
cat $O/side.jsonl
