# A/B of library variants on config-5 frames and the bench: bash tools/ab_lag.sh OUTDIR v1 v2 ...
# (v = default or the name of variants/NAME.so)
O=gpurun_out/$1; shift
mkdir -p $O
for v in "$@"; do
  if [ $v = default ]; then unset MVSV_LIBRARY; else export MVSV_LIBRARY=$PWD/variants/$v.so; fi
  echo "== $v" >> $O/out.txt
  timeout -k 10 100 python tools/c5_frame.py >> $O/out.txt 2>/dev/null || exit 1
  timeout -k 10 100 python tools/c5_frame.py --frames 2 >> $O/out.txt 2>/dev/null || exit 1
  MVSV_TRI_STATS=1 timeout -k 10 100 python tools/c5_frame.py 2>&1 >/dev/null | grep "span" >> $O/out.txt || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 --inflight 1 --profile-steps 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'))" >> $O/out.txt || exit 1
done
