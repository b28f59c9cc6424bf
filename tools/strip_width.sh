set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_strip_width.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sgbm or stream or config" 2>&1 | tail -2 || exit 1
for cfg in "--frames 1 --width 640 --height 480" "--frames 2 --width 640 --height 480" "--frames 1" "--frames 8"; do
  for wv in 0 15; do
    MVSV_STRIP_WAVES=$wv timeout -k 10 120 python bench.py --no-cpu-baseline $cfg 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); s=d['stages_ms_per_step']; print('$cfg wv=$wv', d['median_ms_per_step'], s['path_strips'], s['path_lines'], s['final_wta_lr'])" || exit 1
  done
done
