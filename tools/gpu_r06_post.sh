set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r06h; mkdir -p $O
MVSV_GRAPH_DEBUG=1 timeout -k 10 120 python tools/graph_ab.py > $O/graph_ab.json 2> $O/graph_ab.err || { tail $O/graph_ab.err; exit 1; }
cat $O/graph_ab.json; grep "mvsv graph" $O/graph_ab.err | sort | uniq -c
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graphs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "speckle or graph or config or bm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
C4="--frames 8 --width 1280 --height 960 --ndisp 128 --mind 1 --bs 13 --p1 0 --p2 0"
for v in base new; do
  if [ $v = base ]; then export MVSV_LIBRARY=$GRAFT_REPO_ROOT/variants/base.so; else unset MVSV_LIBRARY; fi
  timeout -k 10 60 python tools/stage_times.py $C4 --mode 1 | python -c "import json,sys; d=json.load(sys.stdin); print('$v', d['ms_per_call'], d['stages'])"
done
