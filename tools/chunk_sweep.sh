set -u
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/chunk1; mkdir -p $OUT; cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_frontier.py tests/test_gpu_arena.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for c in 64 32 128 16; do
  BK_CHUNK=$c timeout -k 10 120 python3 bench.py --no-cpu-baseline > $OUT/bench_c$c.jsonl 2>$OUT/bench_c$c.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_c$c.jsonl')); print('chunk $c', round(d['value']/1e6,2), 'M/s', round(d['roofline']['kernel_ms'],3),'ms')"
done
BK_CHUNK=64 timeout -k 10 120 python3 bench.py --no-cpu-baseline --rollouts 4096 > $OUT/bench_1m.jsonl 2>&1 || exit 1
python3 -c "import json; d=json.load(open('$OUT/bench_1m.jsonl')); print('1M chunk64', round(d['value']/1e6,2))"
