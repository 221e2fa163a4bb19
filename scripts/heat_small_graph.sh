# Small-grid heat rows (BASELINE #12-14, #17-18) eager vs hipGraph replay
set -o pipefail
mkdir -p gpurun_out/hsg
timeout -k 10 300 python -u -m pytest tests/test_graphs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hsg/pytest.log 2>&1 || { tail -30 gpurun_out/hsg/pytest.log; exit 1; }
tail -1 gpurun_out/hsg/pytest.log
timeout -k 10 300 python -u benchmarks/bench_heat.py --n 1000 2000 --dtypes fp64 --orders 8 --variants stream stream2_fma stream3_fma --iters 1000 --reps 3 --graph > gpurun_out/hsg/hw5.jsonl 2>&1 || { tail gpurun_out/hsg/hw5.jsonl; exit 1; }
timeout -k 10 300 python -u benchmarks/bench_heat.py --n 4000 --dtypes fp32 --orders 2 4 8 --variants shared stream stream4_fma pipe3_fma pipe4_fma --iters 120 --reps 5 --graph > gpurun_out/hsg/h4000.jsonl 2>&1 || { tail gpurun_out/hsg/h4000.jsonl; exit 1; }
timeout -k 10 300 python -u benchmarks/bench_heat.py --n 4000 --dtypes fp64 --orders 4 --variants global shared stream2_fma stream3_fma --iters 120 --reps 5 --graph > gpurun_out/hsg/h4000d.jsonl 2>&1 || { tail gpurun_out/hsg/h4000d.jsonl; exit 1; }
grep -h '^{' gpurun_out/hsg/*.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['n'], d['dtype'], d['order'], d['variant'], d['ms_per_iter'], d.get('graph_ms_per_iter'), d['total_ms'], d.get('graph_total_ms'))
"
