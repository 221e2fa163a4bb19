# fp64 wave-pipelined pass: bitwise tests, then the hw5 / 4000^2 fp64 rows against streamN
set -o pipefail
mkdir -p gpurun_out/p64
timeout -k 10 600 python -u -m pytest tests/test_heat_pipe.py tests/test_dist_gpu.py tests/test_heat.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/p64/pytest.log 2>&1 || { tail -30 gpurun_out/p64/pytest.log; exit 1; }
tail -1 gpurun_out/p64/pytest.log
timeout -k 10 300 python -u benchmarks/bench_heat.py --n 1000 2000 --dtypes fp64 --orders 8 --variants stream3_fma pipe3_fma pipe4_fma --iters 1200 --reps 3 > gpurun_out/p64/hw5.jsonl 2>&1 || { tail gpurun_out/p64/hw5.jsonl; exit 1; }
timeout -k 10 300 python -u benchmarks/bench_heat.py --n 4000 8000 --dtypes fp64 --orders 4 8 --variants stream3_fma pipe3_fma pipe4_fma --iters 120 --reps 5 > gpurun_out/p64/big.jsonl 2>&1 || { tail gpurun_out/p64/big.jsonl; exit 1; }
grep -h '^{' gpurun_out/p64/hw5.jsonl gpurun_out/p64/big.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['n'], d['dtype'], d['order'], d['variant'], d['ms_per_iter'], d['total_ms'])
"
