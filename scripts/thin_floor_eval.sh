# Thin-region chunk floor only for multi-region launches: small standalone grids and one rank's share
set -o pipefail
mkdir -p gpurun_out/tf
timeout -k 10 300 python -u -m pytest tests/test_heat_pipe.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/tf/pytest.log 2>&1 || { tail -30 gpurun_out/tf/pytest.log; exit 1; }
tail -1 gpurun_out/tf/pytest.log
timeout -k 10 300 python -u benchmarks/bench_heat.py --n 1000 2000 --dtypes fp64 --orders 8 --variants stream3_fma pipe4_fma --iters 1200 --reps 3 > gpurun_out/tf/hw5.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u benchmarks/bench_heat.py --n 1000 2000 4000 --dtypes fp32 --orders 8 --variants stream4_fma pipe4_fma --iters 120 --reps 5 > gpurun_out/tf/f32.jsonl 2>&1 || exit 1
grep -h '^{' gpurun_out/tf/hw5.jsonl gpurun_out/tf/f32.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['n'], d['dtype'], d['order'], d['variant'], d['ms_per_iter'], d['total_ms'])
"
timeout -k 10 300 python -u benchmarks/bench_dist_rank.py --kernel pipe --tblock 4 --steps 240 --reps 3 > gpurun_out/tf/rank.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u benchmarks/bench_dist_rank.py --kernel pipe --tblock 4 --steps 240 --reps 3 --method 2 > gpurun_out/tf/rank2.jsonl 2>&1 || exit 1
for f in rank rank2; do grep -h '^{' gpurun_out/tf/$f.jsonl | python3 -c 'import sys,json; print([json.loads(l)["ms_per_step"] for l in sys.stdin])'; done
timeout -k 10 200 python bench.py > gpurun_out/tf/bench.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/tf/bench.log
