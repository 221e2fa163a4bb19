# tapered chunking (CME_PIPE_TAPER) on the GPU box: bitwise tests, then the
# flagship bench with taper off / auto alternating, a bench_ic sweep, and
# one rank's N = 1 / 2 shares -> gpurun_out/taper_*.jsonl
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_heat_pipe.py -m gpu -x -q --timeout 200 --timeout-method thread -k "taper or fast_arms or wide" > gpurun_out/taper_tests.log 2>&1 || exit 1
for t in 0 -1 0 -1; do
  CME_PIPE_TAPER=$t timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/taper_bench.jsonl 2>&1 || exit 2
done
timeout -k 10 400 python benchmarks/bench_ic.py --variants pipe4_fast --windows 4 --steps 60 --tune pipe_taper=0/-1/11/33 > gpurun_out/taper_ic.jsonl 2>&1 || exit 3
for t in 0 -1; do
  timeout -k 10 200 python benchmarks/bench_dist_rank.py --kernel pipe --tblock 4 --arith fast --world 1 2 --tune pipe_taper=$t >> gpurun_out/taper_rank.jsonl 2>&1 || exit 4
done
