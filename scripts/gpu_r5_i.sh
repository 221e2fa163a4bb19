set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_heat_tile.py tests/test_heat_tile_res.py > gpurun_out/ttile2.log 2>&1 && \
timeout -k 10 200 python -u benchmarks/bench_hw5.py --n 1000 --reps 7 > gpurun_out/hw5_v2.jsonl 2>&1 && \
timeout -k 10 200 python -u benchmarks/bench_hw5.py --n 1000 --reps 7 --fma >> gpurun_out/hw5_v2.jsonl 2>&1 && \
timeout -k 10 200 python -u benchmarks/trace_tile.py --n 1000 --ns 4 --fma 0 1 --nts 1 > gpurun_out/trace_tile_v2.jsonl 2>&1
