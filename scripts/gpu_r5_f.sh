set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_heat_tile_res.py > gpurun_out/tres.log 2>&1 && \
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_heat_tile.py > gpurun_out/ttile.log 2>&1 && \
timeout -k 10 200 python -u benchmarks/bench_hw5.py --n 1000 --reps 5 > gpurun_out/hw5_res.jsonl 2>&1 && \
timeout -k 10 200 python -u benchmarks/bench_hw5.py --n 1000 --reps 5 --fma >> gpurun_out/hw5_res.jsonl 2>&1 && \
timeout -k 10 200 python -u benchmarks/bench_hw5.py --n 1000 --reps 5 --tune tile_res=0 >> gpurun_out/hw5_res.jsonl 2>&1 && \
timeout -k 10 200 python -u benchmarks/bench_hw5.py --n 1000 --reps 5 --tune tile_res_ns=4 >> gpurun_out/hw5_res.jsonl 2>&1 && \
timeout -k 10 100 python -u benchmarks/trace_tile_res.py --out gpurun_out/trace_res.jsonl && \
timeout -k 10 100 python -u benchmarks/trace_tile_res.py --fma --out gpurun_out/trace_res.jsonl && \
timeout -k 10 100 python -u benchmarks/trace_tile_res.py --ns 4 --passes 250 --out gpurun_out/trace_res.jsonl
