set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/trace_res3.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_heat_tile_res.py > gpurun_out/tres3.log 2>&1 && \
timeout -k 10 100 python -u benchmarks/trace_tile_res.py --out gpurun_out/trace_res3.jsonl && \
timeout -k 10 100 python -u benchmarks/trace_tile_res.py --fma --out gpurun_out/trace_res3.jsonl && \
timeout -k 10 100 python -u benchmarks/trace_tile_res.py --ns 4 --passes 250 --out gpurun_out/trace_res3.jsonl
