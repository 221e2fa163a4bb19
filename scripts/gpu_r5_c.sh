set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_heat_flow.py > gpurun_out/t2.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_heat_pipe.py tests/test_heat_fast.py tests/test_heat_tile.py tests/test_heat.py tests/test_spmv.py tests/test_bench_contract.py > gpurun_out/t3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-primitives > gpurun_out/b2.json 2> gpurun_out/b2.err && \
CME_HEAT_FLOW=0 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-primitives > gpurun_out/b2off.json 2> gpurun_out/b2off.err && \
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 --no-primitives > gpurun_out/b3.json 2> gpurun_out/b3.err && \
CME_HEAT_FLOW=0 timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 --no-primitives > gpurun_out/b3off.json 2> gpurun_out/b3off.err
