set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_heat_tile.py > gpurun_out/tile_tests.log 2>&1 &&
timeout -k 10 200 python3 -u benchmarks/bench_hw5.py --n 1000 > gpurun_out/hw5_r4c.jsonl 2>&1 &&
timeout -k 10 200 python3 -u benchmarks/bench_hw5.py --n 1000 --fma >> gpurun_out/hw5_r4c.jsonl 2>&1 &&
timeout -k 10 200 python3 -u benchmarks/trace_tile.py --n 1000 --nts 1 > gpurun_out/tile_trace_r4c.jsonl 2>&1 &&
timeout -k 10 840 python3 -u benchmarks/bench_primitives.py > gpurun_out/prims_r4b.jsonl 2> gpurun_out/prims_r4b.err
