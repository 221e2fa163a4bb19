# fp32 small grids on the tile pass: tile / driver tests, then the small-grid variant sweep at orders 2 and 4
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_heat_tile.py tests/test_drivers.py tests/test_heat_fast.py > gpurun_out/small_tile_tests.log 2>&1 &&
timeout -k 10 400 python3 -u benchmarks/bench_small_variants.py --order 2 4 --n 500 1000 1500 > gpurun_out/small_variants_o24_r4.jsonl 2>/dev/null
