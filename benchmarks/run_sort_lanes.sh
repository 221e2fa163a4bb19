# radix downsweep arms (tuning knob radix_ds) on the GPU box: tests, then
# bench_sort.py per arm and key kind -> gpurun_out/sort_lanes.jsonl
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_radix_onesweep.py tests/test_library.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sort_tests.log 2>&1 || exit 1
for arm in ${ARMS:-2 10 14}; do
  for kind in ${KINDS:-random small}; do
    timeout -k 10 120 python benchmarks/bench_sort.py --n 16777216 50331648 --algo radix --kind $kind --tune radix_ds=$arm $EXTRA >> gpurun_out/sort_lanes.jsonl 2>&1 || exit 2
  done
  timeout -k 10 120 python benchmarks/bench_sort.py --n 16777216 --dtype int32 --values --algo radix --tune radix_ds=$arm $EXTRA >> gpurun_out/sort_lanes.jsonl 2>&1 || exit 3
done
for mb in ${MAXBLOCKS:-}; do
  timeout -k 10 120 python benchmarks/bench_sort.py --n 16777216 50331648 --algo radix --tune radix_ds=14 radix_max_blocks=$mb >> gpurun_out/sort_lanes.jsonl 2>&1 || exit 4
done
