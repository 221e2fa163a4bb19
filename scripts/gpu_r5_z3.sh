set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ms3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_radix_onesweep.py -m gpu -k "merge" > gpurun_out/ms3/tests.log 2>&1 || exit 1
for cfg in "merge_part=0" "merge_part=64" "merge_part=32" "merge_part=16" "merge_part=8" "merge_part=64 merge_tile=8192" "merge_part=16 merge_tile=8192" "merge_part=8 merge_tile=8192"; do
  timeout -k 10 120 python3 benchmarks/bench_sort.py --n 16777216 50331648 --dtype int32 --algo merge --reps 10 --tune $cfg >> gpurun_out/ms3/bench.jsonl 2>>gpurun_out/ms3/bench.err || exit 1
done
