set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ms4
for cfg in "merge_part=4" "merge_part=8" "merge_part=4" "merge_part=8" "merge_part=0"; do
  timeout -k 10 120 python3 benchmarks/bench_sort.py --n 1048576 16777216 50331648 --dtype int32 --algo merge --reps 10 --tune $cfg >> gpurun_out/ms4/bench.jsonl 2>>gpurun_out/ms4/bench.err || exit 1
  timeout -k 10 120 python3 benchmarks/bench_sort.py --n 16777216 50331648 --dtype int32 --algo merge --values --reps 10 --tune $cfg >> gpurun_out/ms4/bench.jsonl 2>>gpurun_out/ms4/bench.err || exit 1
done
timeout -k 10 120 python3 benchmarks/bench_sort.py --n 1048576 16777216 50331648 --dtype int32 --algo torch --reps 10 >> gpurun_out/ms4/bench.jsonl 2>>gpurun_out/ms4/bench.err
