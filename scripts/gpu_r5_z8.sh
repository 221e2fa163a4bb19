set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rx8
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_radix_onesweep.py -m gpu > gpurun_out/rx8/tests.log 2>&1 || exit 1
for u in 4 -4 4 -4; do
  for kind in random small sorted; do
    timeout -k 10 120 python3 benchmarks/bench_sort.py --n 16777216 --algo radix --kind $kind --reps 20 --tune radix_up_unr=$u >> gpurun_out/rx8/bench.jsonl 2>>gpurun_out/rx8/bench.err || exit 1
  done
  timeout -k 10 120 python3 benchmarks/bench_sort.py --n 50331648 --algo radix --reps 20 --tune radix_up_unr=$u >> gpurun_out/rx8/bench.jsonl 2>>gpurun_out/rx8/bench.err || exit 1
done
