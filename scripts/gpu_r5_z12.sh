set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ms12
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_radix_onesweep.py tests/test_sort_text.py tests/test_algorithms.py -m gpu > gpurun_out/ms12/tests.log 2>&1 || exit 1
for r in 1 2; do
timeout -k 10 120 python3 benchmarks/bench_sort.py --n 1048576 4194304 16777216 50331648 --dtype int32 --algo merge --reps 10 >> gpurun_out/ms12/bench.jsonl 2>>gpurun_out/ms12/bench.err || exit 1
timeout -k 10 120 python3 benchmarks/bench_sort.py --n 16777216 50331648 --dtype int32 --algo merge --values --reps 10 >> gpurun_out/ms12/bench.jsonl 2>>gpurun_out/ms12/bench.err || exit 1
done
