set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ms7
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_radix_onesweep.py tests/test_sort_text.py tests/test_drivers.py tests/test_algorithms.py -m gpu > gpurun_out/ms7/tests.log 2>&1 || exit 1
timeout -k 10 120 python3 benchmarks/bench_sort.py --n 1048576 4194304 16777216 50331648 --dtype int32 --algo merge --reps 10 >> gpurun_out/ms7/bench.jsonl 2>>gpurun_out/ms7/bench.err || exit 1
timeout -k 10 120 python3 benchmarks/bench_sort.py --n 16777216 50331648 --dtype int32 --algo merge --values --reps 10 >> gpurun_out/ms7/bench.jsonl 2>>gpurun_out/ms7/bench.err || exit 1
timeout -k 10 120 python3 benchmarks/bench_sort.py --n 4194304 --dtype int32 --algo merge --reps 10 --tune merge_part=8 >> gpurun_out/ms7/bench.jsonl 2>>gpurun_out/ms7/bench.err || exit 1
timeout -k 10 120 python3 benchmarks/bench_sort.py --n 16777216 --dtype float32 --algo merge --reps 10 >> gpurun_out/ms7/bench.jsonl 2>>gpurun_out/ms7/bench.err || exit 1
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ms7 -o k -- python3 benchmarks/bench_sort.py --n 50331648 --dtype int32 --algo merge --reps 3 > gpurun_out/ms7/run.log 2>&1
