set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ms2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_radix_onesweep.py -m gpu -k "merge" > gpurun_out/ms2/tests.log 2>&1 && \
for p in 1 0 1 0; do timeout -k 10 120 python3 benchmarks/bench_sort.py --n 16777216 50331648 --dtype int32 --algo merge --reps 10 --tune merge_part=$p >> gpurun_out/ms2/bench.jsonl 2>>gpurun_out/ms2/bench.err || exit 1; done && \
timeout -k 10 120 python3 benchmarks/bench_sort.py --n 50331648 --dtype int32 --algo merge --values --reps 10 --tune merge_part=1 >> gpurun_out/ms2/bench.jsonl 2>>gpurun_out/ms2/bench.err && \
timeout -k 10 120 python3 benchmarks/bench_sort.py --n 50331648 --dtype int32 --algo merge --values --reps 10 --tune merge_part=0 >> gpurun_out/ms2/bench.jsonl 2>>gpurun_out/ms2/bench.err && \
export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ms2 -o k -- python3 benchmarks/bench_sort.py --n 50331648 --dtype int32 --algo merge --reps 3 > gpurun_out/ms2/run.log 2>&1
