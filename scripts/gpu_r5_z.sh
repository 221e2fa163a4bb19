set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ms
export TMPDIR=/tmp
timeout -k 10 120 python3 benchmarks/bench_sort.py --n 50331648 --dtype int32 --algo merge torch --reps 10 > gpurun_out/ms/bench.jsonl 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ms -o k -- python3 benchmarks/bench_sort.py --n 50331648 --dtype int32 --algo merge --reps 3 > gpurun_out/ms/run.log 2>&1
