# Kernel timeline of one N=8 rank's native schedule (pipe, 4 steps/pass, exchange off)
set -o pipefail
mkdir -p gpurun_out/dtrace
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dtrace/t -o tr -- python3 benchmarks/bench_dist_rank.py --kernel pipe --tblock 4 --steps 240 --world 8 --reps 2 > gpurun_out/dtrace/run.log 2>&1 || { tail gpurun_out/dtrace/run.log; exit 1; }
find gpurun_out/dtrace -name "*kernel_trace.csv" | head -3
