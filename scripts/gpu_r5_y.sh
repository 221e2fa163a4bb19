set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_sort
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmc_sort -o p -- python3 benchmarks/bench_sort.py --n 16777216 --algo radix --reps 3 > gpurun_out/pmc_sort/run.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/pmc_sort -o q -- python3 benchmarks/bench_sort.py --n 16777216 --algo radix --reps 3 >> gpurun_out/pmc_sort/run.log 2>&1 && \
timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_sort -o k -- python3 benchmarks/bench_sort.py --n 16777216 --algo radix --reps 3 >> gpurun_out/pmc_sort/run.log 2>&1
