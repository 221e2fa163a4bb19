set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_2000
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_2000 -o p -- python3 benchmarks/bench_hw5.py --n 2000 --reps 1 > gpurun_out/pmc_2000/run.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_2000 -o k -- python3 benchmarks/bench_hw5.py --n 2000 --reps 1 >> gpurun_out/pmc_2000/run.log 2>&1
