set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_tile
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_tile -o tile -- python3 benchmarks/bench_hw5.py --n 1000 --reps 1 > gpurun_out/pmc_tile/run.log 2>&1
