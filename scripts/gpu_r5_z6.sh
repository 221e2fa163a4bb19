set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ms6
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/ms6 -o p -- python3 benchmarks/bench_sort.py --n 50331648 --dtype int32 --algo merge --reps 2 > gpurun_out/ms6/run.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD --output-format csv -d gpurun_out/ms6 -o q -- python3 benchmarks/bench_sort.py --n 50331648 --dtype int32 --algo merge --reps 2 >> gpurun_out/ms6/run.log 2>&1
