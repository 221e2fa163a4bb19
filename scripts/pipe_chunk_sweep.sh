# Chunk rule / steps per pass of the production pipelined pass on the bench's field (IC 5.0)
set -o pipefail
mkdir -p gpurun_out/pcs
TUNE_DATA=const TUNE_SPIN=2 TUNE_REPS=12 TUNE_H=16384,2048 TUNE_NS=4 TUNE_RB=4 TUNE_PD=11 TUNE_PERCU=0,3,4,5,6,8,10 TUNE_CHUNKS=64,96,128,192,256,400,640 timeout -k 10 400 python -u benchmarks/tune_heat_pipe.py > gpurun_out/pcs/sweep.jsonl 2>&1 || { tail -20 gpurun_out/pcs/sweep.jsonl; exit 1; }
grep -h '^{"H' gpurun_out/pcs/sweep.jsonl | cut -c1-150 | head -12
grep -h '^{"H": 2048' gpurun_out/pcs/sweep.jsonl | cut -c1-150 | head -6
TUNE_DATA=const TUNE_SPIN=2 TUNE_REPS=12 TUNE_H=16384,2048 TUNE_NS=5,6 TUNE_RB=4 TUNE_PD=11 TUNE_PERCU=0,2,3 timeout -k 10 400 python -u benchmarks/tune_heat_pipe.py > gpurun_out/pcs/ns56.jsonl 2>&1 || { tail -20 gpurun_out/pcs/ns56.jsonl; exit 1; }
grep -h '^{"H' gpurun_out/pcs/ns56.jsonl | cut -c1-150 | head -12
