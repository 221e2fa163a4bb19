# Reassociated ("fast") arithmetic arms of the pipelined pass vs FMA, random and constant data
set -o pipefail
mkdir -p gpurun_out/fast
TUNE_SPIN=2 TUNE_REPS=12 TUNE_H=16384,2048 TUNE_NS=4 TUNE_RB=4 TUNE_PD=11,12,13 TUNE_PERCU=0 timeout -k 10 300 python -u benchmarks/tune_heat_pipe.py > gpurun_out/fast/rand.jsonl 2>&1 || { tail -20 gpurun_out/fast/rand.jsonl; exit 1; }
TUNE_DATA=const TUNE_SPIN=2 TUNE_REPS=12 TUNE_H=16384,2048 TUNE_NS=4 TUNE_RB=4 TUNE_PD=11,12,13 TUNE_PERCU=0 timeout -k 10 300 python -u benchmarks/tune_heat_pipe.py > gpurun_out/fast/const.jsonl 2>&1 || { tail -20 gpurun_out/fast/const.jsonl; exit 1; }
grep -h '^{"H' gpurun_out/fast/rand.jsonl gpurun_out/fast/const.jsonl | cut -c1-140
