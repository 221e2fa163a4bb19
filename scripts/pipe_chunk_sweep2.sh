# Tasks-per-CU rule of the production pipelined pass on the bench's field, finer sweep
set -o pipefail
mkdir -p gpurun_out/pcs
TUNE_DATA=const TUNE_SPIN=2 TUNE_REPS=12 TUNE_H=16384,8192,4096,2048 TUNE_NS=4 TUNE_RB=4 TUNE_PD=11 TUNE_PERCU=0,8,10,12,14,16,20 timeout -k 10 400 python -u benchmarks/tune_heat_pipe.py > gpurun_out/pcs/sweep2.jsonl 2>&1 || { tail -20 gpurun_out/pcs/sweep2.jsonl; exit 1; }
grep -h '^{"H' gpurun_out/pcs/sweep2.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    if d['kernel'] == 'pipe': print(d['H'], d['per_cu'], d['ms_per_step'])
"
