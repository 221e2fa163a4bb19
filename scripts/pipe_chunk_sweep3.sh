# Height-dependent tasks-per-CU default vs fixed arms; tests; bench; one rank share
set -o pipefail
mkdir -p gpurun_out/pcs
timeout -k 10 300 python -u -m pytest tests/test_heat_pipe.py tests/test_dist_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pcs/pytest.log 2>&1 || { tail -30 gpurun_out/pcs/pytest.log; exit 1; }
tail -1 gpurun_out/pcs/pytest.log
TUNE_DATA=const TUNE_SPIN=2 TUNE_REPS=12 TUNE_H=16384,8192,4096,2048 TUNE_NS=4 TUNE_RB=4 TUNE_PD=11 TUNE_PERCU=0,8,14 timeout -k 10 400 python -u benchmarks/tune_heat_pipe.py > gpurun_out/pcs/sweep3.jsonl 2>&1 || { tail -20 gpurun_out/pcs/sweep3.jsonl; exit 1; }
grep -h '^{"H' gpurun_out/pcs/sweep3.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    if d['kernel'] == 'pipe': print(d['H'], d['per_cu'], d['ms_per_step'])
"
timeout -k 10 200 python bench.py > gpurun_out/pcs/bench.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/pcs/bench.log
timeout -k 10 300 python -u benchmarks/bench_dist_rank.py --kernel pipe --tblock 4 --steps 240 --reps 3 > gpurun_out/pcs/rank.jsonl 2>&1 || exit 1
grep -h '^{' gpurun_out/pcs/rank.jsonl | python3 -c 'import sys,json; print([json.loads(l)["ms_per_step"] for l in sys.stdin])'
