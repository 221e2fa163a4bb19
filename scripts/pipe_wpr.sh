# Pipelined pass: unconditional prefetch (no phi copies waiting on fresh loads) -- tests, bench, sweep
set -o pipefail
mkdir -p gpurun_out/wpr
timeout -k 10 300 python -u -m pytest tests/test_heat_pipe.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wpr/pytest.log 2>&1 || { tail -30 gpurun_out/wpr/pytest.log; exit 1; }
tail -1 gpurun_out/wpr/pytest.log
timeout -k 10 200 python bench.py > gpurun_out/wpr/bench.log 2>&1 || { tail gpurun_out/wpr/bench.log; exit 1; }
cut -c1-400 gpurun_out/wpr/bench.log
TUNE_SPIN=2 TUNE_REPS=12 TUNE_H=16384,2048 TUNE_NS=4 TUNE_RB=4 TUNE_PD=1,2,11,21,41 TUNE_PERCU=0,1,2 timeout -k 10 500 python -u benchmarks/tune_heat_pipe.py > gpurun_out/wpr/tune4c.jsonl 2>&1 || { tail -20 gpurun_out/wpr/tune4c.jsonl; exit 1; }
cut -c1-160 gpurun_out/wpr/tune4c.jsonl
