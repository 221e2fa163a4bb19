# Wave-pipelined heat pass as the default: tests (single grid, distributed loopback, IPC processes),
# bench.py with each kernel, one-rank schedule, NT arm
set -o pipefail
mkdir -p gpurun_out/pipe2
timeout -k 10 600 python -u -m pytest tests/test_heat_pipe.py tests/test_dist_gpu.py tests/test_dist_ipc_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pipe2/pytest.log 2>&1 || { tail -30 gpurun_out/pipe2/pytest.log; exit 1; }
tail -2 gpurun_out/pipe2/pytest.log
timeout -k 10 200 python bench.py > gpurun_out/pipe2/bench_pipe.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --kernel streamn > gpurun_out/pipe2/bench_streamn.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --kernel pipe --tblock 3 > gpurun_out/pipe2/bench_pipe3.log 2>&1 || exit 1
timeout -k 10 300 python -u benchmarks/bench_dist_rank.py --kernel pipe --tblock 4 --steps 240 > gpurun_out/pipe2/dist_rank.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u benchmarks/bench_dist_rank.py --kernel pipe --tblock 4 --steps 240 --method 2 >> gpurun_out/pipe2/dist_rank.jsonl 2>&1 || exit 1
TUNE_NS=4 TUNE_RB=4 TUNE_PD=1,2,11 TUNE_PERCU=0 timeout -k 10 300 python -u benchmarks/tune_heat_pipe.py > gpurun_out/pipe2/tune_nt.jsonl 2>&1 || exit 1
grep -h ms_per_step gpurun_out/pipe2/*.log | cut -c1-400; cat gpurun_out/pipe2/dist_rank.jsonl
