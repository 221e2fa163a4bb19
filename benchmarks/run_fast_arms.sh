set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_heat_pipe.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fast_arms or pipe_bitwise or wide" > gpurun_out/fast_tests.log 2>&1 || exit 1
TUNE_NS=4 TUNE_RB=2 TUNE_PD=85,91,92,95,96 TUNE_PERCU=0 TUNE_H=16384,2048 TUNE_DATA=rand timeout -k 10 240 python benchmarks/tune_heat_pipe.py > gpurun_out/fast_rand.jsonl 2>&1 || exit 2
TUNE_NS=4 TUNE_RB=2 TUNE_PD=85,91,92,95,96 TUNE_PERCU=0 TUNE_H=16384,2048 TUNE_DATA=const timeout -k 10 240 python benchmarks/tune_heat_pipe.py > gpurun_out/fast_const.jsonl 2>&1 || exit 3
