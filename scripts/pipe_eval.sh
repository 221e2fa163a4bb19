# Wave-pipelined heat pass: tests, kernel sweep, one-rank strong-scaling schedule
set -o pipefail
mkdir -p gpurun_out/pipe
timeout -k 10 300 python -u -m pytest tests/test_heat_pipe.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe/pytest.log 2>&1 || { tail -30 gpurun_out/pipe/pytest.log; exit 1; }
tail -2 gpurun_out/pipe/pytest.log
TUNE_NS=3,4 TUNE_RB=4,8 TUNE_PD=1,2 TUNE_PERCU=0,8,12 timeout -k 10 300 python -u benchmarks/tune_heat_pipe.py > gpurun_out/pipe/tune2.jsonl 2>&1 || exit 1
for k in "pipe 4" "pipe 3" "streamn 3" "streamn 4"; do
  set -- $k
  timeout -k 10 300 python -u benchmarks/bench_dist_rank.py --kernel $1 --tblock $2 --steps 240 >> gpurun_out/pipe/dist_rank.jsonl 2>&1 || exit 1
done
timeout -k 10 200 python bench.py > gpurun_out/pipe/bench_streamn.log 2>&1 || exit 1
cat gpurun_out/pipe/dist_rank.jsonl gpurun_out/pipe/bench_streamn.log
