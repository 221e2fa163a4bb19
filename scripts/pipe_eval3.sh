# Production pipe (NT stores): tests, bench, one-rank schedule, rocprofv3 stats + counters
set -o pipefail
mkdir -p gpurun_out/pipe3
timeout -k 10 300 python -u -m pytest tests/test_heat_pipe.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe3/pytest.log 2>&1 || { tail -30 gpurun_out/pipe3/pytest.log; exit 1; }
tail -1 gpurun_out/pipe3/pytest.log
timeout -k 10 200 python bench.py > gpurun_out/pipe3/bench.log 2>&1 || exit 1
timeout -k 10 300 python -u benchmarks/bench_dist_rank.py --kernel pipe --tblock 4 --steps 240 > gpurun_out/pipe3/dist_rank.jsonl 2>&1 || exit 1
cat gpurun_out/pipe3/bench.log gpurun_out/pipe3/dist_rank.jsonl | cut -c1-300
bash scripts/profile_heat.sh || exit 1
