# Unconditional prefetch in every streaming heat kernel: tests, both bench kernels, BASELINE heat rows
set -o pipefail
mkdir -p gpurun_out/hpf
timeout -k 10 400 python -u -m pytest tests/test_heat.py tests/test_heat_pipe.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/hpf/pytest.log 2>&1 || { tail -30 gpurun_out/hpf/pytest.log; exit 1; }
tail -1 gpurun_out/hpf/pytest.log
timeout -k 10 200 python bench.py > gpurun_out/hpf/bench_pipe.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --kernel streamn --tblock 3 > gpurun_out/hpf/bench_streamn.log 2>&1 || exit 1
cut -c1-330 gpurun_out/hpf/bench_pipe.log gpurun_out/hpf/bench_streamn.log
timeout -k 10 300 python -u benchmarks/bench_heat.py --n 4000 --dtypes fp32 --orders 2 4 8 --variants stream stream2_fma stream3_fma stream4_fma pipe3_fma pipe4_fma > gpurun_out/hpf/heat4000.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u benchmarks/bench_heat.py --n 1000 2000 --dtypes fp64 --orders 8 --variants stream stream2_fma stream3_fma > gpurun_out/hpf/heat_fp64.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u benchmarks/bench_heat.py --n 4000 --dtypes fp64 --orders 4 --variants shared stream2_fma stream3_fma > gpurun_out/hpf/heat4000_fp64.jsonl 2>&1 || exit 1
cat gpurun_out/hpf/heat4000.jsonl gpurun_out/hpf/heat_fp64.jsonl gpurun_out/hpf/heat4000_fp64.jsonl | grep '^{' | cut -c1-160
