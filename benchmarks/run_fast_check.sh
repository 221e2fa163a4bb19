# reassociated-arithmetic default on the GPU box: bench contract GPU tests,
# then bench.py default (fast) twice and --arith fma once, back to back
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_bench_contract.py tests/test_heat_fast.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fast_tests2.log 2>&1 || exit 1
for a in "" "--arith fma" ""; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 $a >> gpurun_out/fast_bench2.jsonl 2>&1 || exit 2
done
