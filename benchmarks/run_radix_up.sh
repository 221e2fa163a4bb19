# radix upsweep loads in flight (tuning knob radix_up_unr) A/B: 16M / 48M uint32, 16M int32 key-value, 16M small keys
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_radix_onesweep.py tests/test_sort_text.py > gpurun_out/radix_up_tests.log 2>&1 || exit 1
for r in 1 2; do
for u in 4 8 16; do
  timeout -k 10 120 python3 -u benchmarks/bench_sort.py --algo radix --n 16000000 48000000 --tune radix_up_unr=$u 2>/dev/null | sed "s/^{/{\"up_unr\": $u, /" >> gpurun_out/radix_up.jsonl || exit 1
  timeout -k 10 120 python3 -u benchmarks/bench_sort.py --algo radix --n 16000000 --dtype int32 --values --tune radix_up_unr=$u 2>/dev/null | sed "s/^{/{\"up_unr\": $u, /" >> gpurun_out/radix_up.jsonl || exit 1
  timeout -k 10 120 python3 -u benchmarks/bench_sort.py --algo radix --n 16000000 --kind small --tune radix_up_unr=$u 2>/dev/null | sed "s/^{/{\"up_unr\": $u, /" >> gpurun_out/radix_up.jsonl || exit 1
done
done
