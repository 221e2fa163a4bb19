# Fused distributed schedule (CME_DIST_SCHEDULE=2): correctness under IPC / RCCL-world-1 / bench rehearsal, then timing
set -o pipefail
mkdir -p gpurun_out/fused
export CME_DIST_SCHEDULE=2
timeout -k 10 600 python -u -m pytest tests/test_dist_ipc_gpu.py tests/test_dist_gpu.py tests/test_bench_contract.py -x -q --timeout 280 --timeout-method thread -m gpu > gpurun_out/fused/pytest.log 2>&1 || { tail -40 gpurun_out/fused/pytest.log; exit 1; }
tail -1 gpurun_out/fused/pytest.log
for sch in 0 2; do
  CME_DIST_SCHEDULE=$sch timeout -k 10 300 python -u benchmarks/bench_dist_rank.py --kernel pipe --tblock 4 --steps 240 --reps 3 > gpurun_out/fused/rank_$sch.jsonl 2>&1 || { tail gpurun_out/fused/rank_$sch.jsonl; exit 1; }
  echo "schedule=$sch method1: $(grep -h '^{' gpurun_out/fused/rank_$sch.jsonl | python3 -c 'import sys,json; print([json.loads(l)["ms_per_step"] for l in sys.stdin])')"
  CME_DIST_SCHEDULE=$sch timeout -k 10 300 python -u benchmarks/bench_dist_rank.py --kernel pipe --tblock 4 --steps 240 --reps 3 --method 2 > gpurun_out/fused/rank2_$sch.jsonl 2>&1 || { tail gpurun_out/fused/rank2_$sch.jsonl; exit 1; }
  echo "schedule=$sch method2: $(grep -h '^{' gpurun_out/fused/rank2_$sch.jsonl | python3 -c 'import sys,json; print([json.loads(l)["ms_per_step"] for l in sys.stdin])')"
  for us in 20 40 80; do
    CME_DIST_FAKE_XCHG_US=$us CME_DIST_SCHEDULE=$sch timeout -k 10 300 python -u benchmarks/bench_dist_rank.py --kernel pipe --tblock 4 --steps 240 --reps 3 --world 8 > gpurun_out/fused/chain_${sch}_$us.jsonl 2>&1 || { tail gpurun_out/fused/chain_${sch}_$us.jsonl; exit 1; }
    echo "schedule=$sch N=8 fake exchange ${us}us: $(grep -h '^{' gpurun_out/fused/chain_${sch}_$us.jsonl | python3 -c 'import sys,json; print([json.loads(l)["ms_per_step"] for l in sys.stdin])')"
  done
done
