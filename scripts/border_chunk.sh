# Border-strip chunk floor of the pipelined pass: one rank's share at N=1..8, methods 1 and 2
set -o pipefail
mkdir -p gpurun_out/bc
for t in 4 16 32 64 128; do
  CME_PIPE_THIN_MIN=$t timeout -k 10 300 python -u benchmarks/bench_dist_rank.py --kernel pipe --tblock 4 --steps 240 --reps 3 > gpurun_out/bc/m1_$t.jsonl 2>&1 || { tail gpurun_out/bc/m1_$t.jsonl; exit 1; }
  echo "thin_min=$t method1: $(grep -h '^{' gpurun_out/bc/m1_$t.jsonl | python3 -c 'import sys,json; print([json.loads(l)["ms_per_step"] for l in sys.stdin])')"
done
for t in 4 64; do
  CME_PIPE_THIN_MIN=$t timeout -k 10 300 python -u benchmarks/bench_dist_rank.py --kernel pipe --tblock 4 --steps 240 --reps 3 --method 2 > gpurun_out/bc/m2_$t.jsonl 2>&1 || { tail gpurun_out/bc/m2_$t.jsonl; exit 1; }
  echo "thin_min=$t method2: $(grep -h '^{' gpurun_out/bc/m2_$t.jsonl | python3 -c 'import sys,json; print([json.loads(l)["ms_per_step"] for l in sys.stdin])')"
done
