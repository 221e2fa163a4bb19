# Steps per pass under the fused schedule: one rank's share at N = 1..8, tblock 3 vs 4, stripes and blocks
set -o pipefail
mkdir -p gpurun_out/ftb
for tb in 3 4; do
  for m in 1 2; do
    timeout -k 10 300 python -u benchmarks/bench_dist_rank.py --kernel pipe --tblock $tb --method $m --steps 240 --reps 3 > gpurun_out/ftb/r_${tb}_$m.jsonl 2>&1 || { tail gpurun_out/ftb/r_${tb}_$m.jsonl; exit 1; }
    echo "tblock=$tb method=$m: $(grep -h '^{' gpurun_out/ftb/r_${tb}_$m.jsonl | python3 -c 'import sys,json; print([json.loads(l)["ms_per_step"] for l in sys.stdin])')"
  done
done
