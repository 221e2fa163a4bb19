# Pipelined pass after the prefetch fix: rocprofv3 stats + counters, one rank's share at N=1..8
set -o pipefail
mkdir -p gpurun_out/hpf
timeout -k 10 400 python -u benchmarks/bench_dist_rank.py --kernel pipe --tblock 4 --steps 240 > gpurun_out/hpf/dist_rank.jsonl 2>&1 || { tail gpurun_out/hpf/dist_rank.jsonl; exit 1; }
grep '^{' gpurun_out/hpf/dist_rank.jsonl | cut -c1-250
bash scripts/profile_heat.sh || exit 1
python scripts/summarize_prof.py gpurun_out/prof_heat gpurun_out/hpf/prof.md "rocprofv3: pipelined 4-step pass after the prefetch fix" || exit 1
