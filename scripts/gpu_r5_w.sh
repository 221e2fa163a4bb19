set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/sort_cap.jsonl
for cap in 1024 1536 2048 3072 4096; do
  timeout -k 10 200 python -u benchmarks/bench_sort.py --n 16777216 48000000 --algo radix --tune radix_maxblocks=$cap >> gpurun_out/sort_cap.jsonl 2>/dev/null || exit 1
done
