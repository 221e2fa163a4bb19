set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3 4 5; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bv_$i.json 2>/dev/null || exit 1
  tail -1 gpurun_out/bv_$i.json >> gpurun_out/bench_variance_r5.jsonl
done
