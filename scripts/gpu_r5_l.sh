set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for tb in 4 3; do
  timeout -k 10 200 python -u benchmarks/bench_dist_rank.py --kernel pipe --tblock $tb --world 2 4 8 --arith fma >> gpurun_out/drank_tb.jsonl 2>&1 || exit 1
done
