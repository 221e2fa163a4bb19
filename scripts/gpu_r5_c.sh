set -o pipefail
cd $GRAFT_REPO_ROOT
for n in 2048 4096 8192 16384; do
timeout -k 10 200 python -u benchmarks/trace_flow.py --n $n --passes 5 --out gpurun_out/trace_flow_sizes.jsonl >> gpurun_out/tfs.log 2>&1 || exit 1
done
