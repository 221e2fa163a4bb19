set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prims
timeout -k 10 900 python3 -u benchmarks/bench_primitives.py > gpurun_out/prims/bench_primitives_r5.jsonl 2> gpurun_out/prims/err.log
