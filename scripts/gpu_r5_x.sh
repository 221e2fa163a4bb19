set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/hw5_tblock_sweep.py --n 2000 > gpurun_out/hw5_tb.jsonl 2>/dev/null && \
timeout -k 10 300 python -u benchmarks/hw5_tblock_sweep.py --n 2000 --fma >> gpurun_out/hw5_tb.jsonl 2>/dev/null
