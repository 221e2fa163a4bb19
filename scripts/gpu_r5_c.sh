set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u benchmarks/trace_flow.py --n 16384 --passes 6 --out gpurun_out/trace_flow.jsonl > gpurun_out/tf.log 2>&1 && \
timeout -k 10 200 python -u benchmarks/trace_flow.py --n 16384 --passes 6 --mode 4096 --out gpurun_out/trace_flow.jsonl >> gpurun_out/tf.log 2>&1 && \
timeout -k 10 200 python -u benchmarks/trace_pipe_tasks.py --n 16384 --world 1 > gpurun_out/tp.log 2>&1
