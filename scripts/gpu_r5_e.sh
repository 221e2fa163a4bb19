set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_dist_ipc_gpu.py -k eight > gpurun_out/t8.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --share-gpu --steps 20 --warmup 5 > gpurun_out/share8.json 2> gpurun_out/share8.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 --share-gpu --steps 200 --warmup 20 > gpurun_out/share8_200.json 2> gpurun_out/share8_200.err
