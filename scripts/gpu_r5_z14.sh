set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/d14
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dist_ipc_gpu.py tests/test_rccl_self_gpu.py tests/test_dist_gpu.py -m gpu > gpurun_out/d14/tests.log 2>&1
