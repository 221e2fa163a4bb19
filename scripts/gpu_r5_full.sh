set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/full_gpu.log 2>&1
