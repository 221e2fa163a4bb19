set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_heat_flow.py tests/test_heat_tile_res.py > gpurun_out/tpersist.log 2>&1
