set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_spmv.py tests/test_library.py > gpurun_out/tspmv3.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-arith-compare > gpurun_out/br.json 2> gpurun_out/br.err
