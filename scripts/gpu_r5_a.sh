set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_spmv.py tests/test_radix_onesweep.py tests/test_bench_contract.py > gpurun_out/t1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b1.json 2> gpurun_out/b1.err
