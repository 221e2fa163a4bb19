set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_spmv.py > gpurun_out/tspmv2.log 2>&1 && \
timeout -k 10 300 python -u benchmarks/bench_spmv.py --mats 5pt-1M 5pt-16M 27pt-1M random-1M --fmts ell hyb --out gpurun_out/spmv_ell.jsonl > gpurun_out/bse.log 2>&1
