set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_spmv.py tests/test_studies.py > gpurun_out/tspmv.log 2>&1 && \
timeout -k 10 200 python -u benchmarks/bench_spmv.py --mats 5pt-1M 5pt-16M --fmts csr_short csr_stream csr_scalar ell --out gpurun_out/spmv_short.jsonl > gpurun_out/bs1.log 2>&1 && \
timeout -k 10 200 python -u benchmarks/bench_spmv.py --mats 5pt-1M 5pt-16M --fmts csr_short --tune spmv_short_rpt=1 --out gpurun_out/spmv_short.jsonl > gpurun_out/bs2.log 2>&1 && \
timeout -k 10 200 python -u benchmarks/bench_spmv.py --mats 5pt-1M 5pt-16M --fmts csr_short --tune spmv_short_rpt=4 --out gpurun_out/spmv_short.jsonl > gpurun_out/bs3.log 2>&1 && \
timeout -k 10 200 python -u benchmarks/bench_spmv.py --mats 27pt-1M random-1M --fmts csr_short csr_stream --out gpurun_out/spmv_short.jsonl > gpurun_out/bs4.log 2>&1
