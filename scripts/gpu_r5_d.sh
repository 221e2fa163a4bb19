set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_spmv.py > gpurun_out/t5.log 2>&1 && \
for r in 256 512 1024; do
timeout -k 10 200 python -u benchmarks/bench_spmv.py --mats 5pt-1M 27pt-1M --fmts csr_stream csr_scalar ell --tune spmv_stream_rows=$r --out gpurun_out/spmv_stream_r5.jsonl > gpurun_out/spmv2.log 2>&1 || exit 1
done
