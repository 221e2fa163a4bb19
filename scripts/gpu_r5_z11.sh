set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sp11
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_spmv.py -m gpu > gpurun_out/sp11/tests.log 2>&1 || exit 1
for r in 1 2; do
timeout -k 10 200 python3 benchmarks/bench_spmv.py --mats 5pt-1M 5pt-16M 27pt-1M random-1M --fmts csr_short csr_scalar csr_stream ell --out gpurun_out/sp11/spmv.jsonl > /dev/null 2>>gpurun_out/sp11/err.log || exit 1
done
timeout -k 10 200 python3 benchmarks/bench_spmv.py --mats 5pt-1M 5pt-16M --fmts csr_short --tune spmv_short_rpt=2 --out gpurun_out/sp11/spmv.jsonl > /dev/null 2>>gpurun_out/sp11/err.log
