# SpMV after the size-based stream-load default (spmv_nt=2): GPU tests, cold/warm table, primitives SpMV set
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_spmv.py > gpurun_out/spmv_tests.log 2>&1 &&
timeout -k 10 400 python3 -u benchmarks/bench_spmv.py > gpurun_out/spmv_cold_r4.jsonl 2>/dev/null &&
timeout -k 10 200 python3 -u benchmarks/bench_primitives.py --only spmv > gpurun_out/prims_spmv_r4.jsonl 2>/dev/null
