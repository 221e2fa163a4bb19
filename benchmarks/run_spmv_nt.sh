# A/B of the non-temporal CSR stream loads (tuning knob spmv_nt): bench_primitives SpMV set (one operand set,
# batched calls) and bench_spmv cold/warm (hipGraph, 768 MB rotation) for the aligned and column-blocked CSR
set -o pipefail
cd $GRAFT_REPO_ROOT
for nt in 1 0 1 0; do
  CME_SPMV_NT=$nt timeout -k 10 200 python3 -u benchmarks/bench_primitives.py --only spmv 2>/dev/null | sed "s/^{/{\"spmv_nt\": $nt, /" >> gpurun_out/spmv_nt_ab.jsonl || exit 1
done
for nt in 1 0 1 0; do
  CME_SPMV_NT=$nt timeout -k 10 300 python3 -u benchmarks/bench_spmv.py --fmts csr_aligned csr_cb 2>/dev/null | sed "s/^{/{\"spmv_nt\": $nt, /" >> gpurun_out/spmv_nt_cold.jsonl || exit 1
done
