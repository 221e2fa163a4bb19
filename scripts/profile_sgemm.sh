#!/bin/bash
# rocprofv3 counters for the production SGEMM at 8192^3 (and torch.mm for
# comparison): SQ stall breakdown + MFMA busy, then LDS conflicts -- one
# counter group per run (benchmarks/tune_sgemm.py with no tuning arms).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
OUT=$R/gpurun_out/prof_sgemm
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
D="$R/benchmarks/tune_sgemm.py"
A="--n 8192 --arms --calls 1 --reps 1"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES --output-format csv -d "$OUT/sq" -o sg -- python3 $D $A > "$OUT/sq.log" 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_F32 --output-format csv -d "$OUT/lds" -o sg -- python3 $D $A > "$OUT/lds.log" 2>&1 || exit $?
echo all-ok
