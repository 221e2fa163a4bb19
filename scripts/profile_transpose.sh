#!/bin/bash
# rocprofv3 counters for the transpose ladder (8192^2): LDS bank conflicts and
# LDS instructions, then HBM bytes -- one counter group per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
OUT=$R/gpurun_out/prof_transpose
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
D="$R/benchmarks/transpose_prof_driver.py"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o tr -- python3 $D > "$OUT/stats.log" 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAVES --output-format csv -d "$OUT/lds" -o tr -- python3 $D > "$OUT/lds.log" 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o tr -- python3 $D > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o tr -- python3 $D > "$OUT/write.log" 2>&1 || exit $?
echo all-ok
