#!/bin/bash
# rocprofv3 FETCH_SIZE / WRITE_SIZE per SpMV format (cache-defeated operand
# rotation, eager launches), one counter group per run (FETCH_SIZE takes 3 of
# the 4 TCC counters, WRITE_SIZE 2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
OUT=$R/gpurun_out/prof_spmv
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
B="$R/benchmarks/bench_spmv.py --eager --calls 8 --mats ${MATS:-5pt-1M 5pt-16M 27pt-1M random-1M skew-1M}"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o spmv -- python3 $B > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o spmv -- python3 $B > "$OUT/write.log" 2>&1 || exit $?
echo all-ok
