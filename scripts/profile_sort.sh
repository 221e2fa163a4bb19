#!/bin/bash
# rocprofv3 for the radix sort (bench_sort.py, 16M uint32 keys): kernel-trace
# stats, then SQ counter passes, each its own run (never --pmc with tracing).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
OUT=$R/gpurun_out/prof_sort
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
step() {  # name secs cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log"; exit $rc; fi
}
B="$R/benchmarks/bench_sort.py --algo radix --reps 5 ${SORT_ARGS:-}"
step stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o sort -- python3 $B
step sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$OUT/sq" -o sort -- python3 $B
step mem 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o sort -- python3 $B
step wr 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o sort -- python3 $B
echo all-ok
