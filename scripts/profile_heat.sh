#!/bin/bash
# rocprofv3 for the flagship heat kernel (bench.py defaults): kernel-trace
# stats, then one PMC pass per counter group in its own run (never --pmc with
# runtime/sys tracing; at most 8 SQ / 4 TCC counters per pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
OUT=$R/gpurun_out/prof_heat
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
B="$R/bench.py --steps ${STEPS:-30} --warmup 3 ${BENCH_ARGS:-}"
step stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o heat -- python3 $B
step fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o heat -- python3 $B
step write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o heat -- python3 $B
step sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD --output-format csv -d "$OUT/sq" -o heat -- python3 $B
step wait 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/wait" -o heat -- python3 $B
echo all-ok
