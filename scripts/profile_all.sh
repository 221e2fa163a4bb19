#!/bin/bash
# rocprofv3 runs for the committed profiles/ summaries. Kernel-trace stats and
# PMC counters are collected in SEPARATE runs (never --pmc with sys/runtime
# tracing). Each step is time-limited; stop at the first crash.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
cd /tmp || exit 1
step() {  # name secs cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name" | tee -a "$R/gpurun_out/prof/steps.log"
  timeout -k 10 "$secs" "$@" > "$R/gpurun_out/prof/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$R/gpurun_out/prof/steps.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step bench_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof/bench" -o bench -- python3 "$R/bench.py" --steps 30 --warmup 3
step prims_stats 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof/prims" -o prims -- python3 "$R/benchmarks/bench_primitives.py" --only scan transpose spmv sort
step transpose_lds 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES --output-format csv -d "$R/gpurun_out/prof/transpose_pmc" -o tr -- python3 "$R/benchmarks/transpose_study.py"
step heat_bytes 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/prof/heat_fetch" -o heat -- python3 "$R/bench.py" --steps 5 --warmup 1
step heat_wbytes 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/prof/heat_write" -o heat -- python3 "$R/bench.py" --steps 5 --warmup 1
echo all-ok
