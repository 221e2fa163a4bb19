#!/bin/bash
# The one parameterised GPU runner (it replaced round 5's 59 one-off
# scripts/gpu_r5_*.sh launchers). Runs a sequence of named steps, each under
# its own time limit, from the repository root; every step's output goes to
# gpurun_out/<name>.log and a summary line to gpurun_out/session.log. Stops at
# the first step that crashed or timed out (any exit code other than 0 = ok
# and 1 = test failure), so nothing more touches a GPU that may be faulted.
#
#   scripts/gpu_session.sh "<name>:<seconds>:<command>" ...
#
# Examples (through /usr/local/graft/bin/gpurun):
#   bash scripts/gpu_session.sh "tests:900:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" \
#                               "smoke:120:python -u -c 'import __graft_entry__ as g; g.smoke()'" \
#                               "bench:300:python -u bench.py --gpus 1 --steps 20 --warmup 5"
#   bash scripts/gpu_session.sh "rank:300:python -u benchmarks/bench_dist_rank.py --kernel pipe --tblock 4 --arith fast"
#   bash scripts/gpu_session.sh "prof:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o x -- python3 benchmarks/scan_algos_once.py"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] ($secs s) $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start )) s" | tee -a gpurun_out/session.log
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: step $name exited $rc" | tee -a gpurun_out/session.log
    exit $rc
  fi
done
exit 0
