#!/usr/bin/env bash
# OMP_NUM_THREADS sweep of the hw4 CPU sorts -- the equivalent of the
# reference's PBS job (hw/hw4/programming/pa4.pbs: radixsort / mergesort for
# thread counts 1..64). Output: one "threads <t>" header followed by each
# program's own timing lines.
#   scripts/omp_sweep.sh [n] [max_threads]
set -euo pipefail
N=${1:-40000000}
MAXT=${2:-$(nproc)}
cd "$(dirname "$0")/.."
t=1
while [ "$t" -le "$MAXT" ]; do
    echo "threads $t"
    OMP_NUM_THREADS=$t python -m cme213x radixsort "$N" 8
    OMP_NUM_THREADS=$t python -m cme213x mergesort 2048 2048 "$N" 0
    t=$((t * 2))
done
