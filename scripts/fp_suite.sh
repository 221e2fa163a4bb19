#!/usr/bin/env bash
# Run the final-project SpMV-scan over a benchmark suite -- the equivalent of
# hw/hw_final/programming/do_test.sh (loop over ~/benchmarksuite/*/): each
# subdirectory holds a.txt / x.txt (see `python -m cme213x readmm|genfp`);
# fp writes b.txt there and the checker prints the error norms.
#   scripts/fp_suite.sh <suite_dir> [--algo lookback|wave|serial]
set -euo pipefail
SUITE=${1:?usage: fp_suite.sh <suite_dir> [--algo ALGO]}
shift
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
for d in "$SUITE"/*/; do
    [ -f "$d/a.txt" ] && [ -f "$d/x.txt" ] || continue
    echo "== $(basename "$d")"
    (cd "$d" && python "$ROOT/cme213x_cli.py" fp a.txt x.txt "$@" && python "$ROOT/cme213x_cli.py" checker a.txt x.txt b.txt)
done
