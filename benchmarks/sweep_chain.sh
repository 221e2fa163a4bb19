# Rehearsal of the border -> exchange -> border chain of an N = 8 rank on one
# GPU: transport "none" plus a fixed-latency stand-in for the network part of
# each exchange (CME_DIST_FAKE_XCHG_US), against the share of resident waves
# the interior may take (CME_STREAMN_CAPPCT). Results: profiles/dist_chain_r2.md
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
FX=${FX:-"0 20 40"}
CAPS=${CAPS:-"100 85 70"}
TBS=${TBS:-"3 4"}
for fx in $FX; do for cp in $CAPS; do for tb in $TBS; do
  echo "fx=$fx cap=$cp tb=$tb" >> gpurun_out/chain.log
  CME_DIST_FAKE_XCHG_US=$fx CME_STREAMN_CAPPCT=$cp timeout -k 10 120 python -u benchmarks/bench_dist_rank.py --world 8 --tblock $tb --steps 240 --reps 3 >> gpurun_out/chain.log 2>&1 || exit 1
done; done; done
echo done >> gpurun_out/chain.log
