set -o pipefail
cd $GRAFT_REPO_ROOT
for tb in 3 4; do for mc in 64 96 128 192; do for r in 1 2 3; do
  echo "tb=$tb minchunk=$mc rounds=$r" >> gpurun_out/n4sweep.log
  CME_STREAMN_MINCHUNK=$mc CME_STREAMN_ROUNDS=$r timeout -k 10 120 python -u benchmarks/bench_dist_rank.py --world 4 8 --tblock $tb --steps 240 --reps 3 >> gpurun_out/n4sweep.log 2>&1 || exit 1
done; done; done
