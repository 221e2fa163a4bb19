set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u benchmarks/stress_persistent.py --reps 40 > gpurun_out/stress.json 2> gpurun_out/stress.err
