set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_r5
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r5 -o bench -- python3 bench.py --steps 20 --warmup 5 --no-primitives --no-arith-compare > gpurun_out/prof_r5/bench.json 2> gpurun_out/prof_r5/bench.err
