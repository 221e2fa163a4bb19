set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_scan
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_scan -o scan -- python3 benchmarks/scan_algos_once.py > gpurun_out/prof_scan/run.log 2>&1
