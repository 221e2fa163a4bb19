set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_scan2
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_scan.py > gpurun_out/tscan2.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_scan2 -o scan -- python3 benchmarks/scan_algos_once.py > gpurun_out/prof_scan2/run.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-arith-compare > gpurun_out/bn.json 2> gpurun_out/bn.err
