set -o pipefail
mkdir -p gpurun_out/verify
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/verify/pytest_gpu.log 2>&1 && \
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/verify/smoke.log 2>&1 && \
timeout -k 10 180 python bench.py > gpurun_out/verify/bench.log 2>&1
echo "rc=$?"; tail -3 gpurun_out/verify/pytest_gpu.log; cat gpurun_out/verify/bench.log
