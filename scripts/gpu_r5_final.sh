set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/final_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 && \
timeout -k 10 200 python -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err
