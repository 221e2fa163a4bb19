set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_heat_tile_res.py > gpurun_out/tres.log 2>&1 && \
for a in "" "--tune tile_res_minr=2" "--tune tile_res_minr=3" "--ns 4 --passes 250" "--ns 4 --passes 250 --tune tile_res_minr=2" "--fma" "--fma --tune tile_res_minr=2"; do
  timeout -k 10 100 python -u benchmarks/trace_tile_res.py $a --out gpurun_out/trace_res2.jsonl || exit 1
done
