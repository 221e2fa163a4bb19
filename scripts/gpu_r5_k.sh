set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CME_TILE_STORE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_heat_tile.py -k "1000 or hw5" > gpurun_out/tts1.log 2>&1 && \
CME_TILE_STORE=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_heat_tile.py -k "1000 or hw5" > gpurun_out/tts2.log 2>&1 && \
for a in "" "--tune tile_store=1" "--tune tile_store=2" "" "--tune tile_store=1" "--tune tile_store=2"; do
  timeout -k 10 120 python -u benchmarks/bench_hw5.py --n 1000 --reps 7 $a >> gpurun_out/hw5_store.jsonl 2>&1 || exit 1
  timeout -k 10 120 python -u benchmarks/bench_hw5.py --n 1000 --reps 7 --fma $a >> gpurun_out/hw5_store.jsonl 2>&1 || exit 1
done
