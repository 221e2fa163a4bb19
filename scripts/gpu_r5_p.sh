set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
for pc in 0 2 3 4 6; do
  CME_PIPE_PER_CU=$pc timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-primitives --no-arith-compare > gpurun_out/pc_$pc.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/pc_$pc.json').read().strip().splitlines()[-1]); print('per_cu=$pc', d['ms_per_step'], d['ms_per_step_uniform'])" >> gpurun_out/pc_sweep.txt
done
done
