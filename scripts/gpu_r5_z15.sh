set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/h15
run() {  # $1 label, rest: env assignments
  local label=$1; shift
  env "$@" timeout -k 10 150 python3 bench.py --ic random --no-primitives --no-arith-compare --steps 20 --warmup 5 > gpurun_out/h15/one.json 2>>gpurun_out/h15/err.log || return 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/h15/one.json').read().strip().splitlines()[-1]); print(json.dumps({'label': '$label', 'ms': d['ms_per_step'], 'value': d['value']}))" >> gpurun_out/h15/sweep.jsonl
}
for rep in 1 2; do
  run default CME_DUMMY=0 || exit 1
  run per_cu2 CME_PIPE_PER_CU=2 || exit 1
  run per_cu4 CME_PIPE_PER_CU=4 || exit 1
  run vw4 CME_PIPE_VW=4 || exit 1
  run taper CME_PIPE_TAPER=-1 || exit 1
done
