set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sc13
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_scan.py -m gpu > gpurun_out/sc13/tests.log 2>&1 || exit 1
cat > /tmp/sc13.py <<'PY'
import json, torch, sys
sys.path.insert(0, ".")
import cme213x
from cme213x.ops import scan as sc
n = 1 << 26
g = torch.Generator(device="cuda").manual_seed(0)
x = (torch.rand(n, device="cuda", generator=g) < 0.2).float()
y = torch.empty_like(x)
ref = torch.cumsum(x.double(), 0).float()
for rep in range(3):
    for algo in ("lookback", "blelloch_lookback", "blelloch", "rts"):
        sc.scan(x, False, y, algo)
        ok = bool(torch.equal(y, ref))
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); sc.scan(x, False, y, algo); e1.record(); e1.synchronize(); ts.append(e0.elapsed_time(e1))
        ts.sort()
        print(json.dumps({"algo": algo, "n": n, "ms": round(ts[10], 4), "ok": ok}), flush=True)
PY
timeout -k 10 120 python3 /tmp/sc13.py > gpurun_out/sc13/bench.jsonl 2> gpurun_out/sc13/err.log
