#!/usr/bin/env python3
"""Look-back scan tuning / diagnosis at 2^26 fp32: rows per lane x lookback
on/off, against torch.cumsum and the 16-B copy of the same bytes."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import cme213x
    from cme213x import _ext
    from cme213x.ops.scan import workspace

    _ext.proto(_ext.TUNE_PROTOS, "cme_scan_tune", "ppqiipp")
    n = 1 << 26
    x = torch.rand(n, device="cuda")
    y = torch.empty_like(x)
    ws = workspace(x.device, (n // 1024 + 1) * 16 + (n // 65536 + 1) * 16 + 64)
    s = _ext.stream_ptr()
    arms = [int(a) for a in os.environ.get("CME_SCAN_ARMS", "1,0,3,6,7,8,9,10").split(",")]
    cfgs = [(r, lb) for r in (4, 8, 16) for lb in arms]
    fns = {c: (lambda c=c: _ext.call_hip("cme_scan_tune", x.data_ptr(), y.data_ptr(), n, c[0], c[1],
                                         ws.data_ptr(), s)) for c in cfgs}
    fns["cumsum"] = lambda: torch.cumsum(x, 0, out=y)
    from cme213x.ops.scan import scan as cscan
    fns["rts"] = lambda: cscan(x, True, y, "rts")
    from cme213x.ops.scan import _tw

    times = {k: [] for k in fns}
    for k, fn in fns.items():  # one warm call per arm, with its give-up word checked
        fn()
        torch.cuda.synchronize()
        print(json.dumps({"warm": str(k), "timeout": int(_tw().value)}), flush=True)
        _tw().value = 0
    for _ in range(7):
        for k, fn in fns.items():
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / 10)
    for k, t in times.items():
        ms = sorted(t)[3]
        print(json.dumps({"cfg": k, "ms": round(ms, 4), "GBps": round(8 * n / ms / 1e6, 1)}), flush=True)
    # correctness of the production arms
    ref = torch.cumsum(x.double(), 0) - x.double()
    for c in cfgs:
        if c[1] == 0:
            continue
        fns[c]()
        torch.cuda.synchronize()
        err = ((y.double() - ref).abs().max() / ref.abs().max()).item()
        timed_out = int(_tw().value)
        _tw().value = 0
        print(json.dumps({"cfg": c, "max_rel_err": err, "timeout": timed_out}))


def spmv_main():
    """--spmv: segmented (SpMV-scan) look-back variants on three final-project
    shapes: rows per lane 4/8 x next-tile prefetch."""
    import torch

    import cme213x
    from cme213x import _ext
    from cme213x.models.spmv_scan import BENCH_SHAPES, SpmvScanSolver, generate
    from cme213x.ops.scan import _run_ws

    _ext.proto(_ext.TUNE_PROTOS, "cme_spmv_scan_tune", "pppqipiip")
    s = _ext.stream_ptr()
    mats = os.environ.get("CME_SPMV_MATS", "pwtk webbase-1M mac_econ_fwd500 jonheart").split()
    modes = [int(m) for m in os.environ.get("CME_SPMV_MODES", "0 1 2 3 6 7").split()]
    rows_list = [int(r) for r in os.environ.get("CME_SPMV_ROWS", "4 8 16").split()]
    for name in mats:
        n, p, N = BENCH_SHAPES[name]
        sol = SpmvScanSolver(generate(n, p, 100000, N, seed=1), "cuda")
        ws = _run_ws(sol.a)
        a0 = sol.a.clone()
        ref = None
        from cme213x.ops.scan import _tw
        for rows in rows_list:
            for pf in modes:  # bit 0 prefetch, bit 1 two-level look-back, bit 2 one launch for all steps
                f = lambda: _ext.call_hip("cme_spmv_scan_tune", sol.a.data_ptr(), sol.xx.data_ptr(),  # noqa
                                          sol.flags.data_ptr(), n, N, ws.data_ptr(), rows, pf, s)
                sol.a.copy_(a0)
                f()
                torch.cuda.synchronize()
                if ref is None:
                    ref = sol.a.clone()
                err = float(((sol.a - ref).abs().max() / ref.abs().max().clamp(min=1e-30)).item())
                print(json.dumps({"matrix": name, "rows": rows, "mode": pf, "rel_err_vs_r4m0": err,
                                  "timeout": int(_tw().value)}), flush=True)
                _tw().value = 0
                ts = []
                for _ in range(5):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    f()
                    e1.record()
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1))
                ms = sorted(ts)[2]
                print(json.dumps({"matrix": name, "rows": rows, "mode": pf, "ms": round(ms, 4),
                                  "GBps": round(12 * n * N / ms / 1e6)}), flush=True)


if __name__ == "__main__":
    spmv_main() if "--spmv" in sys.argv else main()
