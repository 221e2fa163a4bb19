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

    _ext.proto(_ext.HIP_PROTOS, "cme_scan_tune", "ppqiipp")
    n = 1 << 26
    x = torch.rand(n, device="cuda")
    y = torch.empty_like(x)
    ws = workspace(x.device, (n // 1024 + 1) * 8 + 16)
    s = _ext.stream_ptr()
    cfgs = [(r, lb) for r in (4, 8) for lb in (1, 0)]
    fns = {c: (lambda c=c: _ext.call_hip("cme_scan_tune", x.data_ptr(), y.data_ptr(), n, c[0], c[1],
                                         ws.data_ptr(), s)) for c in cfgs}
    fns["cumsum"] = lambda: torch.cumsum(x, 0, out=y)
    from cme213x.ops.scan import scan as cscan
    fns["rts"] = lambda: cscan(x, True, y, "rts")
    times = {k: [] for k in fns}
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
        print(json.dumps({"cfg": k, "ms": round(ms, 4), "GBps": round(8 * n / ms / 1e6, 1)}))
    # correctness of the production arms
    for r in (4, 8):
        fns[(r, 1)]()
        ref = torch.cumsum(x.double(), 0) - x.double()
        err = ((y.double() - ref).abs().max() / ref.abs().max()).item()
        print(json.dumps({"rows": r, "max_rel_err": err}))


if __name__ == "__main__":
    main()
