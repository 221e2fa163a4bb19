#!/usr/bin/env python3
"""Cold A/B of the look-back scan arms (csrc/hip_tune/scan_tune.hip
cme_scan_tune: rows per lane x look-back mode), bench.py's cold protocol:
3 operand sets of 2^26 fp32 uniform(0, 1) round-robin, median of 7 batches;
each arm checked against a float64 exclusive prefix first. Production is
rows 16, arm 18 (two-level look-back, two tiles in flight, non-temporal
stores).

    python benchmarks/tune_scan_cold.py [--rows 8 16] [--arms 18 15 14 16 1]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", default=[8, 16])
    ap.add_argument("--arms", type=int, nargs="+", default=[18, 15, 14, 16, 1])
    a = ap.parse_args()

    import torch

    import cme213x  # noqa: F401
    from cme213x import _ext
    from cme213x.ops.scan import _tw, workspace
    from bench import _cold_ms

    _ext.proto(_ext.TUNE_PROTOS, "cme_scan_tune", "ppqiipp")
    n = 1 << 26
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    sets = [(torch.rand(n, device=dev, generator=g), torch.empty(n, device=dev)) for _ in range(3)]
    ws = workspace(dev, (n // 1024 + 1) * 16 + (n // 65536 + 1) * 16 + 64)
    x0 = sets[0][0].double()
    ref = torch.cumsum(x0, 0) - x0
    scale = ref.abs().clamp_min(1.0)
    for rows in a.rows:
        for arm in a.arms:
            def fn(s, rows=rows, arm=arm):
                _ext.call_hip("cme_scan_tune", s[0].data_ptr(), s[1].data_ptr(), n, rows, arm, ws.data_ptr(),
                              _ext.stream_ptr(dev))
            fn(sets[0])
            torch.cuda.synchronize(dev)
            err = float(((sets[0][1].double() - ref).abs() / scale).max())
            timeout = int(_tw().value)
            _tw().value = 0
            ms = _cold_ms(dev, sets, fn)
            print(json.dumps({"bench": "scan_tune_cold", "rows": rows, "arm": arm, "ms_cold": round(ms, 4),
                              "GBps_8B": round(8 * n / ms / 1e6, 1), "max_rel_err": err, "timeout": timeout,
                              "ok": err < 1e-5 and not timeout}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
