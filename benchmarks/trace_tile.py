#!/usr/bin/env python3
"""Where a tile pass's time goes (hw5 1000^2 / 2000^2, fp64, order 8): two
back-to-back ns-step passes of the production tile shape (64 x 64, 1024
threads) with per-workgroup wall-clock stamps (csrc/hip/heat_tile.h trace:
entry, after the global->LDS load, after every step, after the stores).
Prints one JSON line per pass: median / p90 phase durations over the
workgroups, the pass span (first entry to last store) and the idle gap
between the two passes. Needs the tuning library (make TUNE=1).

    python benchmarks/trace_tile.py [--n 1000] [--ns 4] [--fma 0]"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[1000])
    ap.add_argument("--ns", type=int, default=4)
    ap.add_argument("--fma", type=int, nargs="+", default=[0, 1])
    ap.add_argument("--nts", type=int, nargs="+", default=[0], help="1: non-temporal output stores")
    args = ap.parse_args()
    import numpy as np
    import torch

    import cme213x  # noqa: F401
    from cme213x import _ext
    from cme213x.models.heat2d import HeatGrid
    from cme213x.utils.params import SimParams

    _ext.proto(_ext.TUNE_PROTOS, "cme_heat_tile_trace", "ppiiiiiiiiiddpp")
    mhz = 100.0  # wall_clock64 rate on gfx950
    for n in args.n:
        p = SimParams(nx=n, ny=n, order=8, ic=3.0, bc=(0.0, 10.0, 0.0, 10.0))
        g = HeatGrid(p, torch.float64, "cuda")
        B = g.B
        gen = torch.Generator(device="cuda").manual_seed(2)
        g.buf[:, B:B + n, B:B + n] = torch.rand((n, n), generator=gen, device="cuda", dtype=torch.float64) * 10
        tiles = ((n + 63) // 64) ** 2
        tr = [torch.zeros(8 * tiles, dtype=torch.int64, device="cuda") for _ in range(2)]
        for fma, nts in [(f, m) for f in args.fma for m in args.nts]:
            def one(k, t):
                _ext.call_hip("cme_heat_tile_trace", g.buf[k].data_ptr(), g.buf[1 - k].data_ptr(), g.pitch, g.gy,
                              *g.interior, args.ns, fma, nts, g.xcfl, g.ycfl, t.data_ptr() if t is not None else None,
                              _ext.stream_ptr())

            t_end = time.perf_counter() + 1.0  # clock ramp
            while time.perf_counter() < t_end:
                for i in range(50):
                    one(i & 1, None)
                torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(200):
                one(i & 1, None)
            e1.record()
            e1.synchronize()
            us_per_pass = e0.elapsed_time(e1) * 1e3 / 200
            one(0, tr[0])
            one(1, tr[1])
            torch.cuda.synchronize()
            a = [t.view(tiles, 8).cpu().numpy().astype(np.int64) for t in tr]
            ns = args.ns
            for pi, x in enumerate(a):
                ph = {"load": x[:, 1] - x[:, 0]}
                for s in range(1, ns + 1):
                    ph[f"step{s}"] = x[:, 1 + s] - x[:, s]
                ph["store"] = x[:, ns + 2] - x[:, ns + 1]
                ph["workgroup"] = x[:, ns + 2] - x[:, 0]
                rec = {"bench": "tile_trace", "n": n, "ns": ns, "fma": fma, "nts": nts, "pass": pi, "tiles": tiles,
                       "span_us": round(float(x[:, ns + 2].max() - x[:, 0].min()) / mhz, 2),
                       "start_spread_us": round(float(x[:, 0].max() - x[:, 0].min()) / mhz, 2)}
                for k, v in ph.items():
                    rec[f"{k}_median_us"] = round(float(np.median(v)) / mhz, 2)
                    rec[f"{k}_p90_us"] = round(float(np.percentile(v, 90)) / mhz, 2)
                rec["us_per_pass_200"] = round(us_per_pass, 2)
                if pi == 1:
                    rec["gap_after_prev_us"] = round(float(x[:, 0].min() - a[0][:, ns + 2].max()) / mhz, 2)
                print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
