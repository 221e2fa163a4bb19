#!/usr/bin/env python3
"""Tile shape / workgroup size sweep of the LDS-resident tile pass
(csrc/hip/heat_tile.h) on the hw5 shapes: fp64, order 8, 1000 timesteps.
Needs the tuning library (CME_TUNE=1: cme_heat_tile_tune). Every arm is
checked bit for bit against single steps first.

    python benchmarks/tune_tile.py [--n 1000 2000] [--ns 2 3 4] [--cfg 0 1 2 3 4 5 6 7]"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[1000, 2000])
    ap.add_argument("--ns", type=int, nargs="+", default=[1, 2, 3, 4])
    ap.add_argument("--cfg", type=int, nargs="+", default=list(range(8)))
    ap.add_argument("--fma", type=int, nargs="+", default=[0, 1])
    ap.add_argument("--iters", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch

    import cme213x  # noqa: F401
    from cme213x import _ext
    from cme213x.models.heat2d import HeatGrid
    from cme213x.ops.stencil import heat_run
    from cme213x.utils.params import SimParams

    _ext.proto(_ext.TUNE_PROTOS, "cme_heat_tile_tune", "ppiiiiiiiiiiddpp")
    for n in args.n:
        p = SimParams(nx=n, ny=n, order=8, ic=3.0, bc=(0.0, 10.0, 0.0, 10.0))
        g = HeatGrid(p, torch.float64, "cuda")
        B = g.B
        gen = torch.Generator(device="cuda").manual_seed(2)
        g.buf[:, B:B + n, B:B + n] = torch.rand((n, n), generator=gen, device="cuda", dtype=torch.float64) * 10
        init = g.buf.clone()
        ref = {}
        for fma in args.fma:
            a, b = init[0].clone(), init[1].clone()
            ref[fma] = heat_run(a, b, g.interior, 8, g.xcfl, g.ycfl, 9, "fma" if fma else "stream").clone()
        fin = ctypes.c_int(0)

        def run(ns, fma, cfg, iters):
            _ext.call_hip("cme_heat_tile_tune", g.buf[0].data_ptr(), g.buf[1].data_ptr(), g.pitch, g.gy,
                          *g.interior, ns, fma, cfg, iters, g.xcfl, g.ycfl, ctypes.addressof(fin),
                          _ext.stream_ptr())
            return g.buf[fin.value]

        for ns in args.ns:
            for fma in args.fma:
                for cfg in args.cfg:
                    g.buf.copy_(init)
                    try:
                        out = run(ns, fma, cfg, 9)
                    except RuntimeError:
                        continue  # arm not compiled for this ns
                    torch.cuda.synchronize()
                    ok = bool(torch.equal(out, ref[fma]))
                    ts = []
                    for _ in range(args.reps):
                        g.buf.copy_(init)
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        run(ns, fma, cfg, args.iters)
                        e1.record()
                        e1.synchronize()
                        ts.append(e0.elapsed_time(e1))
                    ts.sort()
                    print(json.dumps({"bench": "tile_tune", "n": n, "ns": ns, "fma": fma, "cfg": cfg, "bitwise": ok,
                                      "ms_total": round(ts[len(ts) // 2], 3),
                                      "us_per_step": round(ts[len(ts) // 2] * 1e3 / args.iters, 3)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
