#!/usr/bin/env python3
"""Small-grid heat variants (order 8, 1000 timesteps, random interior): the
LDS-resident tile passes against the pipelined passes, fp32 and fp64, to
check which one the solver's auto choice (models/heat2d_dist.py auto_kernel)
should take per dtype and size. One JSON line per (dtype, n, variant); every
variant is checked bitwise against the same-arithmetic single-step run first.

    python benchmarks/bench_small_variants.py [--n 500 1000 1500 2000]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[500, 1000, 1500, 2000])
    ap.add_argument("--dtype", nargs="+", default=["fp32", "fp64"])
    ap.add_argument("--order", type=int, nargs="+", default=[8])
    ap.add_argument("--iters", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", nargs="*", default=None, help="override the per-dtype variant list")
    args = ap.parse_args()
    import torch

    import cme213x  # noqa: F401
    from cme213x.models.heat2d import HeatGrid
    from cme213x.ops.stencil import heat_run
    from cme213x.utils.params import SimParams

    variants = {"fp32": ["pipe3_fma", "pipe4_fma", "tile3_fma", "tile4_fma", "pipe3", "pipe4", "tile3", "tile4"],
                "fp64": ["pipe3_fma", "pipe4_fma", "tile3_fma", "tile4_fma", "pipe4", "tile4"]}
    for dn, order in [(d, o) for o in args.order for d in args.dtype]:
        dt = torch.float32 if dn == "fp32" else torch.float64
        for n in args.n:
            p = SimParams(nx=n, ny=n, order=order, ic=3.0, bc=(0.0, 10.0, 0.0, 10.0))
            g = HeatGrid(p, dt, "cuda")
            B = g.B
            gen = torch.Generator(device="cuda").manual_seed(3)
            g.buf[:, B:B + n, B:B + n] = (torch.rand((n, n), generator=gen, device="cuda") * 10).to(dt)
            init = g.buf.clone()
            ref = {}
            for ar in ("stream", "fma"):
                a, b = init[0].clone(), init[1].clone()
                ref[ar] = heat_run(a, b, g.interior, order, g.xcfl, g.ycfl, 12, ar).clone()
            for v in args.variants or variants[dn]:
                a, b = init[0].clone(), init[1].clone()
                out = heat_run(a, b, g.interior, order, g.xcfl, g.ycfl, 12, v)
                ok = (bool(torch.equal(out, ref["fma" if v.endswith("_fma") else "stream"]))
                      if not v.endswith("_fast") else None)
                ts = []
                for _ in range(args.reps):
                    a, b = init[0].clone(), init[1].clone()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    heat_run(a, b, g.interior, order, g.xcfl, g.ycfl, args.iters, v)
                    e1.record()
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1))
                ts.sort()
                print(json.dumps({"bench": "small_variants", "dtype": dn, "order": order, "n": n, "variant": v, "bitwise": ok,
                                  "ms": round(ts[len(ts) // 2], 3)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
