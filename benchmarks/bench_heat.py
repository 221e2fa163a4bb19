#!/usr/bin/env python3
"""Single-GPU heat-stencil sweep timing per kernel variant / order / dtype.

Prints one JSON line per configuration: ms per iteration, effective GB/s in
the reference's 24/40/72 B/pt convention, and minimum-traffic HBM GB/s.
Reference numbers are 4000^2, 10 iterations on Fermi.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[4000, 16384])
    ap.add_argument("--orders", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--variants", nargs="+", default=["global", "shared", "lds_nopad", "stream"])
    ap.add_argument("--dtypes", nargs="+", default=["fp32", "fp64"])
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import torch

    import cme213x
    from cme213x.models.heat2d import HeatGrid, bytes_per_point
    from cme213x.utils.params import SimParams

    for n in args.n:
        for dt in args.dtypes:
            dtype = torch.float32 if dt == "fp32" else torch.float64
            for order in args.orders:
                p = SimParams(nx=n, ny=n, order=order, iters=args.iters)
                g = HeatGrid(p, dtype, "cuda")
                for v in args.variants:
                    g.run(2, v)
                    torch.cuda.synchronize()
                    s = torch.cuda.Event(enable_timing=True)
                    e = torch.cuda.Event(enable_timing=True)
                    s.record()
                    g.run(args.iters, v)
                    e.record()
                    e.synchronize()
                    ms = s.elapsed_time(e) / args.iters
                    pts = n * n
                    esz = 4 if dtype == torch.float32 else 8
                    rec = {"n": n, "dtype": dt, "order": order, "variant": v, "ms_per_iter": round(ms, 4),
                           "eff_GBps": round(pts * bytes_per_point(order, dtype) / ms / 1e6, 1),
                           "hbm_GBps": round(pts * 2 * esz / ms / 1e6, 1)}
                    print(json.dumps(rec), flush=True)
                del g
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
