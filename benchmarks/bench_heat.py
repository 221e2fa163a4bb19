#!/usr/bin/env python3
"""Single-GPU heat-stencil sweep timing per kernel variant / order / dtype.

Prints one JSON line per configuration: ms per iteration, effective GB/s in
the reference's 24/40/72 B/pt convention, and minimum-traffic HBM GB/s.
Reference numbers are 4000^2, 10 iterations on Fermi.

Each variant is warmed with a few full passes (so a multi-step kernel's first
launch is not timed) and timed as the median of --reps event-timed runs of
--iters iterations. --graph also times the same run recorded once as a
hipGraph and replayed (utils/graphs.py): small grids are launch-bound, and
the graph removes the per-launch gaps (the reference's hw5 shape, 1000^2 x
1000 iterations, is 333 three-step passes of ~10 us each).
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
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--graph", action="store_true", help="also time the run replayed from a hipGraph")
    args = ap.parse_args()
    import torch

    import cme213x
    from cme213x.models.heat2d import HeatGrid, bytes_per_point
    from cme213x.utils.graphs import GraphRunner
    from cme213x.utils.params import SimParams

    for n in args.n:
        for dt in args.dtypes:
            dtype = torch.float32 if dt == "fp32" else torch.float64
            for order in args.orders:
                p = SimParams(nx=n, ny=n, order=order, iters=args.iters)
                g = HeatGrid(p, dtype, "cuda")
                for v in args.variants:
                    g.run(16, v)  # every kernel of this variant launched once (full passes + tails)
                    torch.cuda.synchronize()

                    def timed(fn):
                        ts = []
                        for _ in range(args.reps):
                            s = torch.cuda.Event(enable_timing=True)
                            e = torch.cuda.Event(enable_timing=True)
                            s.record()
                            fn()
                            e.record()
                            e.synchronize()
                            ts.append(s.elapsed_time(e))
                        return sorted(ts)[len(ts) // 2] / args.iters

                    ms = timed(lambda: g.run(args.iters, v))
                    pts = n * n
                    esz = 4 if dtype == torch.float32 else 8
                    rec = {"n": n, "dtype": dt, "order": order, "variant": v, "iters": args.iters,
                           "ms_per_iter": round(ms, 5), "total_ms": round(ms * args.iters, 3),
                           "eff_GBps": round(pts * bytes_per_point(order, dtype) / ms / 1e6, 1),
                           "hbm_GBps": round(pts * 2 * esz / ms / 1e6, 1)}
                    if args.graph:
                        cur0 = g.cur
                        runner = GraphRunner(lambda: g.run(args.iters, v), warmup=0)
                        g.cur = cur0
                        gms = timed(runner)
                        rec.update({"graph_ms_per_iter": round(gms, 5), "graph_total_ms": round(gms * args.iters, 3),
                                    "graph_eff_GBps": round(pts * bytes_per_point(order, dtype) / gms / 1e6, 1)})
                        del runner
                    print(json.dumps(rec), flush=True)
                del g
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
