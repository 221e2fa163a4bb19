#!/usr/bin/env python3
"""One N-GPU rank's share as ONE region: the 16384/N x 16384 stripe of a
strong-scaled 16384^2 run computed as a single grid (Dirichlet rows where the
rank has halos), fast arithmetic, four steps per pass -- the schedule a rank
would run if its 16-row border strips were folded into the first / last
chunk of every strip instead of separate gated regions. Compare with
bench_dist_rank.py --kernel pipe --tblock 4 --arith fast (three regions per
pass: deep interior + two border strips).

    python benchmarks/bench_rank_shape.py [--world 1 2 4 8] [--steps 100]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--world", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variant", default="pipe4_fast")
    args = ap.parse_args()
    import torch

    import cme213x  # noqa: F401
    from cme213x.models.heat2d import HeatGrid
    from cme213x.ops.stencil import heat_run
    from cme213x.utils.params import SimParams

    base = None
    for w in args.world:
        p = SimParams(nx=args.n, ny=args.n // w, order=8, ic=5.0, bc=(0.0, 10.0, 0.0, 10.0), flavor="hw5")
        g = HeatGrid(p, torch.float32, "cuda")
        gen = torch.Generator(device="cuda").manual_seed(7)
        B = g.B
        g.buf[:, B:B + p.ny, B:B + p.nx] = torch.rand((p.ny, p.nx), generator=gen, device="cuda") * 10.0
        a, b = g.buf[0], g.buf[1]

        def run(k):
            heat_run(a, b, g.interior, 8, g.xcfl, g.ycfl, k, args.variant)

        run(40)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(args.steps)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / args.steps)
        ms = sorted(ts)[len(ts) // 2]
        base = base or ms * w
        print(json.dumps({"world": w, "rows": p.ny, "variant": args.variant, "ms_per_step": round(ms, 4),
                          "share_eff": round(base / (ms * w), 3)}), flush=True)
        del g, a, b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
