#!/usr/bin/env python3
"""Data dependence of the flagship pass: ms per timestep of the 16384^2
order-8 fp32 grid from the reference's uniform IC (5.0) and from a
random-init field (uniform(0, 10)), per pass variant, in windows over a long
run (the pass is power-bound: the clock a window gets depends on the data's
switching activity and on how long the GPU has been busy).

    python benchmarks/bench_ic.py [--variants pipe4_fma,pipe5_fma] [--windows 10] [--steps 40]

One JSON line per (variant, data): per-window ms/step, the median, and
bitwise agreement of every variant with pipe4_fma's result where the steps
match."""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--variants", default="pipe4_fma,pipe5_fma,pipe6_fma,pipe3_fma")
    ap.add_argument("--data", default="uniform,random")
    ap.add_argument("--windows", type=int, default=8)
    ap.add_argument("--steps", type=int, default=60, help="timesteps per window (a multiple of 60 suits 3/4/5/6)")
    ap.add_argument("--spin", type=float, default=0.5)
    ap.add_argument("--tune", nargs="*", default=[],
                    help="tuning knobs name=value[/value...] (cme213x.utils.tuning); one run per value combination")
    args = ap.parse_args()
    import torch

    import cme213x  # noqa: F401
    from cme213x.models.heat2d import HeatGrid
    from cme213x.ops.stencil import heat_run
    from cme213x.utils.params import SimParams

    p = SimParams(nx=args.n, ny=args.n, order=8, ic=5.0, bc=(0.0, 10.0, 0.0, 10.0))
    g = HeatGrid(p, torch.float32, "cuda")
    H = g.H
    init = {}
    init["uniform"] = g.buf.clone()
    gen = torch.Generator(device="cuda").manual_seed(1234)
    r = g.buf.clone()
    r[:, H:H + g.ny, H:H + g.nx] = torch.rand((g.ny, g.nx), generator=gen, device="cuda") * 10.0
    init["random"] = r

    def run(v, k):
        a, b = g.buf[g.cur], g.buf[1 - g.cur]
        out = heat_run(a, b, g.interior, g.order, g.xcfl, g.ycfl, k, v)
        g.cur = g.cur if out is a else 1 - g.cur

    from cme213x.utils import tuning
    import itertools

    knob_vals = [[(kv.split("=")[0], int(v)) for v in kv.split("=")[1].split("/")] for kv in args.tune]
    combos = list(itertools.product(*knob_vals)) if knob_vals else [()]
    variants = args.variants.split(",")
    t_end = time.perf_counter() + args.spin
    while time.perf_counter() < t_end:
        for v in variants:
            run(v, 12)
        torch.cuda.synchronize()
    for combo in combos:
        for k, v in combo:
            tuning.set(k, v)
        knobs = {k: v for k, v in combo}
        finals = {}
        for data in args.data.split(","):
            for v in variants:
                g.buf.copy_(init[data])
                g.cur = 0
                run(v, 12)  # warm-up on this data
                torch.cuda.synchronize()
                g.buf.copy_(init[data])
                g.cur = 0
                win = []
                for _ in range(args.windows):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    run(v, args.steps)
                    e1.record()
                    e1.synchronize()
                    win.append(e0.elapsed_time(e1) / args.steps)
                finals[(data, v)] = g.buf[g.cur].clone()
                same = None
                if v != "pipe4_fma" and (data, "pipe4_fma") in finals:
                    same = bool(torch.equal(finals[(data, v)], finals[(data, "pipe4_fma")]))
                print(json.dumps({"bench": "heat_ic", "n": args.n, "variant": v, "data": data, "tune": knobs,
                                  "ms_per_step_windows": [round(x, 4) for x in win],
                                  "ms_per_step_median": round(statistics.median(win), 4),
                                  "ms_per_step_first": round(win[0], 4), "bitwise_vs_pipe4": same}), flush=True)
        for k, _ in combo:
            tuning.reset(k)
    return 0


if __name__ == "__main__":
    sys.exit(main())
