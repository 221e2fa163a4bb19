#!/usr/bin/env python3
"""Per-pass timeline of the resident-tile run (csrc/hip/heat_tile_res.hip).

    python benchmarks/trace_tile_res.py [--n 1000] [--passes 500] [--ns 2] [--fma] [--out FILE]

One traced launch of `passes` exchanges (2 steps each by default: 1000 steps
at the default) on the hw5 grid, fp64 order 8. Each (pass, tile) carries five
wall-clock stamps (100 MHz): pass start, inner cone done, halo in, outer ring
done (ring stores issued), ring published (during the next pass).
Prints one JSON line: medians over tiles and passes of each phase (us), the
halo wait (inner done -> halo in), the per-pass span, and the whole launch
from the first stamp to the last; `--out` appends it to a JSONL file."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--passes", type=int, default=500)
    ap.add_argument("--ns", type=int, default=2)
    ap.add_argument("--fma", action="store_true")
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--out", default=None)
    ap.add_argument("--tune", nargs="*", default=[], help="tuning knobs name=value, e.g. tile_res_minr=2")
    a = ap.parse_args()

    import torch

    from cme213x.models.heat2d import HeatGrid
    from cme213x.ops.stencil import heat_tile_res
    from cme213x.utils.params import SimParams

    from cme213x.utils import tuning

    knobs = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in a.tune}
    for k, v in knobs.items():
        tuning.set(k, v)
    dt = torch.float32 if a.fp32 else torch.float64
    p = SimParams(nx=a.n, ny=a.n, order=8, ic=3.0, bc=(0.0, 10.0, 0.0, 10.0), flavor="hw5")
    g = HeatGrid(p, dt, "cuda")
    args = (g.interior, 8, g.xcfl, g.ycfl)
    heat_tile_res(g.buf[0], g.buf[1], *args, 4, ns=a.ns, fma=a.fma)  # warm-up
    # untraced timing of the same launch
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        heat_tile_res(g.buf[0], g.buf[1], *args, a.passes, ns=a.ns, fma=a.fma)
    untraced_ms = (time.perf_counter() - t0) / reps * 1e3
    _, tr, ntiles = heat_tile_res(g.buf[0], g.buf[1], *args, a.passes, ns=a.ns, fma=a.fma, trace=True)
    t = tr.view(a.passes, ntiles, 5).double() / 100.0  # us
    med = lambda x: round(float(x.median()), 3)  # noqa: E731
    rec = {
        "bench": "trace_tile_res", "n": a.n, "dtype": "fp32" if a.fp32 else "fp64", "ns": a.ns, "fma": a.fma,
        "passes": a.passes, "steps": a.passes * a.ns, "tiles": ntiles, "tune": knobs,
        "inner_us": med(t[..., 1] - t[..., 0]),
        "halo_wait_and_load_us": med(t[..., 2] - t[..., 1]),
        "outer_and_store_us": med(t[..., 3] - t[..., 2]),
        "publish_after_next_start_us": med(t[:-1, :, 4] - t[1:, :, 0]) if a.passes > 1 else None,
        "pass_span_us": med(t[1:, :, 0] - t[:-1, :, 0]) if a.passes > 1 else None,
        "launch_span_ms": round(float(t[..., 4].max() - t[..., 0].min()) / 1e3, 4),
        "untraced_call_ms": round(untraced_ms, 4),
        "halo_wait_p90_us": round(float((t[..., 2] - t[..., 1]).flatten().quantile(0.9)), 3),
    }
    line = json.dumps(rec)
    print(line, flush=True)
    if a.out:
        with open(a.out, "a") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
