#!/usr/bin/env python3
"""Repeated runs of the two persistent heat launches against their per-pass
references (race hunting: distinct buffers, random data, several shapes).

    python benchmarks/stress_persistent.py [--reps 40]

Prints one JSON line: runs and mismatches per launch family."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=40)
    a = ap.parse_args()
    import torch

    from cme213x.models.heat2d import HeatGrid
    from cme213x.ops.stencil import heat_flow, heat_run, heat_tile_res
    from cme213x.utils import tuning
    from cme213x.utils.params import SimParams

    def grid(n, m, dtype, seed):
        g = HeatGrid(SimParams(nx=n, ny=m, order=8, flavor="hw5"), dtype, "cuda")
        gen = torch.Generator().manual_seed(seed)
        xb, xe, yb, ye = g.interior
        for k in (0, 1):  # distinct interiors: a stale read of either buffer shows
            g.buf[k, yb:ye, xb:xe] = (torch.rand((ye - yb, xe - xb), generator=gen, dtype=torch.float64) * 10).to(
                device="cuda", dtype=dtype)
        return g

    out = {"res_runs": 0, "res_bad": 0, "flow_runs": 0, "flow_bad": 0}
    for r in range(a.reps):
        for (n, m, ns, npass) in ((1000, 1000, 2, 7), (1000, 1000, 4, 5), (777, 1000, 2, 6)):
            g = grid(n, m, torch.float64, r)
            with tuning.override(tile_res=0):
                ref = heat_run(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, ns * npass,
                               "tile4" if ns == 4 else "tile2").clone()
            got = heat_tile_res(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, npass, ns=ns)
            out["res_runs"] += 1
            out["res_bad"] += int(not torch.equal(got, ref))
        g = grid(4096, 4096, torch.float32, 100 + r)
        with tuning.override(heat_flow=0):
            ref = heat_run(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, 12, "pipe4_fma").clone()
        got = heat_flow(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, 3, fma="fma")
        out["flow_runs"] += 1
        out["flow_bad"] += int(not torch.equal(got, ref))
    print(json.dumps(out), flush=True)
    return 0 if out["res_bad"] == 0 and out["flow_bad"] == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
