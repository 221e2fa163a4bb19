#!/usr/bin/env python3
"""Dataflow launch diagnostics with the per-ticket trace: repeat a 2-pass
4096^2 run until a result differs from per-pass launches, then print, for
every wrong task, its pass-1 trace row and its pass-0 neighbours' rows
(ticket time, start, end in 100 MHz ticks relative to the first ticket; HW id)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import cme213x
    from cme213x.models.heat2d import HeatGrid
    from cme213x.ops.stencil import heat_flow, heat_run
    from cme213x.utils import tuning
    from cme213x.utils.params import SimParams

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    npass = 2
    p = SimParams(nx=n, ny=n, order=8, flavor="hw5")
    g = HeatGrid(p, torch.float32, "cuda")
    r = torch.rand(g.buf[0].shape, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3)) * 10
    g.buf[0].copy_(r)
    g.buf[1].copy_(r)
    xb, xe, yb, ye = g.interior
    with tuning.override(heat_flow=0):
        ref = heat_run(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, 4 * npass, "pipe4_fma").clone()
    for rep in range(20):
        a, b = g.buf[0].clone(), g.buf[1].clone()
        out, tr, tpp = heat_flow(a, b, g.interior, 8, g.xcfl, g.ycfl, npass, fma="fma", trace=True)
        diff = out != ref
        nbad = int(diff.sum())
        print(f"rep {rep}: bad {nbad}", flush=True)
        if not nbad:
            continue
        strips = -(-(xe - (xb & ~7)) // 480)
        nch = tpp // strips
        chunk = -(-(ye - yb) // nch)
        t0 = int(tr[:, 0].min())
        ys, xs = torch.nonzero(diff, as_tuple=True)
        cs = ((ys - yb) // chunk).cpu()
        ss = ((xs - (xb & ~7)) // 480).cpu()
        tasks = sorted(set(zip(cs.tolist(), ss.tolist())))
        print(f"tpp {tpp} strips {strips} nch {nch} chunk {chunk}; wrong tasks (chunk, strip): {tasks[:20]}", flush=True)
        for c, s in tasks[:6]:
            cnt = int(((cs == c) & (ss == s)).sum())
            t1 = tpp + c * strips + s
            row = tr[t1].tolist()
            print(f" task c{c} s{s}: {cnt} wrong cells; pass1 tk {row[0]-t0} start {row[1]-t0} end {row[2]-t0} hw {row[3]:#x}")
            for dc in (-1, 0, 1):
                for ds in (-1, 0, 1):
                    c2, s2 = c + dc, s + ds
                    if 0 <= c2 < nch and 0 <= s2 < strips:
                        q = tr[c2 * strips + s2].tolist()
                        print(f"   pass0 c{c2} s{s2}: tk {q[0]-t0} start {q[1]-t0} end {q[2]-t0} hw {q[3]:#x}"
                              f" {'<-- ends AFTER pass1 start' if q[2] > row[1] else ''}", flush=True)
        break


if __name__ == "__main__":
    main()
