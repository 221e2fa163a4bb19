#!/usr/bin/env python3
"""Per-pass pipelined launches (no dataflow) with explicit chunk heights
against the default chunk rule, on a field whose two buffers differ (so a
task that reads the wrong buffer or overlaps a neighbour shows)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import cme213x
    from cme213x.models.heat2d import HeatGrid
    from cme213x.ops.stencil import heat_run
    from cme213x.utils import tuning
    from cme213x.utils.params import SimParams

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    p = SimParams(nx=n, ny=n, order=8, flavor="hw5")
    g = HeatGrid(p, torch.float32, "cuda")
    gen = torch.Generator(device="cuda").manual_seed(3)
    g.buf[0].copy_(torch.rand(g.buf[0].shape, device="cuda", generator=gen) * 10)
    g.buf[1].copy_(torch.rand(g.buf[0].shape, device="cuda", generator=gen) * 10)
    # the BC ring must be the same in both buffers: copy buffer 0's outside the interior
    xb, xe, yb, ye = g.interior
    keep = g.buf[1, yb:ye, xb:xe].clone()
    g.buf[1].copy_(g.buf[0])
    g.buf[1, yb:ye, xb:xe] = keep
    with tuning.override(heat_flow=0):
        ref = heat_run(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, 8, "pipe4_fma").clone()
        for chunk in (16, 18, 20, 26, 50, 74):
            for rep in range(3):
                out = heat_run(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, 8, "pipe4_fma",
                               chunk)
                torch.cuda.synchronize()
                print(f"per-pass chunk {chunk} rep {rep}: bad {int((out != ref).sum())}", flush=True)
        for per_cu in (0, 2, 4, 6, 8):
            with tuning.override(heat_flow=1, flow_per_cu=per_cu):
                for rep in range(3):
                    out = heat_run(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, 8, "pipe4_fma")
                    torch.cuda.synchronize()
                    print(f"flow per_cu {per_cu} rep {rep}: bad {int((out != ref).sum())}", flush=True)


if __name__ == "__main__":
    main()
