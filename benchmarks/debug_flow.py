#!/usr/bin/env python3
"""Diagnostics of the dataflow launch (csrc/hip/heat_flow.hip): one and two
passes on a small grid with a short spin bound; prints the outcome, the
control words and any give-up records (ticket, pass, strip, chunk, the
completion words the waiting lanes saw)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import cme213x
    from cme213x import _ext
    from cme213x.models.heat2d import HeatGrid
    from cme213x.ops.stencil import flow_timed_out, heat_run
    from cme213x.utils import tuning
    from cme213x.utils.params import SimParams

    n, m = (int(a) for a in (sys.argv[1:3] if len(sys.argv) > 2 else (1500, 1100)))
    p = SimParams(nx=n, ny=m, order=8, flavor="hw5")
    g = HeatGrid(p, torch.float32, "cuda")
    r = torch.rand(g.buf[0].shape, device="cuda") * 10
    g.buf[0].copy_(r)
    g.buf[1].copy_(r)
    xb, xe, yb, ye = g.interior
    rows, pitch = g.buf[0].shape
    for npass in (1, 2, 3):
        with tuning.override(heat_flow=0):
            ref = heat_run(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, 4 * npass,
                           "pipe4_fma").clone()
        a, b = g.buf[0].clone(), g.buf[1].clone()
        with tuning.override(flow_spins=1 << 16):
            t0 = time.time()
            _ext.call_hip("cme_heat_flow_f32", a.data_ptr(), b.data_ptr(), pitch, rows, xb, xe, yb, ye, 8, 1, 4,
                          g.xcfl, g.ycfl, npass, _ext.stream_ptr(a.device))
            torch.cuda.synchronize()
            dt = time.time() - t0
        out = b if npass % 2 else a
        words = (ctypes.c_uint * 8192)()
        _ext.call_hip("cme_heat_flow_debug", ctypes.addressof(words), 8192)
        to = flow_timed_out(reset=True)
        print(f"npass {npass}: {dt * 1e3:.1f} ms timed_out {to} equal {bool(torch.equal(out, ref))} "
              f"ctl {list(words[:4])}", flush=True)
        if to:
            ng = min(64, words[2])
            # completion words follow ctl; records after tpp words: find tpp from the first record's layout
            print("done[0:64]", list(words[4:68]), flush=True)
            tpp = words[3]
            for k in range(ng):
                rec = list(words[4 + tpp + 16 * k: 4 + tpp + 16 * k + 13])
                print("giveup", rec, flush=True)
            break


if __name__ == "__main__":
    main()
