#!/usr/bin/env python3
"""Diagnostics of the dataflow launch (csrc/hip/heat_flow.hip): npass = 1..4
on a grid (default 4096^2) against per-pass launches; for a mismatch, where
the wrong cells sit relative to the task grid (strips of 480 columns, chunks
of `chunk` rows), and the control words / give-up records."""
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

    n, m = (int(a) for a in (sys.argv[1:3] if len(sys.argv) > 2 else (4096, 4096)))
    arith = sys.argv[3] if len(sys.argv) > 3 else "fma"
    knobs = dict(kv.split("=") for kv in sys.argv[4:])
    p = SimParams(nx=n, ny=m, order=8, flavor="hw5")
    g = HeatGrid(p, torch.float32, "cuda")
    gen = torch.Generator(device="cuda").manual_seed(3)
    g.buf[0].copy_(torch.rand(g.buf[0].shape, device="cuda", generator=gen) * 10)
    g.buf[1].copy_(torch.rand(g.buf[0].shape, device="cuda", generator=gen) * 10)
    xb, xe, yb, ye = g.interior
    keep = g.buf[1, yb:ye, xb:xe].clone()  # same BC ring in both buffers, different interiors
    g.buf[1].copy_(g.buf[0])
    g.buf[1, yb:ye, xb:xe] = keep
    rows, pitch = g.buf[0].shape
    var = {"fma": "pipe4_fma", "exact": "pipe4", "fast": "pipe4_fast"}[arith]
    code = {"exact": 0, "fma": 1, "fast": 2}[arith]
    modes = [int(x) for x in knobs.pop("modes", "0").split(",")]
    passes = [int(x) for x in knobs.pop("passes", "1,2,3,4,6").split(",")]
    reps = int(knobs.pop("reps", "3"))
    if knobs.pop("seq", "0") == "1":
        # E1: npass single-pass flow launches in sequence (kernel boundaries between passes)
        for npass in passes:
            with tuning.override(heat_flow=0):
                ref = heat_run(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, 4 * npass,
                               var).clone()
            for rep in range(reps):
                bufs = [g.buf[0].clone(), g.buf[1].clone()]
                for q in range(npass):
                    src, dst = bufs[q % 2], bufs[(q + 1) % 2]
                    _ext.call_hip("cme_heat_flow_f32", src.data_ptr(), dst.data_ptr(), pitch, rows, xb, xe, yb, ye,
                                  8, code, 4, g.xcfl, g.ycfl, 1, _ext.stream_ptr(src.device))
                torch.cuda.synchronize()
                out = bufs[npass % 2]
                print(f"seq npass {npass} rep {rep}: bad {int((out != ref).sum())}", flush=True)
    for mode in modes:
      knobs["flow_mode"] = mode
      print(f"== flow_mode {mode}", flush=True)
      for npass in passes:
          with tuning.override(heat_flow=0):
              ref = heat_run(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, 4 * npass, var).clone()
          bad_runs = 0
          for rep in range(reps):
              a, b = g.buf[0].clone(), g.buf[1].clone()
              with tuning.override(flow_spins=1 << 20, **{k: int(v) for k, v in knobs.items()}):
                  t0 = time.time()
                  _ext.call_hip("cme_heat_flow_f32", a.data_ptr(), b.data_ptr(), pitch, rows, xb, xe, yb, ye, 8, code,
                                4, g.xcfl, g.ycfl, npass, _ext.stream_ptr(a.device))
                  torch.cuda.synchronize()
                  dt = time.time() - t0
              out = b if npass % 2 else a
              words = (ctypes.c_uint * 8)()
              _ext.call_hip("cme_heat_flow_debug", ctypes.addressof(words), 8)
              to = flow_timed_out(reset=True)
              diff = (out != ref)
              nbad = int(diff.sum())
              line = f"npass {npass} rep {rep}: {dt * 1e3:.2f} ms timed_out {to} bad {nbad} ctl {list(words[:4])}"
              if nbad:
                  bad_runs += 1
                  ys, xs = torch.nonzero(diff, as_tuple=True)
                  tpp = words[3]
                  strips = -(-(xe - (xb & ~7)) // 480)
                  nch = tpp // strips
                  chunk = -(-(ye - yb) // nch)
                  ry = (ys - yb).cpu()
                  rx = (xs - (xb & ~7)).cpu()
                  line += (f" tpp {tpp} strips {strips} nch {nch} chunk~{chunk}"
                           f" rows[{int(ys.min())},{int(ys.max())}] cols[{int(xs.min())},{int(xs.max())}]"
                           f" row-in-chunk hist {torch.bincount((ry % chunk).clamp(max=chunk - 1) // max(1, chunk // 8)).tolist()}"
                           f" col-in-strip hist {torch.bincount((rx % 480) // 60).tolist()}"
                           f" maxabs {float((out - ref).abs().max()):.3g}")
              print(line, flush=True)


if __name__ == "__main__":
    main()
