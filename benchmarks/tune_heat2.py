#!/usr/bin/env python3
"""Sweep the two-step (temporal-blocking) heat kernel, order 8, 16384^2:
rows per register block (rb), waves-per-EU register cap (wpe; 1 = none),
exact vs FMA stencil, fp32 / fp64, default vs fixed row chunk. Interleaved
rounds in one process, median of 5; prints ms per TIMESTEP (a pass = 2)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import cme213x
    from cme213x import _ext
    from cme213x.models.heat2d import HeatGrid
    from cme213x.utils.params import SimParams

    _ext.proto(_ext.TUNE_PROTOS, "cme_heat_stream2_tune", "ppiiiiiiiddiiiip")
    n = int(os.environ.get("TUNE_N", "16384"))
    s = _ext.stream_ptr()
    for dtype in (torch.float32, torch.float64):
        p = SimParams(nx=n, ny=n, order=8)
        g = HeatGrid(p, dtype, "cuda")
        xb, xe, yb, ye = g.interior
        dt = 0 if dtype == torch.float32 else 1

        def run(cfg):
            rb, wpe, fma, chunk = cfg
            _ext.call_hip("cme_heat_stream2_tune", g.buf[0].data_ptr(), g.buf[1].data_ptr(), dt, g.pitch, g.gy,
                          xb, xe, yb, ye, g.xcfl, g.ycfl, chunk, rb, wpe, fma, s)

        chunks = [int(c) for c in os.environ.get("TUNE_CHUNKS", "0,128").split(",")]
        rbs = [int(c) for c in os.environ.get("TUNE_RB", "2,4,8").split(",")]
        wpes = [int(c) for c in os.environ.get("TUNE_WPE", "1,2,3,4").split(",")]
        cfgs = [(rb, wpe, fma, ch) for rb in rbs for wpe in wpes for fma in (0, 1) for ch in chunks]
        times = {c: [] for c in cfgs}
        for _ in range(5):
            for c in cfgs:
                run(c)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    run(c)
                e1.record()
                e1.synchronize()
                times[c].append(e0.elapsed_time(e1) / 5)
        for c in cfgs:
            ms = sorted(times[c])[2] / 2
            print(json.dumps({"dtype": str(dtype).split(".")[-1], "rb": c[0], "wpe": c[1], "fma": c[2],
                              "chunk": c[3], "ms_per_step": round(ms, 4)}), flush=True)
        del g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
