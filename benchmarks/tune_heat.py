#!/usr/bin/env python3
"""Sweep the streaming heat kernel's tuning space (order 8, fp32, 16384^2) and
calibrate against a 16-B copy of the same byte count. One process, interleaved
rounds (median reported)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import cme213x
    from cme213x import _ext
    from cme213x.models.heat2d import HeatGrid
    from cme213x.ops.elementwise import copy_
    from cme213x.utils.params import SimParams

    _ext.proto(_ext.TUNE_PROTOS, "cme_heat_stream_tune_f32", "ppiiiiiiffiiiip")
    n = int(os.environ.get("TUNE_N", "16384"))
    p = SimParams(nx=n, ny=n, order=8)
    g = HeatGrid(p, torch.float32, "cuda")
    s = _ext.stream_ptr()
    xb, xe, yb, ye = g.interior

    def run(cfg):
        rb, wpb, nt, chunk = cfg
        a, b = g.buf[0], g.buf[1]
        _ext.call_hip("cme_heat_stream_tune_f32", a.data_ptr(), b.data_ptr(), g.pitch, g.gy, xb, xe, yb, ye,
                      g.xcfl, g.ycfl, rb, wpb, nt, chunk, s)

    cfgs = [(rb, wpb, nt, ch) for rb in (4, 8, 12) for wpb in (4, 8, 16) for nt in (0, 1) for ch in (0, 1024)]
    times = {c: [] for c in cfgs}
    src = g.buf[0]
    dst = torch.empty_like(src)
    copy_t = []
    for rnd in range(5):
        for c in cfgs:
            run(c)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                run(c)
            e1.record()
            e1.synchronize()
            times[c].append(e0.elapsed_time(e1) / 5)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            copy_(dst, src)
        e1.record()
        e1.synchronize()
        copy_t.append(e0.elapsed_time(e1) / 5)
    pts = n * n
    copy_ms = sorted(copy_t)[2]
    print(json.dumps({"copy_ms": copy_ms, "copy_GBps": 2 * src.numel() * 4 / copy_ms / 1e6}))
    for c in cfgs:
        ms = sorted(times[c])[2]
        print(json.dumps({"rb": c[0], "wpb": c[1], "nt": c[2], "chunk": c[3], "ms": round(ms, 4),
                          "hbm_GBps": round(pts * 8 / ms / 1e6, 1)}))


if __name__ == "__main__":
    main()
