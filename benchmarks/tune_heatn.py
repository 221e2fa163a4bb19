#!/usr/bin/env python3
"""Sweep the NS-step temporal-blocking heat kernels (order 8, fp32, FMA,
16384^2): steps per HBM pass ns (2 = the stream2 kernel, 3 / 4 = streamN),
rows per register block rb, prefetch depth pd (streamN), row chunk per wave
(0 = default rule).
Interleaved rounds in one process, median of 5; prints ms per TIMESTEP.

    TUNE_NS=3,4 TUNE_RB=1,2 TUNE_CHUNKS=0,64,128 python benchmarks/tune_heatn.py
"""
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
    p = SimParams(nx=n, ny=n, order=8)
    g = HeatGrid(p, torch.float32, "cuda")
    xb, xe, yb, ye = g.interior

    def run(cfg):
        ns, rb, pd, chunk = cfg
        if ns == 2:
            _ext.call_hip("cme_heat_stream2_tune", g.buf[0].data_ptr(), g.buf[1].data_ptr(), 0, g.pitch, g.gy,
                          xb, xe, yb, ye, g.xcfl, g.ycfl, chunk, rb, 1, 1, s)
        else:
            _ext.call_hip("cme_heat_streamn_tune", g.buf[0].data_ptr(), g.buf[1].data_ptr(), g.pitch, g.gy,
                          xb, xe, yb, ye, g.xcfl, g.ycfl, chunk, rb, ns, pd, s)

    nss = [int(c) for c in os.environ.get("TUNE_NS", "2,3,4").split(",")]
    rbs = [int(c) for c in os.environ.get("TUNE_RB", "1,2,4").split(",")]
    chunks = [int(c) for c in os.environ.get("TUNE_CHUNKS", "0,64,96,128,192,256").split(",")]
    pds = [int(c) for c in os.environ.get("TUNE_PD", "1,2").split(",")]
    cfgs = []
    for ns in nss:
        for rb in rbs:
            if ns == 2 and rb == 1:
                continue  # stream2 tune entry has rb 2/4/8
            for pd in (pds if ns > 2 else [1]):
                for ch in chunks:
                    cfgs.append((ns, rb, pd, ch))
    times = {c: [] for c in cfgs}
    for _ in range(5):
        for c in cfgs:
            run(c)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(4):
                run(c)
            e1.record()
            e1.synchronize()
            times[c].append(e0.elapsed_time(e1) / 4)
    for c in sorted(cfgs, key=lambda c: sorted(times[c])[2] / c[0]):
        ms = sorted(times[c])[2] / c[0]
        print(json.dumps({"n": n, "ns": c[0], "rb": c[1], "pd": c[2], "chunk": c[3],
                          "ms_per_step": round(ms, 4),
                          "hbm_TBps": round(n * n * 8 / c[0] / (ms * 1e-3) / 1e12, 2)}), flush=True)


if __name__ == "__main__":
    main()
