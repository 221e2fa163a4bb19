#!/usr/bin/env python3
"""Wave-pipelined NS-step heat pass (heat_pipe.hip) vs the streamN pass
(heat2d.hip) on the shapes one rank of an N-GPU strong-scaled 16384^2 run
computes: a full-width region of H rows (H = 16384 / N), order 8, fp32, FMA.

Every arm is first checked bit for bit against the streamN pass with the
same steps per pass on random data; then interleaved rounds, median of 5,
ms per TIMESTEP.

    TUNE_H=16384,2048 TUNE_NS=3,4 TUNE_RB=2,4,8 TUNE_PD=1,2 TUNE_PERCU=1,2,4,8 \\
        python benchmarks/tune_heat_pipe.py

TUNE_PD codes: 1 / 2 input prefetch depth; 11 depth 1 + non-temporal stores;
21 / 41 the same with two / four waves per timestep role (RB 4); 81 wide
lanes (8 columns per lane, RB 2 or 4). Combinations that are not compiled
are skipped. TUNE_SPIN
seconds of clock ramp first, TUNE_REPS launches per sample.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ints(name, default):
    return [int(c) for c in os.environ.get(name, default).split(",") if c]


def main():
    import torch

    import cme213x  # noqa: F401
    from cme213x import _ext
    from cme213x.models.heat2d import HeatGrid
    from cme213x.utils.params import SimParams

    _ext.proto(_ext.TUNE_PROTOS, "cme_heat_pipe_tune", "ppiiiiiiffiiiiip")
    n = int(os.environ.get("TUNE_N", "16384"))
    s = _ext.stream_ptr()
    p = SimParams(nx=n, ny=n, order=8)
    g = HeatGrid(p, torch.float32, "cuda")
    gen = torch.Generator(device="cuda").manual_seed(1)
    g.buf[0].copy_(torch.rand(g.buf[0].shape, device="cuda", generator=gen) * 10)
    if os.environ.get("TUNE_DATA", "rand") == "const":  # bench.py's field (IC 5.0): lower switching power
        g.buf[0].fill_(5.0)
    xb, xe, yb0, ye0 = g.interior

    def streamn(ns, H, out):
        yb = yb0 + (ye0 - yb0 - H) // 2
        rb, pd = (4, 1) if ns == 3 else (2, 21)
        _ext.call_hip("cme_heat_streamn_tune", g.buf[0].data_ptr(), out.data_ptr(), g.pitch, g.gy,
                      xb, xe, yb, yb + H, g.xcfl, g.ycfl, 0, rb, ns, pd, s)

    def pipe(cfg, H, out):
        ns, rb, pd, per_cu, chunk = cfg
        yb = yb0 + (ye0 - yb0 - H) // 2
        _ext.call_hip("cme_heat_pipe_tune", g.buf[0].data_ptr(), out.data_ptr(), g.pitch, g.gy,
                      xb, xe, yb, yb + H, g.xcfl, g.ycfl, chunk, rb, ns, pd, per_cu, s)

    hs = ints("TUNE_H", "16384,8192,4096,2048")
    nss = ints("TUNE_NS", "3,4")
    cfgs = []
    for ns in nss:
        for rb in ints("TUNE_RB", "2,4,8"):
            if ns > 4 and rb != 4:
                continue
            for pd in ints("TUNE_PD", "1,2"):
                for pc in ints("TUNE_PERCU", "1,2,3,4,6"):
                    cfgs.append((ns, rb, pd, pc, 0))
    for ch in ints("TUNE_CHUNKS", ""):
        for ns in nss:
            cfgs.append((ns, 4, 1, 0, ch))

    # bitwise check against streamN (same NS) on the first H
    ref = {}
    for ns in sorted({c[0] for c in cfgs} & {3, 4}):
        o = g.buf[1].clone()
        streamn(ns, hs[0], o)
        ref[ns] = o
    ok = {}
    for c in cfgs:
        if c[0] not in ref:
            ok[c] = None
            continue
        o = g.buf[1].clone()
        try:
            pipe(c, hs[0], o)
        except RuntimeError:  # an arm this (ns, rb, pd) combination does not compile
            ok[c] = "n/a"
            continue
        torch.cuda.synchronize()
        ok[c] = bool(torch.equal(o, ref[c[0]]))
        if not ok[c]:
            d = (o != ref[c[0]]).nonzero()
            print(json.dumps({"MISMATCH": c, "n_bad": int(d.shape[0]), "first": d[:4].tolist()}), flush=True)

    out = g.buf[1]
    spin_cfg = next(c for c in cfgs if ok[c] != "n/a")
    # clock ramp: TUNE_SPIN seconds of back-to-back passes before timing
    import time
    t_end = time.perf_counter() + float(os.environ.get("TUNE_SPIN", "1.5"))
    while time.perf_counter() < t_end:
        for _ in range(8):
            pipe(spin_cfg, hs[0], out)
        torch.cuda.synchronize()
    reps = int(os.environ.get("TUNE_REPS", "4"))
    for H in hs:
        arms = [("streamn", ns) for ns in nss if ns in (3, 4)] + [("pipe", c) for c in cfgs if ok[c] != "n/a"]
        times = {a: [] for a in arms}
        for _ in range(5):
            for a in arms:
                f = (lambda: streamn(a[1], H, out)) if a[0] == "streamn" else (lambda: pipe(a[1], H, out))
                f()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    f()
                e1.record()
                e1.synchronize()
                times[a].append(e0.elapsed_time(e1) / reps)
        for a in sorted(arms, key=lambda a: sorted(times[a])[2] / (a[1] if a[0] == "streamn" else a[1][0])):
            ns = a[1] if a[0] == "streamn" else a[1][0]
            ms = sorted(times[a])[2] / ns
            rec = {"H": H, "kernel": a[0], "ns": ns, "ms_per_step": round(ms, 5),
                   "ideal_vs_16384": round(ms * 16384 / H, 4)}
            if a[0] == "pipe":
                rec.update({"rb": a[1][1], "pd": a[1][2], "per_cu": a[1][3], "chunk": a[1][4],
                            "bitwise_vs_streamn": ok[a[1]]})
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
