"""Lecture studies as commands (one JSON line per measurement).

    python -m cme213x occupancy                       kernel resources + occupancy
    python -m cme213x study divergence|coalescing|summation|openmp
"""
from __future__ import annotations

import argparse
import json


def _time(fn, iters=10):
    import torch

    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def divergence_study(n=1 << 24, work=256):
    import torch

    from ..ops.studies import divergence

    out = torch.empty(n, device="cuda")
    for stride in (1, 2, 4, 8, 16, 32, 64, 128):
        ms = _time(lambda: divergence(out, stride, work))
        yield {"study": "divergence", "stride": stride, "ms": round(ms, 4), "MThreads_per_s": round(n / ms / 1e3, 1),
               "diverged": stride < 64}


def coalescing_study(n=1 << 24):
    import torch

    from ..ops.studies import strided_copy

    src = torch.rand(n * 33 + 64, device="cuda")
    for stride in (1, 2, 4, 8, 16, 32):
        ms = _time(lambda: strided_copy(src, n, stride))
        yield {"study": "coalescing", "stride": stride, "offset": 0, "ms": round(ms, 4),
               "useful_GBps": round(8 * n / ms / 1e6, 1)}
    for offset in (0, 1, 3, 16, 17, 32):
        ms = _time(lambda: strided_copy(src, n, 1, offset))
        yield {"study": "coalescing", "stride": 1, "offset": offset, "ms": round(ms, 4),
               "useful_GBps": round(8 * n / ms / 1e6, 1)}


def summation(device):
    from ..ops.studies import summation_study

    for row in summation_study(device=device):
        yield {"study": "summation", **{k: (v if k == "n" else float(f"{v:.3e}")) for k, v in row.items()}}


def openmp_study():
    import numpy as np

    from ..ops.studies import omp_schedule_study, omp_sum

    for r in omp_schedule_study():
        yield {"study": "openmp_schedule", **r}
    x = np.random.default_rng(0).random(1 << 24)
    for mode in ("for", "task"):
        s, sec = omp_sum(x, mode)
        yield {"study": "openmp_sum", "mode": mode, "seconds": sec, "sum": s}


def study_main(argv=None) -> int:
    import torch

    ap = argparse.ArgumentParser(prog="cme213x study")
    ap.add_argument("which", choices=["divergence", "coalescing", "summation", "openmp"])
    a = ap.parse_args(argv)
    gpu = torch.cuda.is_available()
    if a.which in ("divergence", "coalescing") and not gpu:
        print("study needs a GPU")
        return 1
    gen = {"divergence": divergence_study, "coalescing": coalescing_study, "openmp": openmp_study}.get(a.which)
    rows = gen() if gen else summation("cuda" if gpu else None)
    for r in rows:
        print(json.dumps(r), flush=True)
    return 0


def occupancy_main(argv=None) -> int:
    from ..utils.occupancy import main

    return main(argv)
