#!/usr/bin/env python3
"""SpMV per-format table with the MALL / L2 defeated (BASELINE config #4 and
Bell & Garland §4).

MI355X's 256 MB Infinity Cache (MALL) holds a whole 1M-row 5-point Laplacian
(~50 MB), so timing one operand set over and over measures cache bandwidth,
not HBM. Here every format is timed twice:
  * ``cold``: R device copies of (matrix, x, y) whose total footprint is
    >= 768 MB (3x the MALL) are visited round-robin, one multiply each, so
    no call finds its operands in any cache;
  * ``warm``: the same operand set every call (the round-1 number).
Both loops are captured in hipGraphs (GPU time, not the Python launch rate).
Reported per format: ms per multiply, GFLOP/s (2 nnz / t), the minimum HBM
bytes of the format (every matrix array + x + y once) and that rate as % of
the measured 16-B copy bandwidth. ``auto`` is ``ops.spmv.prepare(a,
"auto")`` and its ratio to the best format of the matrix.

    python benchmarks/bench_spmv.py [--mats 5pt-1M 5pt-16M ...] [--fmts ...]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FOOTPRINT = 768 << 20


def tensors_of(m):
    from dataclasses import fields, is_dataclass

    import torch

    out = []
    if is_dataclass(m):
        for f in fields(m):
            v = getattr(m, f.name)
            if isinstance(v, torch.Tensor):
                out.append(v)
            elif is_dataclass(v):
                out.extend(tensors_of(v))
            elif isinstance(v, tuple):  # column blocks
                for e in v:
                    if is_dataclass(e):
                        out.extend(tensors_of(e))
    return out


def clone(m):
    """Deep copy of a format dataclass (every tensor cloned on its device)."""
    from dataclasses import fields, is_dataclass, replace

    import torch

    kw = {}
    for f in fields(m):
        v = getattr(m, f.name)
        if isinstance(v, torch.Tensor):
            kw[f.name] = v.clone()
        elif is_dataclass(v):
            kw[f.name] = clone(v)
        elif isinstance(v, tuple) and v and is_dataclass(v[0]):
            kw[f.name] = tuple(clone(e) for e in v)
    return replace(m, **kw)


def nbytes(m) -> int:
    return sum(t.numel() * t.element_size() for t in tensors_of(m))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mats", nargs="*", default=["5pt-1M", "5pt-16M", "27pt-1M", "random-1M", "skew-1M"])
    ap.add_argument("--fmts", nargs="*", default=None)
    ap.add_argument("--calls", type=int, default=64)
    ap.add_argument("--out", default=None)
    ap.add_argument("--eager", action="store_true", help="no hipGraph capture (for rocprofv3 counter runs)")
    ap.add_argument("--tune", nargs="*", default=[], help="tuning knobs name=value, e.g. spmv_stream_rows=1024")
    args = ap.parse_args()
    import torch

    import cme213x
    from cme213x.ops import elementwise
    from cme213x.ops.spmv import choose_format, laplacian, matrix_stats, prepare, random_csr, spmv

    out = open(args.out, "a") if args.out else None
    from cme213x.utils import tuning

    knobs = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in args.tune}
    for k, v in knobs.items():
        tuning.set(k, v)

    def emit(**kw):
        s = json.dumps(kw)
        print(s, flush=True)
        if out:
            out.write(s + "\n")
            out.flush()

    def t_ms(fn, reps=5):
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return sorted(ts)[reps // 2]

    # calibration: 1 GiB 16-B copy
    a = torch.empty(1 << 28, dtype=torch.float32, device="cuda")
    b = torch.empty_like(a)
    elementwise.copy_(b, a)
    copy_GBps = 2 * a.numel() * 4 / t_ms(lambda: elementwise.copy_(b, a)) / 1e6
    del a, b
    emit(bench="copy", GBps=round(copy_GBps, 1))

    gens = {"5pt-1M": lambda: laplacian("5pt", 1000), "5pt-16M": lambda: laplacian("5pt", 4000),
            "27pt-1M": lambda: laplacian("27pt", 100), "random-1M": lambda: random_csr(1 << 20, 1 << 20, 16, seed=1),
            "skew-1M": lambda: random_csr(1 << 20, 1 << 20, 16, seed=2, skew=True)}
    for name in args.mats:
        A = gens[name]()
        st = matrix_stats(A)
        auto = choose_format(A, st)
        fmts = args.fmts or ["csr_scalar", "csr_vector", "csr_stream", "csr_short", "csr_aligned", "csr_cb", "coo", "hyb", "ell",
                             "dia"]
        res = {}
        for f in fmts:
            if f == "ell" and (st.max_row > 64 or st.ell_fill < 0.3):
                continue
            if f == "dia" and (st.ndiag > 64 or st.dia_fill < 0.3):
                continue
            if f in ("csr_scalar", "csr_short", "csr_wave") and st.max_row > 1024:
                continue  # thread-per-row on a power-law row: seconds, not a contender
            _, m = prepare(A, f, "cuda")
            mb = nbytes(m) + 4 * (A.ncols + A.nrows)
            reps = 1 if mb >= FOOTPRINT else min(16, -(-FOOTPRINT // mb))
            sets = [(m, torch.rand(A.ncols, device="cuda"), torch.empty(A.nrows, device="cuda"))]
            for _ in range(reps - 1):
                sets.append((clone(m), torch.rand(A.ncols, device="cuda"), torch.empty(A.nrows, device="cuda")))
            kern = {"csr_scalar": "scalar", "csr_vector": "vector", "csr_stream": "stream", "csr_short": "short",
                    "csr_wave": "wave"}.get(f, "auto")

            def cold():
                for i in range(args.calls):
                    mm, x, y = sets[i % len(sets)]
                    spmv(mm, x, y, kernel=kern)

            def warm():
                mm, x, y = sets[0]
                for _ in range(args.calls):
                    spmv(mm, x, y, kernel=kern)

            # both loops captured in hipGraphs: GPU time, not Python launch rate
            cold()
            warm()
            torch.cuda.synchronize()
            if args.eager:
                ms_cold, ms_warm = t_ms(cold) / args.calls, t_ms(warm) / args.calls
                res[f] = ms_cold
                emit(bench="spmv_eager", matrix=name, fmt=f, ms_cold=round(ms_cold, 5), ms_warm=round(ms_warm, 5))
                del sets
                continue
            gc, gw = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(gc):
                cold()
            with torch.cuda.graph(gw):
                warm()
            gc.replay()
            gw.replay()
            torch.cuda.synchronize()
            ms_cold = t_ms(gc.replay) / args.calls
            ms_warm = t_ms(gw.replay) / args.calls
            del gc, gw
            mb1 = nbytes(m) + 4 * (A.ncols + A.nrows)
            res[f] = ms_cold
            emit(bench="spmv", matrix=name, fmt=f, tune=knobs, nnz=A.nnz, sets=len(sets), ms_cold=round(ms_cold, 5),
                 ms_warm=round(ms_warm, 5), GFLOPs_cold=round(2 * A.nnz / ms_cold / 1e6, 1),
                 GFLOPs_warm=round(2 * A.nnz / ms_warm / 1e6, 1), min_bytes=mb1,
                 GBps_cold=round(mb1 / ms_cold / 1e6, 1), pct_copy_cold=round(100 * mb1 / ms_cold / 1e6 / copy_GBps, 1),
                 auto=(f == auto))
            del sets
            torch.cuda.empty_cache()
        best = min(res, key=res.get)
        emit(bench="spmv_auto", matrix=name, auto=auto, best=best, ms_auto=round(res.get(auto, float("nan")), 5),
             ms_best=round(res[best], 5), auto_vs_best=round(res.get(auto, float("inf")) / res[best], 3),
             stats={k: (round(v, 4) if isinstance(v, float) else v) for k, v in vars(st).items()})


if __name__ == "__main__":
    main()
