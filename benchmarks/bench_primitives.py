#!/usr/bin/env python3
"""Single-GPU benchmarks for the BASELINE.md headline primitives. One JSON line
per measurement with the reference number it is compared against.

  copy       1 GiB 16-B copy (achievable-HBM calibration)
  scan       2^26 elements: look-back / Blelloch / Hillis-Steele (BASELINE #11)
  reduce     2^26 elements
  spmvscan   the 15 final-project shapes (BASELINE #19-21, synthetic values)
  cipher     19.76 MB moby-dick x16 (BASELINE #1-3)
  pagerank   2^21 nodes, avg 8 edges, 20 iterations (BASELINE #5)
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


SINGLE = {}  # last measurement's one-call-per-event-pair median (ms)


def timeit(fn, iters=10, warmup=2):
    """Median ms per call. Each event pair brackets one call; when that call
    is short (< 0.2 ms) the pair brackets max(2, 0.2 ms / t) back-to-back calls
    instead and the time is divided by their count, so the host's per-call
    Python/launch latency (~5-10 us, box-dependent) and the idle-clock ramp
    between isolated calls do not masquerade as kernel time. The one-call
    median stays in SINGLE["ms"] (emitted as ms_single)."""
    import torch

    def med(reps):
        ts = []
        for _ in range(iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / reps)
        ts.sort()
        return ts[len(ts) // 2]

    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    single = med(1)
    SINGLE["ms"] = single
    if single >= 0.2:
        return single
    return min(single, med(max(2, min(100, int(0.2 / max(single, 1e-4))))))


def emit(**kw):
    single = SINGLE.pop("ms", None)
    if single is not None and "ms" in kw and single != kw["ms"]:
        kw["ms_single"] = single
    print(json.dumps(kw), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=None)
    args = ap.parse_args()
    import numpy as np
    import torch

    import cme213x
    from cme213x.ops import elementwise, scan as sc

    want = lambda k: args.only is None or k in args.only  # noqa: E731
    dev = torch.device("cuda")

    if want("copy"):
        a = torch.empty(1 << 28, dtype=torch.float32, device=dev).uniform_()
        b = torch.empty_like(a)
        ms = timeit(lambda: elementwise.copy_(b, a))
        emit(bench="copy", bytes=2 * a.numel() * 4, ms=ms, GBps=2 * a.numel() * 4 / ms / 1e6)
        ms = timeit(lambda: b.copy_(a))
        emit(bench="copy_torch", bytes=2 * a.numel() * 4, ms=ms, GBps=2 * a.numel() * 4 / ms / 1e6)
        del a, b

    if want("scan"):
        n = 1 << 26
        x = torch.rand(n, device=dev)
        y = torch.empty_like(x)
        for algo in ("lookback", "rts", "blelloch", "hillis", "blelloch_mlevel", "hillis_mlevel"):
            ms = timeit(lambda: sc.scan(x, True, y, algo))
            emit(bench="scan", algo=algo, n=n, ms=ms, GBps=8 * n / ms / 1e6, ref_ms=15.85,
                 speedup_vs_ref=15.85 / ms)
        ms = timeit(lambda: torch.cumsum(x, 0, out=y))
        emit(bench="scan", algo="torch.cumsum", n=n, ms=ms, GBps=8 * n / ms / 1e6)
        xi = torch.randint(0, 100, (n,), device=dev, dtype=torch.int32)
        yi = torch.empty_like(xi)
        for algo in ("lookback", "rts"):
            ms = timeit(lambda: sc.scan(xi, True, yi, algo))
            emit(bench="scan", algo=f"{algo}-int32", n=n, ms=ms, GBps=8 * n / ms / 1e6)
        for algo in ("vector", "tree"):
            ms = timeit(lambda: sc.reduce(x, "sum", algo))
            emit(bench="reduce", algo=algo, n=n, ms=ms, GBps=4 * n / ms / 1e6)
        ms = timeit(lambda: x.sum())
        emit(bench="reduce", algo="torch.sum", n=n, ms=ms, GBps=4 * n / ms / 1e6)
        del x, y, xi, yi

    if want("spmvscan"):
        from cme213x.models.spmv_scan import BENCH_SHAPES, REF_MS, SpmvScanSolver, generate

        for name, (n, p, N) in BENCH_SHAPES.items():
            prob = generate(n, p, 100000, N, seed=1)
            sol = SpmvScanSolver(prob, dev)
            sol.run(2)
            ms = timeit(lambda: sol.run(), iters=5, warmup=1)
            emit(bench="spmvscan", matrix=name, n=n, p=p, N=N, ms=ms, GBps=12 * n * N / ms / 1e6,
                 ref_ms=REF_MS[name], speedup_vs_ref=REF_MS[name] / ms)
            # the same N-iteration loop replayed as one hipGraph
            from cme213x.utils.graphs import GraphRunner

            g = GraphRunner(lambda: sol.run())
            ms = timeit(g, iters=5, warmup=1)
            emit(bench="spmvscan_graph", matrix=name, n=n, p=p, N=N, ms=ms, GBps=12 * n * N / ms / 1e6,
                 ref_ms=REF_MS[name], speedup_vs_ref=REF_MS[name] / ms)

    if want("spmvscan_algos"):
        from cme213x.models.spmv_scan import BENCH_SHAPES, REF_MS, SpmvScanSolver, generate

        for name in ("dense2", "mac_econ_fwd500", "webbase-1M", "mc2depi"):
            n, p, N = BENCH_SHAPES[name]
            prob = generate(n, p, 100000, N, seed=1)
            for algo in ("lookback", "wave", "serial"):
                sol = SpmvScanSolver(prob, dev, algo)
                sol.run(1)
                ms = timeit(lambda: sol.run(), iters=3, warmup=1)
                emit(bench="spmvscan_algo", matrix=name, algo=algo, n=n, p=p, N=N, ms=ms,
                     GBps=12 * n * N / ms / 1e6, ref_ms=REF_MS[name], speedup_vs_ref=REF_MS[name] / ms)
                del sol

    if want("algorithms"):
        bench_algorithms(emit, timeit)

    if want("cipher"):
        path = "/root/reference/hw/hw1/programming/mobydick.txt"
        text = np.fromfile(path, dtype=np.uint8) if os.path.exists(path) else \
            np.random.default_rng(0).integers(0, 128, 1235150, dtype=np.uint8)
        for copies in (16, 208):
            d = torch.from_numpy(np.tile(text, copies)).to(dev)
            o = torch.empty_like(d)
            for w in ("char", "uint", "uint2", "uint4"):
                ms = timeit(lambda: elementwise.shift_cipher(d, 3, o, width=w))
                emit(bench="cipher", width=w, bytes=d.numel(), ms=ms, GBps_rw=2 * d.numel() / ms / 1e6)

    if want("transpose"):
        bench_transpose(emit, timeit)

    if want("spmv"):
        bench_spmv(emit, timeit)

    if want("sort"):
        bench_sort(emit, timeit)

    if want("vigenere"):
        bench_vigenere(emit, timeit)

    if want("gemm"):
        bench_gemm(emit, timeit)

    if want("misc"):
        bench_misc(emit, timeit)

    if want("pagerank"):
        from cme213x.ops.graph import bytes_model, iterate, make_graph

        g = make_graph(1 << 21, 8).to(dev)
        x0 = torch.full((1 << 21,), 1.0 / (1 << 21), device=dev)
        for grp in (1, 4, 8, 16):
            ms = timeit(lambda: iterate(g, x0, 20, grp))
            emit(bench="pagerank", group=grp, ms=ms, GBps_model=bytes_model(g, 20) / ms / 1e6, ref_ms=1188.11,
                 speedup_vs_ref=1188.11 / ms)
        from cme213x.ops.graph import block_columns

        for blocks in (2, 4, 8):
            bg = block_columns(g, blocks)
            for grp in (1, 2, 4):
                ms = timeit(lambda: iterate(bg, x0, 20, grp))
                emit(bench="pagerank", blocks=blocks, group=grp, ms=ms, GBps_model=bytes_model(g, 20) / ms / 1e6,
                     ref_ms=1188.11, speedup_vs_ref=1188.11 / ms)


def bench_transpose(emit, timeit):
    import torch

    from cme213x.ops.transpose import VARIANTS, transpose

    from cme213x.ops.transpose import DIAGNOSTICS, diagnostic, transpose_reps

    ref = {8192: None, 4096: 130.0, 2048: 128.0}  # BASELINE #7/#8 best (LDS+pad+unroll, Fermi)
    for n in (8192, 4096, 2048):
        x = torch.rand(n, n, device="cuda")
        out = torch.empty_like(x)
        for v in VARIANTS:
            ms = timeit(lambda: transpose(x, v, out))
            gbps = 2 * n * n * 4 / ms / 1e6
            emit(bench="transpose", n=n, variant=v, ms=ms, GBps=gbps, ref_GBps=ref[n],
                 vs_ref=(gbps / ref[n]) if ref[n] else None)
        for d in DIAGNOSTICS:
            ms = timeit(lambda: diagnostic(x, d, out))
            emit(bench="transpose_diag", n=n, kind=d, ms=ms, GBps=2 * n * n * 4 / ms / 1e6)
        # the paper's two timing modes for the same kernel (lds_pad)
        reps = 20
        ms = timeit(lambda: transpose_reps(x, reps, out)) / reps
        SINGLE.pop("ms", None)
        emit(bench="transpose_timing_mode", n=n, mode="loop inside kernel", ms=ms, GBps=2 * n * n * 4 / ms / 1e6)


def bench_spmv(emit, timeit):
    import torch

    from cme213x.ops.spmv import laplacian, random_csr, spmv, to_coo, to_csr_aligned, to_dia, to_ell, to_hyb

    mats = {"5pt-1M": laplacian("5pt", 1000), "27pt-1M": laplacian("27pt", 100),
            "random-1M": random_csr(1 << 20, 1 << 20, 16, seed=1), "skew-1M": random_csr(1 << 20, 1 << 20, 16,
                                                                                             seed=2, skew=True)}
    for name, a in mats.items():
        x = torch.rand(a.ncols, device="cuda")
        fmts = {"csr_scalar": a, "csr_vector": a, "csr_aligned": to_csr_aligned(a), "coo": to_coo(a),
                "hyb": to_hyb(a)}
        if int((a.rp[1:] - a.rp[:-1]).max()) <= 64:
            fmts["ell"] = to_ell(a)[0]
        if name.startswith(("5pt", "27pt")):
            fmts["dia"] = to_dia(a)
        for f, m in fmts.items():
            md = m.to("cuda")
            y = torch.empty(a.nrows, device="cuda")
            kern = "scalar" if f == "csr_scalar" else "auto"
            ms = timeit(lambda: spmv(md, x, y, kernel=kern), iters=20)
            # Bell & Garland GTX 285: 27-pt DIA 39.6 GFLOP/s; best unstructured HYB 24.2
            ref = 39.6 if (name.startswith("27pt") and f == "dia") else (24.2 if f == "hyb" and name == "random-1M" else None)
            emit(bench="spmv", matrix=name, fmt=f, nnz=a.nnz, ms=ms, GFLOPs=2 * a.nnz / ms / 1e6, ref_GFLOPs=ref,
                 vs_ref=(2 * a.nnz / ms / 1e6 / ref) if ref else None)


def bench_sort(emit, timeit):
    import torch

    from cme213x.ops.sort import sort

    for n, ref_s, ref_name in ((16_000_000, 0.084, "radix 16M keys, 32 OpenMP threads (BASELINE #16)"),
                               (48_000_000, 0.617, "merge sort 48M ints, 32 threads (BASELINE #15)")):
        x = torch.randint(0, 2**31 - 1, (n,), dtype=torch.int32, device="cuda")
        for algo in ("radix", "merge"):
            ms = timeit(lambda: sort(x, algo=algo), iters=5)
            emit(bench="sort", algo=algo, n=n, ms=ms, Mkeys_per_s=n / ms / 1e3, ref_ms=ref_s * 1e3, ref=ref_name,
                 speedup_vs_ref=ref_s * 1e3 / ms)
        ms = timeit(lambda: torch.sort(x), iters=5)
        emit(bench="sort", algo="torch.sort", n=n, ms=ms, Mkeys_per_s=n / ms / 1e3)


def bench_vigenere(emit, timeit):
    import os

    import numpy as np

    from cme213x.models.vigenere import create_cipher, solve_cipher

    path = "/root/reference/hw/hw3/programming/mobydick.txt"
    if os.path.exists(path):
        book = open(path, "rb").read()
    else:  # English-frequency synthetic corpus of the same size
        rng = np.random.default_rng(0)
        en = np.array([8.17, 1.49, 2.78, 4.25, 12.70, 2.23, 2.02, 6.09, 6.97, 0.15, 0.77, 4.03, 2.41, 6.75, 7.51,
                       1.93, 0.10, 5.99, 6.33, 9.06, 2.76, 0.98, 2.36, 0.15, 1.97, 0.07])
        book = rng.choice(np.arange(97, 123, dtype=np.uint8), 1_235_150, p=en / en.sum()).tobytes()
    c, key = create_cipher(book, 500, device="cuda", out_path=None)
    import time

    import torch

    solve_cipher(c, device="cuda", out_path=None, verbose=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        r = solve_cipher(c, device="cuda", out_path=None, verbose=False)
    torch.cuda.synchronize()
    secs = time.perf_counter() - t0
    emit(bench="vigenere_solve_x10", key_length=r["key_length"], seconds=secs, ref_seconds=17.0,
         speedup_vs_ref=17.0 / secs)


def bench_gemm(emit, timeit):
    import torch

    from cme213x.ops.gemm import sgemm

    ref = {"naive": 80.0, "lds": 235.9, "mfma": 784.6}  # GTX 480 GFLOP/s (Lecture09; mfma vs CUBLAS)
    for n in (1024, 4096, 8192):
        A = torch.randn(n, n, device="cuda")
        B = torch.randn_like(A)
        C = torch.empty_like(A)
        for v in (("naive",) if n <= 4096 else ()) + ("lds", "mfma"):
            ms = timeit(lambda: sgemm(A, B, C, variant=v), iters=3, warmup=1)
            gf = 2 * n ** 3 / ms / 1e6
            emit(bench="sgemm", n=n, variant=v, ms=ms, GFLOPs=gf, ref_GFLOPs=ref[v], vs_ref=gf / ref[v])
        torch.backends.cuda.matmul.allow_tf32 = False
        ms = timeit(lambda: torch.mm(A, B, out=C), iters=3, warmup=1)
        emit(bench="sgemm", n=n, variant="torch.mm(hipBLASLt)", ms=ms, GFLOPs=2 * n ** 3 / ms / 1e6)


def bench_algorithms(emit, timeit):
    import torch

    from cme213x.ops import algorithms as A

    n = 1 << 26
    x = torch.rand(n, device="cuda")
    m = x < 0.5
    ms = timeit(lambda: A.copy_if(x, m))
    emit(bench="copy_if", n=n, ms=ms, GBps=(4 * n + 2 * n + 4 * n / 2) / ms / 1e6)
    ms = timeit(lambda: x[m])
    emit(bench="copy_if", impl="torch x[mask]", n=n, ms=ms, GBps=(4 * n + 2 * n + 4 * n / 2) / ms / 1e6)
    ms = timeit(lambda: A.stable_partition(x, m))
    emit(bench="stable_partition", n=n, ms=ms, GBps=(8 * n + 2 * n) / ms / 1e6)
    k = torch.sort(torch.randint(0, 1 << 20, (n,), device="cuda", dtype=torch.int32)).values
    ms = timeit(lambda: A.unique(k))
    emit(bench="unique", n=n, ms=ms, GBps=(4 * n + 4 * (1 << 20)) / ms / 1e6)
    ms = timeit(lambda: torch.unique_consecutive(k))
    emit(bench="unique", impl="torch.unique_consecutive", n=n, ms=ms, GBps=(4 * n + 4 * (1 << 20)) / ms / 1e6)
    v = torch.rand(n, device="cuda")
    ms = timeit(lambda: A.reduce_by_key(k, v))
    emit(bench="reduce_by_key", n=n, segments=1 << 20, ms=ms)
    q = torch.randint(0, 1 << 20, (1 << 24,), device="cuda", dtype=torch.int32)
    ms = timeit(lambda: A.lower_bound(k, q))
    emit(bench="lower_bound", n=n, queries=q.numel(), ms=ms, Gqueries_per_s=q.numel() / ms / 1e6)
    ms = timeit(lambda: torch.searchsorted(k, q))
    emit(bench="lower_bound", impl="torch.searchsorted", n=n, queries=q.numel(), ms=ms,
         Gqueries_per_s=q.numel() / ms / 1e6)
    ms = timeit(lambda: A.max_element(x))
    emit(bench="max_element", n=n, ms=ms, GBps=4 * n / ms / 1e6)
    ms = timeit(lambda: torch.argmax(x).item())
    emit(bench="max_element", impl="torch.argmax", n=n, ms=ms, GBps=4 * n / ms / 1e6)
    keys = torch.randint(0, 256, (n,), device="cuda", dtype=torch.int32)
    ms = timeit(lambda: A.counting_sort(keys, 256))
    emit(bench="counting_sort", n=n, num_keys=256, ms=ms, Gkeys_per_s=n / ms / 1e6)


def bench_misc(emit, timeit):
    import math

    import torch

    from cme213x.ops.atomics import global_max, monte_carlo_pi

    n = 1 << 30
    import time

    monte_carlo_pi(1 << 20, 1, "cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pi, _ = monte_carlo_pi(n, 3, "cuda")
    dt = time.perf_counter() - t0
    emit(bench="monte_carlo_pi", samples=n, seconds=dt, Gsamples_per_s=n / dt / 1e9, err=abs(pi - math.pi))
    x = torch.randn(1 << 26, device="cuda")
    ms = timeit(lambda: global_max(x))
    emit(bench="global_max", n=x.numel(), ms=ms, GBps=4 * x.numel() / ms / 1e6)


if __name__ == "__main__":
    main()
