"""Final-project drivers.

    python -m cme213x fp a.txt x.txt [check] [--algo lookback|wave|serial] [--graph]  -> b.txt (+ b_cpu.txt)
    python -m cme213x checker a.txt x.txt b.txt    (reference_spMVscan-released)
    python -m cme213x readmm <matrix.mtx> <outdir> [q N]   (readMM.py)
    python -m cme213x genfp <name|n p> <outdir> [--q Q] [--iters N]
"""
from __future__ import annotations

import os
import sys

import numpy as np


def fp_main(argv=None) -> int:
    from ..models.spmv_scan import run_fp

    argv = list(sys.argv[1:] if argv is None else argv)
    algo = "lookback"
    if "--algo" in argv:
        i = argv.index("--algo")
        algo = argv[i + 1]
        del argv[i:i + 2]
    graph = "--graph" in argv
    argv = [a for a in argv if a != "--graph"]
    if len(argv) < 2:
        print('Run command: ./fp "file a.txt" "file x.txt"')
        return 0
    res = run_fp(argv[0], argv[1], cpu_check=len(argv) >= 3, algo=algo, graph=graph)
    if "relL2" in res:
        print(f"relative L2 error {res['relL2']:g}, relative Linf error {res['relLinf']:g}")
    return 0


def checker_main(argv=None) -> int:
    """``checker a.txt x.txt b.txt [--legacy]``: the instructor checker
    (reference_spMVscan-released.cu); ``--legacy`` uses the older O(len^2)
    serial algorithm of aux/CheckOutput/serialMV.cu (small inputs)."""
    from ..models.spmv_scan import errors, load, reference_solution, reference_solution_quadratic

    argv = list(sys.argv[1:] if argv is None else argv)
    legacy = "--legacy" in argv
    argv = [a for a in argv if a != "--legacy"]
    if len(argv) != 3:
        print("usage: checker a.txt x.txt b.txt [--legacy]")
        return 1
    prob = load(argv[0], argv[1])
    b = np.fromfile(argv[2], sep=" ")
    ref = reference_solution_quadratic(prob) if legacy else reference_solution(prob)
    e = errors(ref, b[:prob.n])
    print(f"Absolute L2 error: {e['L2']:g}\nRelative L2 error: {e['relL2']:g}\n"
          f"Absolute Linf error: {e['Linf']:g}\nRelative Linf error: {e['relLinf']:g}")
    return 0


def readmm_main(argv=None) -> int:
    """Matrix Market -> a.txt/x.txt with readMM.py's rules (n = nnz,
    p = max(row), random s / k / x)."""
    from ..models.spmv_scan import generate, save
    from ..utils.mmio import read_matrix_market

    argv = sys.argv[1:] if argv is None else argv
    if len(argv) < 2:
        print("usage: readmm <matrix.mtx> <outdir> [q N]")
        return 1
    rng = np.random.default_rng()
    rows, cols, vals, shape = read_matrix_market(argv[0])
    q = int(argv[2]) if len(argv) > 2 else int(rng.integers(1000, 1000001))
    N = int(argv[3]) if len(argv) > 3 else int(rng.uniform(5, 100))
    n = vals.size
    p = int(rows.max())  # readMM.py: p = max(row) (0-based after mmread)
    prob = generate(n, p, q, N, values=vals)
    os.makedirs(argv[1], exist_ok=True)
    save(prob, os.path.join(argv[1], "a.txt"), os.path.join(argv[1], "x.txt"))
    return 0


def genfp_main(argv=None) -> int:
    import argparse

    from ..models.spmv_scan import BENCH_SHAPES, generate, save

    ap = argparse.ArgumentParser(prog="genfp")
    ap.add_argument("shape", nargs="+", help="benchmark matrix name, or n p")
    ap.add_argument("outdir")
    ap.add_argument("--q", type=int, default=100000)
    ap.add_argument("--iters", type=int, default=None)
    a = ap.parse_args(argv)
    if len(a.shape) == 1:
        n, p, N = BENCH_SHAPES[a.shape[0]]
    else:
        n, p, N = int(a.shape[0]), int(a.shape[1]), 10
    prob = generate(n, p, a.q, a.iters or N)
    os.makedirs(a.outdir, exist_ok=True)
    save(prob, os.path.join(a.outdir, "a.txt"), os.path.join(a.outdir, "x.txt"))
    return 0
