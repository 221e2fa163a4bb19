#!/usr/bin/env python3
"""The hw5 workload through the DEFAULT driver path (BASELINE #17 / #18).

    python benchmarks/bench_hw5.py [--n 1000 2000] [--reps 5]

Runs ``run_hw5`` -- the ``heat2d_mpi`` driver (hw/hw5/2dHeat_solution.cpp:630-664)
-- on the reference's params.in (1000^2, order 8, 1000 iterations, IC 3, BCs
0/10/0/10; the 2000^2 row changes only nx, ny), fp64 as the reference, one
rank, with the driver's automatic steps-per-pass and pass-kernel choice
(models/heat2d_dist.py auto_tblock / auto_kernel). Prints one JSON line per
size with the driver's own "took" time (median of reps, files not written)."""
import argparse
import contextlib
import io
import json
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

REF_S = {1000: 2.31, 2000: 9.52}  # BASELINE #17 / #18: P = 9 CPU ranks, 1-D async


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[1000, 2000])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--fma", action="store_true", help="FMA-contracted stencil (the driver default is exact)")
    ap.add_argument("--tune", nargs="*", default=[],
                    help="tuning knobs name=value (cme213x.utils.tuning), e.g. pipe_per_cu=2")
    a = ap.parse_args()

    import torch

    import cme213x  # noqa: F401
    from cme213x.models.heat2d_dist import run_hw5
    from cme213x.utils import tuning

    knobs = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in a.tune}
    for k, v in knobs.items():
        tuning.set(k, v)

    src = open(os.path.join(REPO, "tests", "data", "hw5_params.in")).read().split("\n")
    for n in a.n:
        lines = list(src)
        lines[0] = f"{n} {n}"
        with tempfile.NamedTemporaryFile("w", suffix=".in", delete=False) as f:
            f.write("\n".join(lines))
            path = f.name
        secs = []
        info = {}
        for r in range(a.reps + 1):
            with contextlib.redirect_stdout(io.StringIO()):
                res = run_hw5(path, None, torch.float64, "cuda", write_files=False, fma=a.fma)
            if r:  # first run: warm-up (code objects, allocations)
                secs.append(res["seconds"])
            sim = res["sim"]
            info = {"tblock": sim.tblock, "kernel": sim.kernel, "fma": sim.fma}
        os.unlink(path)
        secs.sort()
        s = secs[len(secs) // 2]
        print(json.dumps({"bench": "hw5", "n": n, "order": 8, "iters": 1000, "dtype": "fp64", "ranks": 1, **info,
                          "tune": knobs,
                          "seconds": round(s, 5), "ms": round(s * 1e3, 3), "ref_s": REF_S.get(n),
                          "speedup_vs_ref": round(REF_S[n] / s, 1) if n in REF_S else None}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
