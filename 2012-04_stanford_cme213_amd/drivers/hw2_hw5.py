"""Heat-diffusion drivers.

    python -m cme213x heat2d params.in [--double] [--variants global shared stream]
    torchrun --nproc-per-node N -m cme213x heat2d_mpi params.in   (hw5 format)
    python -m cme213x heat2d_mpi params.in --ranks 4             (single process, loopback)
"""
from __future__ import annotations

import argparse

import torch


def heat2d_main(argv=None) -> int:
    from ..models.heat2d import run_hw2

    ap = argparse.ArgumentParser(prog="heat2d")
    ap.add_argument("params")
    ap.add_argument("--double", action="store_true")
    ap.add_argument("--variants", nargs="+", default=["global", "shared", "stream"])
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)
    res = run_hw2(a.params, torch.float64 if a.double else torch.float32, a.device, variants=a.variants)
    return 1 if any(v["errors"] for v in res["variants"].values()) else 0


def heat2d_mpi_main(argv=None) -> int:
    from ..models.heat2d_dist import DistHeat, run_hw5
    from ..parallel.comm import init_from_env
    from ..utils.params import SimParams

    ap = argparse.ArgumentParser(prog="heat2d_mpi")
    ap.add_argument("params")
    ap.add_argument("--ranks", type=int, default=0, help="simulate N ranks in one process (loopback)")
    ap.add_argument("--device", default=None)
    ap.add_argument("--float", action="store_true", help="fp32 instead of the reference's fp64")
    ap.add_argument("--tblock", default="auto", help="timesteps per halo exchange / HBM pass (1-4, or auto)")
    ap.add_argument("--kernel", default="auto", choices=["auto", "pipe", "streamn"], help="3-4 step pass kernel")
    ap.add_argument("--fma", action="store_true", help="FMA-contracted stencil (the reference CPU's is not)")
    a = ap.parse_args(argv)
    tblock = a.tblock if a.tblock == "auto" else int(a.tblock)
    dtype = torch.float32 if a.float else torch.float64
    if a.ranks:
        import time

        p = SimParams.from_file(a.params, flavor="hw5")
        print(p.banner())
        dev = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
        sim = DistHeat(p, None, dtype, dev, local_ranks=list(range(a.ranks)), world=a.ranks, tblock=tblock,
                       fma=a.fma, kernel=a.kernel)
        sim.save_text("init")
        t0 = time.perf_counter()
        sim.run(p.iters)
        if torch.device(dev).type == "cuda":
            torch.cuda.synchronize()
        print(f"{p.iters} iterations on a {p.nx} by {p.ny} grid took: {time.perf_counter() - t0} seconds.")
        sim.save_text("final")
        return 0
    comm = init_from_env()
    dev = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    run_hw5(a.params, comm, dtype, dev, tblock=tblock, fma=a.fma, kernel=a.kernel)
    return 0
