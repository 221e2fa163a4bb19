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
    from ..models.heat2d_dist import run_hw5
    from ..parallel.comm import init_from_env

    ap = argparse.ArgumentParser(prog="heat2d_mpi")
    ap.add_argument("params")
    ap.add_argument("--ranks", type=int, default=0, help="simulate N ranks in one process (loopback)")
    ap.add_argument("--device", default=None)
    ap.add_argument("--float", action="store_true", help="fp32 instead of the reference's fp64")
    ap.add_argument("--tblock", default="auto", help="timesteps per halo exchange / HBM pass (1-4, or auto)")
    ap.add_argument("--kernel", default="auto", choices=["auto", "pipe", "streamn", "tile"],
                    help="multi-step pass kernel (tile: LDS-resident tiles, single-grid runs)")
    ap.add_argument("--fma", action="store_true", help="FMA-contracted stencil (the reference CPU's is not)")
    ap.add_argument("--fast", action="store_true",
                    help="reassociated stencil (folded CFL weights, pair sums; within 10 ULP of exact): fp32 "
                         "(--float) order 8 multi-step passes, csrc/hip/heat_fast.hip")
    ap.add_argument("--native", default="auto", choices=["auto", "on", "off"],
                    help="GPU time loop: the native C++ loop after a bitwise self-test (auto), required (on), "
                         "or the Python loop (off)")
    ap.add_argument("--transport", default=None, choices=["rccl", "ipc"],
                    help="native halo transport under torchrun (default: rccl on nccl, ipc with --share-gpu)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="under torchrun: every rank on cuda:0, gloo control plane, IPC halo transport "
                         "(rehearses the multi-process run on one GPU)")
    ap.add_argument("--periodic", default="", choices=["", "x", "y", "xy"],
                    help="wrap the decomposition along x / y (not in the reference; with one rank every halo "
                         "is a self-send)")
    a = ap.parse_args(argv)
    tblock = a.tblock if a.tblock == "auto" else int(a.tblock)
    dtype = torch.float32 if a.float else torch.float64
    periodic = ("x" in a.periodic, "y" in a.periodic)
    fma = "fast" if a.fast else a.fma
    if a.ranks:
        run_hw5(a.params, None, dtype, a.device, tblock=tblock, fma=fma, kernel=a.kernel, native=a.native,
                local_ranks=list(range(a.ranks)), world=a.ranks, periodic=periodic)
        return 0
    comm = init_from_env(backend="gloo" if a.share_gpu else None, share_gpu=a.share_gpu)
    run_hw5(a.params, comm, dtype, a.device, tblock=tblock, fma=fma, kernel=a.kernel, native=a.native,
            periodic=periodic, transport=a.transport or ("ipc" if a.share_gpu else None))
    return 0
