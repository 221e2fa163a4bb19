#!/usr/bin/env python3
"""Distributed SpMV (row-partitioned, Lecture20) on the 5-pt Laplacian of an
n x n grid (n^2 rows; the BASELINE.json SpMV config is n = 1000), one rank per
GPU over RCCL -- the "SpMV GFLOP/s at 1/2/4/8 MI355X" part of the metric.

    python benchmarks/bench_dist_spmv.py [--n 1000] [--mode halo|allgather] [--transport rccl|torch]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 benchmarks/bench_dist_spmv.py --n 4096

``halo`` (default) exchanges only the x entries each neighbour needs (one
grouped P2P batch; ``--transport rccl`` = the framework's own RCCL
communicator on a side stream, ``torch`` = torch.distributed) and overlaps it
with the interior product; ``allgather`` is the lecture's MPI_Allgather
baseline. The JSON line carries the per-rank halo volume (values and peers).

K products y = A x are timed between barriers (max over ranks); rank 0 prints
one JSON line. Strong scaling (fixed matrix). --device cpu runs the same flow
on gloo ranks (tests).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", "--n", dest="n", type=int, default=1000)
    ap.add_argument("--mode", choices=["halo", "allgather"], default="halo")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda")
    ap.add_argument("--transport", choices=["rccl", "torch"], default="rccl")
    args = ap.parse_args()
    import torch

    import cme213x
    from cme213x.models.dist_spmv import RowPartitionedSpMV
    from cme213x.ops.spmv import laplacian, spmv
    from cme213x.parallel.comm import init_from_env

    comm = init_from_env(args.device)
    dev = torch.device("cuda", torch.cuda.current_device()) if args.device == "cuda" else torch.device("cpu")
    sync = (lambda: torch.cuda.synchronize(dev)) if args.device == "cuda" else (lambda: None)
    a = laplacian("5pt", args.n)
    rccl = None
    if args.device == "cuda" and comm.size > 1 and args.transport == "rccl" and args.mode == "halo":
        from cme213x.parallel.rccl import NativeRccl

        rccl = NativeRccl()
    op = RowPartitionedSpMV(a, comm, dev, mode=args.mode, rccl=rccl)
    sent, recvd, peers = op.halo_volume
    vol = torch.tensor([sent, peers], dtype=torch.float64, device=dev)
    comm.allreduce_(vol, "max")
    g = torch.Generator().manual_seed(0)
    x = torch.rand(a.ncols, generator=g)
    xl = op.local_slice(x).to(dev)
    y = op(xl)
    # correctness against the single-device product (rows of this rank)
    ref = spmv(a, x)[op.lo:op.hi]
    err = torch.tensor([float((y.cpu() - ref).abs().max())], device=dev)
    comm.allreduce_(err, "max")
    for _ in range(args.warmup):
        op(xl)
    sync()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        op(xl)
    sync()
    t1 = time.perf_counter()
    comm.barrier()
    el = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    comm.allreduce_(el, "max")
    if rccl is not None:
        rccl.check()
        rccl.close()
    ms = float(el.item()) * 1e3 / args.steps
    if comm.rank == 0:
        gflops = 2 * a.nnz / ms / 1e6
        print(json.dumps({"metric": "SpMV GFLOP/s (5-pt Laplacian, row-partitioned, x exchange included)",
                          "value": round(gflops, 2), "unit": "GFLOP/s", "n_gpus": comm.size, "steps": args.steps,
                          "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "strong",
                          "config": {"rows": a.nrows, "nnz": a.nnz, "mode": args.mode, "device": args.device,
                                     "transport": "rccl-native" if rccl is not None else "torch.distributed"},
                          "max_halo_values_per_rank": int(vol[0].item()), "max_peers_per_rank": int(vol[1].item()),
                          "max_abs_err": float(err.item())}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
