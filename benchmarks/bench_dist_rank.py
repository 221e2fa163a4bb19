#!/usr/bin/env python3
"""Compute side of the strong-scaling flagship on ONE GPU: time one rank's
per-step schedule (deep interior + border strips, tblock fused steps per pass)
for the subdomain an N-GPU run gives each rank, with the halo exchange
replaced by a no-op. ms/step x N vs the N=1 time shows how much of ideal
strong scaling the compute schedule itself keeps (launch overhead, thin
border strips, halo redundancy) -- independent of RCCL.

    python benchmarks/bench_dist_rank.py [--n 16384] [--world 1 2 4 8] [--method 1]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--world", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--method", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--fma", type=int, default=1)
    ap.add_argument("--arith", choices=["fma", "exact", "fast"], default=None,
                    help="stencil arithmetic (overrides --fma); fast = reassociated (csrc/hip/heat_fast.hip)")
    ap.add_argument("--tblock", type=int, default=3, help="timesteps per exchange / HBM pass (1-4)")
    ap.add_argument("--native", type=int, default=1, help="1: native loop (null transport); 0: Python loop")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--kernel", default="streamn", choices=["streamn", "pipe"],
                    help="3-4 step pass kernel: streamN or the wave-pipelined pass")
    ap.add_argument("--sync", action="store_true",
                    help="sync mode: exchange, then every row of the subdomain in one region (no separate border "
                         "strips; with the no-op exchange this bounds what folding the borders in can gain)")
    ap.add_argument("--tune", nargs="*", default=[],
                    help="tuning knobs name=value (cme213x.utils.tuning), e.g. pipe_per_cu=6 pipe_vw=4")
    args = ap.parse_args()
    import torch

    import cme213x
    from cme213x.models.heat2d_dist import DistHeat
    from cme213x.parallel.comm import Comm, Pending
    from cme213x.utils.params import SimParams

    class NullComm(Comm):
        """Pretends to be rank r of W; exchanges complete immediately."""

        def __init__(self, rank, size):
            self.rank, self.size = rank, size

        def exchange(self, ops):
            return Pending()

        def allreduce_(self, t, op="sum"):
            return t

        def barrier(self):
            pass

    from cme213x.utils import tuning

    knobs = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in args.tune}
    for k, v in knobs.items():
        tuning.set(k, v)
    base = None
    for w in args.world:
        rank = w // 2 if w > 1 else 0  # an inner rank: two neighbours
        p = SimParams(nx=args.n, ny=args.n, order=8, grid_method=args.method, sync=args.sync, flavor="hw5")
        arith = args.arith or ("fma" if args.fma else "exact")
        fma_arg = {"exact": False, "fma": True, "fast": "fast"}[arith]
        sim = DistHeat(p, NullComm(rank, w), torch.float32, "cuda", tblock=args.tblock, fma=fma_arg,
                      kernel=args.kernel)

        def run(k):
            if args.native:
                sim.run_native(k, transport=2)
            else:
                sim.run(k)

        run(30)
        torch.cuda.synchronize()
        times = []
        for _ in range(args.reps):  # median of reps (clock / thermal noise is +-5 % per rep)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(args.steps)
            e1.record()
            e1.synchronize()
            times.append(e0.elapsed_time(e1) / args.steps)
        ms = sorted(times)[len(times) // 2]
        base = base or ms * w
        print(json.dumps({"world": w, "rank": rank, "method": args.method, "sync": args.sync, "native": args.native,
                          "tblock": args.tblock,
                          "arith": arith,
                          "kernel": args.kernel, "tune": knobs,
                          "reps": args.reps,
                          "ms_per_step": round(ms, 4),
                          "compute_scaling_eff": round(base / (ms * w), 3)}), flush=True)
        del sim
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
