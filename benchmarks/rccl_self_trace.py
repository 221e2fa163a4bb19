#!/usr/bin/env python3
"""Periodic world-1 run of the native distributed heat loop over RCCL
self-sends (every halo piece an ncclSend/ncclRecv to rank 0 itself), for a
rocprofv3 kernel trace of RCCL's kernels beside the fused gated pass.

    rocprofv3 --kernel-trace -d gpurun_out/rccl_self -- python3 benchmarks/rccl_self_trace.py
    python3 scripts/overlap.py gpurun_out/rccl_self --a heat_pipe --b nccl

Prints one JSON line: ms per step, the schedule that ran, and whether the
final state equals the periodic CPU-oracle-equivalent single-step run on the
GPU (bitwise)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--method", type=int, default=2)
    ap.add_argument("--schedule", choices=["fused", "events"], default="fused")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist

    import cme213x  # noqa: F401
    from cme213x.models.heat2d_dist import DistHeat
    from cme213x.parallel.comm import TorchComm
    from cme213x.parallel.rccl import NativeRccl
    from cme213x.utils.params import SimParams

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29533"), RANK="0",
                      WORLD_SIZE="1", LOCAL_RANK="0")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    periodic = (args.method == 2, True)
    p = SimParams(nx=args.n, ny=args.n, order=8, iters=args.steps, ic=5.0, bc=(0.0, 10.0, 0.0, 10.0),
                  grid_method=args.method, sync=False, flavor="hw5")
    mk = lambda tb: DistHeat(p, TorchComm(), torch.float32, "cuda:0", tblock=tb, fma=True,  # noqa: E731
                             kernel="pipe" if tb > 1 else "streamn", periodic=periodic)
    sim, ref = mk(4), mk(1)
    gen = torch.Generator(device="cuda").manual_seed(7)
    for d in (sim, ref):
        s = next(iter(d.subs.values()))
        g, H = s.grid, s.grid.H
        gen.manual_seed(7)
        g.buf[:, H:H + g.ny, H:H + g.nx] = torch.rand((g.ny, g.nx), generator=gen, device="cuda") * 10.0
        d.exchange(d._cur()).wait()
    rc = NativeRccl()
    fused = args.schedule == "fused"
    sim.run_native(8, rc, fused=fused)  # warm-up (RCCL connection setup, code objects)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sim.run_native(args.steps, rc, fused=fused)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / args.steps
    sim.gate_check()
    rc.check()
    sch = DistHeat.schedule()
    ref.run(args.steps + 8)  # Python loop, single FMA steps, local self-copies
    torch.cuda.synchronize()
    own = lambda d: (lambda s: s.grid.buf[s.grid.cur, s.grid.H:s.grid.H + s.grid.ny,  # noqa: E731
                                          s.grid.H:s.grid.H + s.grid.nx])(next(iter(d.subs.values())))
    rec = {"bench": "rccl_self_periodic", "n": args.n, "method": args.method, "periodic": list(periodic),
           "steps": args.steps, "ms_per_step": round(ms, 4), "schedule": sch, "bitwise_vs_single_steps":
           bool(torch.equal(own(sim), own(ref)))}
    print(json.dumps(rec), flush=True)
    rc.close()
    dist.destroy_process_group()
    return 0 if rec["bitwise_vs_single_steps"] else 1


if __name__ == "__main__":
    sys.exit(main())
