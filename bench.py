#!/usr/bin/env python3
"""Flagship benchmark: distributed 2-D heat-diffusion stencil, 16384^2 global
grid, order 8, fp32, RCCL halo exchange over xGMI (BASELINE.json config #5).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1
launched under torch.distributed.run (one rank per GPU). W untimed steps, then
EXACTLY K timed steps bracketed by barrier + synchronize, max over ranks; rank
0 prints one JSON line.

A "step" is one full timestep of the global grid: the FTCS sweep of every
point plus the halo exchange between neighbouring ranks (1-D stripes, async
mode: deep interior overlapped with the exchange, borders after it). With
``--tblock n`` (default ``auto_tblock``: 4 with the wave-pipelined pass) n
timesteps are fused into one HBM pass (temporal blocking)
and each exchange moves nB-deep halos; K timed steps are still exactly K
timesteps (a K that is not a multiple of n ends with a shorter pass).

Metric convention: effective GB/s = points x 72 B (17 taps + 1
store, fp32) per iteration / time -- the convention the reference's 240 GB/s
(hw2, 4000^2, order 8, LDS kernel, Fermi) is quoted in. Also reported: the
minimum-traffic HBM rate (8 B/pt) and its % of 8 TB/s per GPU. Strong scaling:
the global grid is fixed as N grows.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BASELINE_GBPS = 239.7  # heat 4000^2 order 8 LDS kernel, 48.07 ms / 10 iters, 72 B/pt


def selftest(comm, dev, args) -> bool:
    """Bitwise self-test of the N = 1 timed path (the native multi-pass
    driver, ``heat_run``): a 1024^2 problem with a non-uniform interior runs
    2*tblock+1 timesteps (whole passes plus a tail) and must equal, bit for
    bit, the same number of single steps of the same arithmetic. (N > 1: the solver's own
    :meth:`DistHeat.enable_native` self-test of the native loop against the
    torch.distributed loop.)"""
    import torch

    from cme213x.models.heat2d_dist import DistHeat
    from cme213x.utils.params import SimParams

    iters = 2 * args.tblock + 1
    p = SimParams(nx=1024, ny=1024, iters=iters, order=args.order, ic=5.0, bc=(0.0, 10.0, 3.0, 7.0),
                  grid_method=args.method, sync=(args.mode == "sync"), flavor="hw5")
    a = DistHeat(p, comm, torch.float32, dev, variant=args.variant, tblock=args.tblock, fma=args.fma_arg,
                 kernel=args.kernel)
    b = DistHeat(p, comm, torch.float32, dev, variant=args.variant, tblock=1, fma=args.fma_arg)
    # non-uniform interior so a misplaced pass boundary changes the answer
    for sim in (a, b):
        s = next(iter(sim.subs.values()))
        g, B = s.grid, s.grid.H
        yy = torch.arange(s.blk.ny, device=dev, dtype=torch.float32).view(-1, 1) + s.blk.y0
        xx = torch.arange(s.blk.nx, device=dev, dtype=torch.float32).view(1, -1) + s.blk.x0
        g.buf[:, B:B + s.blk.ny, B:B + s.blk.nx] = 5.0 + torch.sin(0.05 * xx) * torch.cos(0.03 * yy)
        sim.exchange(sim._cur()).wait()
    a.run(iters)
    for _ in range(iters):
        b.step()
    b.finish()
    torch.cuda.synchronize(dev)
    sa, sb = next(iter(a.subs.values())).grid, next(iter(b.subs.values())).grid
    B = sa.B
    va, vb = sa.view()[B:B + sa.ny, B:B + sa.nx], sb.view()[B:B + sb.ny, B:B + sb.nx]
    return bool(torch.equal(va, vb))


def auto_tblock(points_per_rank: int, kernel: str = "pipe") -> int:
    """Timesteps per pass for a subdomain size and pass kernel.

    streamN (one wave holds every step): each wave re-computes 2(NS-1)B
    warm-up rows, a per-pass cost fixed by the resident wave count; 3 steps
    win at 16384^2 / 1, 2, 4 ranks, 4 steps at 8 ranks (profiles/
    dist_rank_r2.md).
    pipe (steps split across the waves of a workgroup, csrc/hip/heat_pipe.hip):
    4 steps win at every rank count (profiles/heat_pipe_r2.md)."""
    if kernel == "pipe":
        return 4
    return 4 if points_per_rank <= 16384 * 16384 // 8 else 3


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--spinup", type=float, default=0.25,
                    help="seconds of untimed solver work before the W warmup steps (GPU clock ramp / first touch; "
                         "with 10 warmup steps alone the first timed steps run ~8%% slow)")
    ap.add_argument("--n", "--grid", dest="n", type=int, default=16384, help="global grid edge (points)")
    ap.add_argument("--order", type=int, default=8)
    ap.add_argument("--method", type=int, default=1, help="1 = 1-D stripes, 2 = 2-D blocks")
    ap.add_argument("--mode", choices=["async", "sync"], default="async")
    ap.add_argument("--variant", default="stream")
    ap.add_argument("--fma", type=int, choices=[0, 1], default=None,
                    help="1 = --arith fma, 0 = --arith exact")
    ap.add_argument("--arith", choices=["fma", "exact", "fast"], default=None,
                    help="stencil arithmetic (default fast): fma = FMA-contracted (what nvcc emits for the "
                         "reference's GPU kernel), exact = no contraction (bitwise = the CPU oracle), fast = "
                         "reassociated (CFL folded into the weights, symmetric pairs summed first: 17 instead of "
                         "20 flop-instructions per point; within the reference's 10-ULP criterion of exact, "
                         "bitwise = the CPU fast oracle); profiles/heat_fast_r4.md has the A/B on one box")
    ap.add_argument("--tblock", type=int, choices=[0, 1, 2, 3, 4], default=0,
                    help="timesteps per halo exchange / per HBM pass (n > 1 = temporal blocking, nB-deep halos); "
                         "0 = by subdomain size (auto_tblock)")
    ap.add_argument("--kernel", choices=["pipe", "streamn"], default="pipe",
                    help="3-4 step pass kernel: pipe = timesteps split across the waves of a workgroup "
                         "(csrc/hip/heat_pipe.hip); streamn = every step in one wave (heat2d.hip)")
    ap.add_argument("--native", choices=["auto", "on", "off"], default="auto",
                    help="multi-GPU: run the K-step loop in C++ over a native communicator (auto: after a "
                         "bitwise self-test against the torch.distributed loop)")
    ap.add_argument("--schedule", choices=["auto", "events"], default="auto",
                    help="native loop: auto = fused one-launch passes where the native loop allows them (falls back "
                         "to events if the self-test fails); events = schedule 0 (border / comm / interior streams)")
    ap.add_argument("--transport", choices=["rccl", "ipc"], default="rccl",
                    help="native halo transport: rccl = grouped ncclSend/Recv; ipc = peers' memory mapped "
                         "with hipIpcOpenMemHandle, pulled by a kernel over xGMI")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu = dry run of the multi-rank control flow on gloo + the OpenMP backend "
                         "(tests; never the reported number)")
    ap.add_argument("--ic", choices=["uniform", "random", "both"], default="both",
                    help="uniform: the reference's IC 5.0 only (the headline value); both: also time the same K "
                         "steps from a random-init field (ms_per_step_random)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal only: every rank on cuda:0 with a gloo control plane and the IPC transport "
                         "(exercises the multi-rank flow on a 1-GPU box; the number is not a scaling result)")
    args = ap.parse_args()
    if args.share_gpu:
        args.transport = "ipc"
    if args.arith is None:
        args.arith = "fast" if args.fma is None else ("fma" if args.fma else "exact")
    args.fma = int(args.arith == "fma")
    # the solver's `fma` argument: False exact, True FMA-contracted, "fast" reassociated
    args.fma_arg = {"exact": False, "fma": True, "fast": "fast"}[args.arith]

    import torch
    import torch.distributed as dist

    import cme213x  # noqa: F401 - the package alias
    from cme213x.models.heat2d import bytes_per_point
    from cme213x.models.heat2d_dist import DistHeat
    from cme213x.parallel.comm import init_from_env
    from cme213x.utils.params import SimParams

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank per GPU under "
              "torch.distributed.run with --nproc-per-node equal to --gpus", file=sys.stderr)
        return 2
    on_gpu = args.device == "cuda"
    comm = init_from_env(args.device, backend="gloo" if args.share_gpu else None, share_gpu=args.share_gpu)
    rank = comm.rank
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")

    def sync():
        if on_gpu:
            torch.cuda.synchronize(dev)

    if args.tblock == 0:
        args.tblock = auto_tblock(args.n * args.n // max(1, comm.size), args.kernel)
    p = SimParams(nx=args.n, ny=args.n, iters=args.steps, order=args.order, ic=5.0, bc=(0.0, 10.0, 0.0, 10.0),
                  grid_method=args.method, sync=(args.mode == "sync"), flavor="hw5")

    sim = DistHeat(p, comm, torch.float32, dev, variant=args.variant if on_gpu else "naive", tblock=args.tblock,
                   fma=args.fma_arg, kernel=args.kernel,
                   native=("off" if (not on_gpu or comm.size == 1) else args.native))
    # N > 1: the solver's own native-loop setup -- transport, then a bitwise
    # self-test against the torch.distributed loop (fused schedule first,
    # schedule 0 if that fails); every rank agrees, "auto" falls back to the
    # torch.distributed loop, "on" raises
    try:
        info = sim.enable_native(args.transport if not args.share_gpu else "ipc", fused=args.schedule == "auto")
    except RuntimeError as e:
        print(f"bench.py: --native on but the native loop failed ({e})", file=sys.stderr)
        return 3
    if args.share_gpu and info["loop"] != "native":
        print("bench.py: --share-gpu needs the native IPC loop, which failed", file=sys.stderr)
        return 3
    use_native = info["loop"] == "native"
    init_state = {(s.blk.x0, s.blk.y0): s.grid.buf.clone() for s in sim.subs.values()} if on_gpu else {}

    def run(k):
        sim.run(k)

    # the timed path's bitwise self-test at N = 1 (N > 1: enable_native above)
    selftest_ok = info["selftest"] if use_native else None
    if on_gpu and comm.size == 1:
        selftest_ok = selftest(comm, dev, args)

    def barrier_sync():
        sync()
        comm.barrier()
        sync()

    # spin-up: untimed passes on a scratch copy of the solver until `spinup`
    # seconds have elapsed (rank 0 decides the count; all ranks run it).
    # First, one run of every pass length (1..tblock steps) so every kernel
    # the warmup/timed loops launch has been loaded: a first launch loads its
    # code object (~5 ms with the GPU idle), after which the clocks take ~10 ms
    # to recover -- the slow timed passes of a 20-step run (gpurun trace,
    # profiles/bench_driver_cmd_r3.md)
    def spin_up(fn) -> int:
        """untimed passes of `fn` until `spinup` seconds have elapsed (the
        clocks drop in the host-side gaps between measurements; every timed
        figure starts from the same warm state); returns the steps run"""
        if not (on_gpu and args.spinup > 0):
            return 0
        n = 0
        t_end = time.perf_counter() + args.spinup
        while True:
            fn(args.tblock * 4)
            sync()
            n += args.tblock * 4
            done = torch.tensor([1.0 if time.perf_counter() >= t_end else 0.0], device=dev)
            comm.allreduce_(done, "min")
            if done.item() >= 1.0:
                return n

    spin = 0
    if on_gpu and args.spinup > 0:
        for k in range(1, args.tblock + 1):
            run(k)
            spin += k
        spin += spin_up(run)
        for s in sim.subs.values():  # restart from the initial condition
            s.grid.buf.copy_(init_state[(s.blk.x0, s.blk.y0)])
            s.grid.iteration = 0
        sim.iteration = 0

    def timed(k, fn=None):
        """W warmup steps, then exactly k timed steps between barrier +
        synchronize; max over ranks (s). The native loop checks its in-kernel
        waits (and RCCL's asynchronous errors) at the end of every run and
        raises instead of reporting a number."""
        fn = fn or run
        fn(args.warmup)
        barrier_sync()
        t0 = time.perf_counter()
        fn(k)
        sync()
        t1 = time.perf_counter()
        comm.barrier()
        elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
        comm.allreduce_(elapsed, "max")
        return float(elapsed.item())

    def sane() -> bool:
        """the solution must stay finite and within the BC/IC bounds"""
        local = next(iter(sim.subs.values())).grid
        st = local.buf[local.cur]
        bad = torch.tensor([float(~torch.isfinite(st).all()) + float(st.abs().max() > 1e3)], device=dev)
        comm.allreduce_(bad, "max")
        return bool(bad.item() == 0)

    secs = timed(args.steps)
    sanity_ok = sane()

    # N = 1: the distributed native schedule (cme_heat_dist_run, the loop the
    # N > 1 points run, exchange off) on the same grid and the same uniform
    # initial field, so the N = 1 point of a scaling curve can be read
    # against the same schedule (same spin-up and warmup as the headline run:
    # with 5 warmup steps right after the host-side gap the first passes ran
    # at a lower clock, 0.166 vs 0.1315 ms/step in bench_dist_rank.py)
    secs_dist1 = None
    if on_gpu and comm.size == 1 and args.kernel == "pipe":
        run_d = lambda k: sim.run_native(k, transport=2)  # noqa: E731
        spin_up(run_d)
        for s in sim.subs.values():
            s.grid.buf.copy_(init_state[(s.blk.x0, s.blk.y0)])
        secs_dist1 = timed(args.steps, run_d)
        sim.gate_check()

    # the same K steps from a random-init field (BASELINE.json: "synthetic
    # random-init inputs"): uniform(0, 10) interior, seeded per rank, same
    # BCs. The pass is issue/power bound, and random data toggles more bits
    # than the reference's uniform IC, so this is the slower figure.
    # The same spin-up as the uniform run, on the random field (the power
    # controller settles to the data's switching activity over ~10 ms: a
    # 20-step window right after the switch from the uniform field ran 0.20
    # ms/step, steady state 0.16-0.17; profiles/heat_random_ic_r4.md), then
    # the field is reset to the random init and timed.
    secs_random = None
    if on_gpu and args.ic in ("both", "random"):
        gen = torch.Generator(device=dev)
        gen.manual_seed(1234 + rank)
        rand_init = {}
        for s in sim.subs.values():
            g, H = s.grid, s.grid.H
            g.buf[:, H:H + g.ny, H:H + g.nx] = torch.rand((g.ny, g.nx), generator=gen, device=dev) * 10.0
            rand_init[(s.blk.x0, s.blk.y0)] = g.buf.clone()
        spin_up(run)
        for s in sim.subs.values():
            s.grid.buf.copy_(rand_init[(s.blk.x0, s.blk.y0)])
        sim.exchange(sim._cur()).wait()
        sync()
        secs_random = timed(args.steps)
        sanity_ok = sanity_ok and sane()

    if use_native:
        sch = DistHeat.schedule()
        schedule = sch["schedule"] + ("" if sch["probe"] == "not run" else f" (queue probe {sch['probe']})")
    else:
        schedule = "python passes" if comm.size > 1 else "heat_run (one native call)"
    pts = args.n * args.n
    bpp = bytes_per_point(args.order, torch.float32)
    from cme213x.utils import tuning

    pipe_vw = tuning.get("pipe_vw") if on_gpu else 0
    eff = pts * bpp * args.steps / secs / 1e9
    # min HBM traffic: one read + one write of the grid per PASS (a pass
    # advances `tblock` timesteps)
    hbm = pts * 8 / args.tblock * args.steps / secs / 1e9
    ms = secs * 1e3 / args.steps
    if rank == 0:
        rec = {
            "metric": "effective GB/s (2-D heat stencil, order 8, fp32, 72 B/pt reference model)",
            "value": round(eff, 2),
            "unit": "GB/s",
            "n_gpus": args.gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(eff / BASELINE_GBPS, 2),
            "dtype": "fp32",
            "data": "synthetic (uniform IC 5.0, Dirichlet BCs 0/10/0/10)",
            "config": {
                "model": f"heat2d-{args.n}x{args.n}-order{args.order} (BASELINE.json config #5)",
                "global_batch": pts,
                "seq_len": 1,
                "parallelism": f"{'stripes' if args.method == 1 else 'blocks'}{args.gpus}-{args.mode}",
                "variant": (args.variant if args.tblock == 1 else
                            f"{'pipe' if args.kernel == 'pipe' and args.tblock >= 3 else 'stream'}{args.tblock} "
                            f"({args.tblock} steps/pass)") + f" {args.arith}",
                "kernel": args.kernel,
                # pipelined fp32 pass: 8 columns per lane at order 8 (tuning knob pipe_vw = 4 / 8 forces one width)
                "lane_columns": ({4: 4, 8: 8}.get(pipe_vw, 8 if args.order == 8 else 4)
                                 if args.kernel == "pipe" and args.tblock >= 3 else 4),
                "fma": bool(args.fma),
                "arith": {"fma": "FMA-contracted", "exact": "exact (no contraction)",
                          "fast": "reassociated (folded CFL weights, pair sums; <= 10 ULP of exact)"}[args.arith],
                "tblock": args.tblock,
                "device": args.device,
                "rehearsal_shared_gpu": bool(args.share_gpu),
                "loop": f"native-{info['transport']}" if use_native else ("torch.distributed" if comm.size > 1
                                                                            else "single (native multi-pass)"),
                "transport": (info["transport"] if use_native else ("torch.distributed" if comm.size > 1 else "none")),
                "schedule": schedule,
            },
            "hbm_GBps_min_traffic": round(hbm, 1),
            "pct_peak_hbm_per_gpu": round(100.0 * hbm / args.gpus / 8000.0, 1),
            "gpoints_per_s": round(pts * args.steps / secs / 1e9, 2),
            # a failed bitwise self-test of the timed path invalidates the record
            "sanity_ok": bool(sanity_ok and selftest_ok is not False),
            "selftest": selftest_ok,
            "native_selftest": (info["selftest"] if comm.size > 1 and on_gpu else None),
            "spinup_steps": spin,
        }
        if secs_random is not None:
            rec["ms_per_step_random"] = round(secs_random * 1e3 / args.steps, 4)
            rec["value_random"] = round(pts * bpp * args.steps / secs_random / 1e9, 2)
            rec["data_random"] = "synthetic random-init interior, uniform(0, 10), seed 1234 + rank, same BCs"
        if secs_dist1 is not None:
            rec["ms_per_step_dist_schedule"] = round(secs_dist1 * 1e3 / args.steps, 4)
        print(json.dumps(rec), flush=True)
    sim.close_native()
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
