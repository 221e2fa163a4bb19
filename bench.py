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


HBM_PEAK_GBPS = 8000.0  # MI355X nominal


def _cold_ms(dev, sets, fn, reps=7, rounds=2):
    """Median ms per call of ``fn(set)`` with the operand sets visited
    round-robin (``rounds`` passes over all of them per timed batch), so every
    call's operands were last touched >= 512 MB of other traffic ago and come
    from HBM, not the 256 MB Infinity Cache. Eager launches, event-timed."""
    import torch

    for s in sets:
        fn(s)
    torch.cuda.synchronize(dev)
    calls = rounds * len(sets)
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(calls):
            fn(sets[i % len(sets)])
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / calls)
    return sorted(ts)[reps // 2]


def _warm_ms(dev, fn, calls=20, reps=7):
    """Median ms per call of back-to-back calls on ONE operand (part of it
    may hit the Infinity Cache: an upper bound, kept for continuity)."""
    import torch

    fn()
    torch.cuda.synchronize(dev)
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(calls):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / calls)
    return sorted(ts)[reps // 2]


def bench_primitives(dev) -> dict:
    """BASELINE.json configs #2-#4 on this rank's GPU, each behind an oracle
    check (``*_ok``), all cache-defeated: every figure cycles through >= 3
    operand sets of >= 768 MB in total, round-robin, so no call reads what
    the 256 MB Infinity Cache kept from the previous one.

    * ``copy_GBps``: the framework's 16-B copy under the same protocol (256
      MiB -> 256 MiB, read + write) -- the in-run ceiling every streaming
      figure is also quoted against (``*_pct_copy``; my-refs/
      MatrixTranspose.pdf p.19 uses copy as the transpose ceiling).
    * #2: the 8192^2 fp32 LDS-tiled transpose (production ``vec`` and the
      padded 32x32 ``lds_pad`` of the lecture ladder; ``torch.equal`` against
      ``x.t()``).
    * #3: the 2^26 fp32 scan (decoupled look-back and Blelloch) and reduction
      on uniform(0, 1) data, checked against a float64 reference within a
      tolerance, and on Bernoulli(0.2) data (every prefix an integer < 2^24:
      bitwise against float64 in any association order; ``*_bernoulli_ms``);
      my-refs/scan.pdf p.16 Table 2.
    * #4: SpMV on the 1M-row 5-point Laplacian in CSR (``auto``: lane-per-row
      for its short regular rows) and ELL, hipGraph-replayed, against a
      float64 reference (refs/Bell SC 2009.pdf §4.2).

    Effective GB/s counts the bytes the algorithm must move (copy, transpose,
    scan: read + write; reduction: read). ``*_warm_ms`` keeps the earlier
    one-operand back-to-back figure of transpose / scan / reduce (an upper
    bound: part of it hits the Infinity Cache)."""
    import torch

    from cme213x.ops import scan as sc
    from cme213x.ops.elementwise import copy_
    from cme213x.ops.spmv import laplacian, prepare, spmv
    from cme213x.ops.transpose import transpose

    out = {}
    nsets = 3
    g = torch.Generator(device=dev).manual_seed(2)

    # in-run copy ceiling: 3 x (256 MiB in + 256 MiB out)
    n = 1 << 26
    cs = [(torch.rand(n, device=dev, generator=g), torch.empty(n, device=dev)) for _ in range(nsets)]
    copy_(cs[0][1], cs[0][0])
    ok = bool(torch.equal(cs[0][1], cs[0][0]))
    ms = _cold_ms(dev, cs, lambda s: copy_(s[1], s[0]))
    copy_gbps = 2 * n * 4 / ms / 1e6
    out.update(copy_ms=round(ms, 4), copy_GBps=round(copy_gbps, 1), copy_pct_peak=round(100 * copy_gbps / HBM_PEAK_GBPS, 1),
               copy_ok=ok)
    del cs

    def rate(prefix, ms, nbytes):
        gbps = nbytes / ms / 1e6
        out[f"{prefix}_ms"] = round(ms, 4)
        out[f"{prefix}_GBps"] = round(gbps, 1)
        out[f"{prefix}_pct_peak"] = round(100 * gbps / HBM_PEAK_GBPS, 1)
        out[f"{prefix}_pct_copy"] = round(100 * gbps / copy_gbps, 1)

    # config #2: transpose 8192^2 fp32, 3 x (256 MiB in + 256 MiB out)
    n = 8192
    ts = [(torch.rand(n, n, device=dev, generator=g), torch.empty(n, n, device=dev)) for _ in range(nsets)]
    for v in ("vec", "lds_pad"):
        ok = True
        for x, y in ts:
            transpose(x, v, y)
            ok = ok and bool(torch.equal(y, x.t()))
        rate(f"transpose_{v}", _cold_ms(dev, ts, lambda s: transpose(s[0], v, s[1])), 2 * n * n * 4)
        out[f"transpose_{v}_ok"] = ok
        x0, y0 = ts[0]
        out[f"transpose_{v}_warm_ms"] = round(_warm_ms(dev, lambda: transpose(x0, v, y0)), 4)
    del ts

    # config #3: 2^26 fp32 scan + reduction, 3 x (256 MiB in + 256 MiB out)
    n = 1 << 26
    uni = [(torch.rand(n, device=dev, generator=g), torch.empty(n, device=dev)) for _ in range(nsets)]
    ref = torch.cumsum(uni[0][0].double(), 0)
    bern = [((torch.rand(n, device=dev, generator=g) < 0.2).float(), torch.empty(n, device=dev)) for _ in range(nsets)]
    bref = torch.cumsum(bern[0][0].double(), 0)
    assert float(bref[-1]) < 2 ** 24
    bref32 = bref.float()
    for algo in ("lookback", "blelloch"):
        x0, y0 = uni[0]
        sc.scan(x0, False, y0, algo)
        # fp32 prefix sums to ~3.4e7: |err| <= 1e-5 x prefix + 1 (the carry
        # chain across 4096-16384-element tiles adds one rounding per tile)
        err = (y0.double() - ref).abs()
        ok = bool((err <= 1e-5 * ref.abs() + 1.0).all())
        b0, by0 = bern[0]
        sc.scan(b0, False, by0, algo)
        ok = ok and bool(torch.equal(by0, bref32))
        rate(f"scan_{algo}", _cold_ms(dev, uni, lambda s: sc.scan(s[0], False, s[1], algo)), 8 * n)
        out[f"scan_{algo}_max_rel_err"] = float((err / ref.abs().clamp_min(1.0)).max())
        out[f"scan_{algo}_ok"] = ok
        out[f"scan_{algo}_bernoulli_ms"] = round(_cold_ms(dev, bern, lambda s: sc.scan(s[0], False, s[1], algo)), 4)
        out[f"scan_{algo}_warm_ms"] = round(_warm_ms(dev, lambda: sc.scan(b0, False, by0, algo)), 4)
    r = float(sc.reduce(uni[0][0], "sum", "vector"))
    rel = abs(r - float(ref[-1])) / float(ref[-1])
    ok = rel <= 1e-5 and float(sc.reduce(bern[0][0], "sum", "vector")) == float(bref[-1])
    rate("reduce", _cold_ms(dev, uni, lambda s: sc.reduce(s[0], "sum", "vector")), 4 * n)
    out["reduce_rel_err"] = rel
    out["reduce_ok"] = ok
    out["reduce_bernoulli_ms"] = round(_cold_ms(dev, bern, lambda s: sc.reduce(s[0], "sum", "vector")), 4)
    x0 = bern[0][0]
    out["reduce_warm_ms"] = round(_warm_ms(dev, lambda: sc.reduce(x0, "sum", "vector")), 4)
    del uni, bern, ref, bref, bref32

    # config #4: 1M x 1M 5-point Laplacian, CSR / ELL, Infinity Cache defeated
    A = laplacian("5pt", 1000)
    xh = torch.rand(A.ncols, generator=torch.Generator().manual_seed(3))
    rows = torch.repeat_interleave(torch.arange(A.nrows), torch.diff(A.rp.long()))
    ref = torch.zeros(A.nrows, dtype=torch.float64).index_add_(0, rows, A.val.double() * xh.double()[A.col.long()])
    for fmt in ("csr", "ell"):
        _, m = prepare(A, fmt, dev)
        yy = spmv(m, xh.to(dev))
        ok = bool(torch.allclose(yy.cpu().double(), ref, rtol=1e-5, atol=1e-5))
        nbytes = sum(t.numel() * t.element_size() for t in vars(m).values() if isinstance(t, torch.Tensor))
        nbytes += 4 * (A.ncols + A.nrows)
        sets = []
        for _ in range(max(1, -(-(768 << 20) // nbytes))):
            mm = type(m)(**{k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in vars(m).items()})
            sets.append((mm, xh.to(dev), torch.empty(A.nrows, device=dev)))
        calls = 2 * len(sets)

        def cold():
            for i in range(calls):
                mm, xx, yo = sets[i % len(sets)]
                spmv(mm, xx, yo)

        cold()
        torch.cuda.synchronize(dev)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            cold()
        ms = _warm_ms(dev, gr.replay, calls=1, reps=5) / calls
        out[f"spmv_{fmt}_ms"] = round(ms, 5)
        out[f"spmv_{fmt}_GFLOPs"] = round(2 * A.nnz / ms / 1e6, 1)
        out[f"spmv_{fmt}_GBps"] = round(nbytes / ms / 1e6, 1)
        out[f"spmv_{fmt}_pct_copy"] = round(100 * nbytes / ms / 1e6 / copy_gbps, 1)
        out[f"spmv_{fmt}_ok"] = ok
        del gr, sets
    torch.cuda.empty_cache()
    out["primitives_data"] = ("synthetic, seeded, cache-defeated (3 operand sets of 512 MB each for copy / transpose / "
                              "scan, 256 MB each for reduce, >= 768 MB for SpMV, visited round-robin): transpose "
                              "uniform(0,1); scan / reduce uniform(0,1) fp32 (float64 reference, tolerance) and "
                              "Bernoulli(0.2) (exact prefixes, bitwise; *_bernoulli_ms); SpMV 5-pt Laplacian of a "
                              "1000^2 grid, x uniform(0,1); *_warm_ms: one operand back to back")
    return out


def bench_cpu_transpose() -> dict:
    """BASELINE.json config #1: the 1024^2 fp32 transpose on the CPU / OpenMP
    backend (runs without a GPU; my-refs/cuda_many_cores.pdf pp.14-17: input
    M[i] = i), blocked, into a preallocated output. Median of single calls
    after warm-up, with the thread count and OpenMP wait policy recorded and
    a ``torch.equal`` check against ``x.t()``."""
    import torch

    from cme213x.ops.transpose import transpose
    from cme213x.utils import cpu_runtime

    n = 1024
    x = torch.arange(n * n, dtype=torch.float32).view(n, n)
    y = torch.empty_like(x)
    info = cpu_runtime.info()
    for _ in range(10):
        transpose(x, "lds", y)
    ok = bool(torch.equal(y, x.t()))
    ts = []
    for _ in range(100):
        t0 = time.perf_counter()
        transpose(x, "lds", y)
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    ms = ts[len(ts) // 2]
    return {"cpu_transpose_1024_ms": round(ms, 4), "cpu_transpose_1024_min_ms": round(ts[0], 4),
            "cpu_transpose_1024_GBps": round(2 * n * n * 4 / ms / 1e6, 2), "cpu_transpose_1024_ok": ok,
            "cpu_threads": info["threads"], "cpu_omp_wait_policy": info["wait_policy"]}


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
                    help="stencil arithmetic (default fast for the fp32 order-8 pipelined GPU pass, else fma): "
                         "fma = FMA-contracted (what nvcc emits for the reference's GPU kernel; <= 8 ULP of exact "
                         "after 200 steps on random data), exact = no contraction (bitwise = the CPU oracle), "
                         "fast = reassociated (CFL folded into weights that sum to exactly one, symmetric pairs "
                         "summed first: 17 instead of 20 flop-instructions per point; bitwise = the CPU fast "
                         "oracle; <= 9 ULP of exact after whole runs: profiles/heat_arith_ulp_r5.md)")
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
    ap.add_argument("--transport", choices=["auto", "rccl", "ipc", "rccl,ipc"], default="auto",
                    help="native halo transport: rccl = grouped ncclSend/Recv; ipc = peers' memory mapped "
                         "with hipIpcOpenMemHandle, pulled by a kernel over xGMI; auto = rccl, then ipc if RCCL "
                         "fails its setup or bitwise self-test, then the torch.distributed loop")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu = dry run of the multi-rank control flow on gloo + the OpenMP backend "
                         "(tests; never the reported number)")
    ap.add_argument("--ic", choices=["uniform", "random", "both"], default="both",
                    help="both (default): time K steps from the reference's uniform IC 5.0 (value_uniform) and from "
                         "a random-init field (the headline value); uniform: the uniform IC only")
    ap.add_argument("--no-primitives", dest="primitives", action="store_false",
                    help="N = 1: skip the BASELINE configs #2-#4 (transpose / scan / SpMV) measured after the stencil")
    ap.add_argument("--no-arith-compare", dest="arith_compare", action="store_false",
                    help="N = 1: skip timing the other arithmetic (fma <-> fast) on the same fields")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal only: every rank on cuda:0 with a gloo control plane and the IPC transport "
                         "(exercises the multi-rank flow on a 1-GPU box; the number is not a scaling result)")
    args = ap.parse_args()
    if args.share_gpu:
        args.transport = "ipc"
    if args.arith is None:
        if args.fma is None:
            fast_ok = args.order == 8 and args.kernel == "pipe" and args.device == "cuda" and args.tblock in (0, 3, 4)
            args.arith = "fast" if fast_ok else "fma"
        else:
            args.arith = "fma" if args.fma else "exact"
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
        info = sim.enable_native("ipc" if args.share_gpu else (None if args.transport == "auto" else args.transport),
                                 fused=args.schedule == "auto")
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

    # N = 1: the other arithmetic on the same two fields with the same
    # protocol, in the same record: the reassociated pass next to
    # the FMA-contracted headline (round 4's default; it leaves the 10-ULP
    # criterion on random data, so it is no longer the headline), or FMA next
    # to an explicitly chosen fast headline
    secs_cmp = {}
    cmp_arith = {"fma": "fast", "fast": "fma"}.get(args.arith)
    if on_gpu and comm.size == 1 and cmp_arith and args.arith_compare and args.order == 8 and args.kernel == "pipe":
        sim_f = DistHeat(p, comm, torch.float32, dev, variant=args.variant, tblock=args.tblock,
                         fma={"fma": True, "fast": "fast"}[cmp_arith], kernel=args.kernel)
        run_f = sim_f.run
        fields = {"uniform": init_state}
        if secs_random is not None:
            fields["random"] = rand_init
        for name, st in fields.items():
            for s in sim_f.subs.values():
                s.grid.buf.copy_(st[(s.blk.x0, s.blk.y0)])
            spin_up(run_f)
            for s in sim_f.subs.values():
                s.grid.buf.copy_(st[(s.blk.x0, s.blk.y0)])
            sync()
            secs_cmp[name] = timed(args.steps, run_f)
        del sim_f
        torch.cuda.empty_cache()

    prims = {}
    if comm.size == 1 and args.primitives:
        # config #1 (CPU / OpenMP, no GPU involved)
        try:
            prims.update(bench_cpu_transpose())
        except Exception as e:  # noqa: BLE001 - recorded in the JSON
            prims["cpu_transpose_error"] = f"{type(e).__name__}: {e}"[:300]
    if on_gpu and comm.size == 1 and args.primitives:
        # configs #2-#4 are extra keys: a failure there is recorded, and the
        # stencil line still prints
        try:
            prims.update(bench_primitives(dev))
        except Exception as e:  # noqa: BLE001 - any op failure, reported in the JSON
            prims["primitives_error"] = f"{type(e).__name__}: {e}"[:300]

    if use_native:
        sch = DistHeat.schedule()
        schedule = sch["schedule"] + ("" if sch["probe"] == "not run" else f" (queue probe {sch['probe']})")
    else:
        schedule = "python passes" if comm.size > 1 else "heat_run (one native call)"
    pts = args.n * args.n
    bpp = bytes_per_point(args.order, torch.float32)
    from cme213x.utils import tuning

    pipe_vw = tuning.get("pipe_vw") if on_gpu else 0
    # the headline is the random-init field (BASELINE.json: "synthetic
    # random-init inputs"); the reference's uniform IC is
    # value_uniform / ms_per_step_uniform
    secs_uniform = secs
    headline_random = secs_random is not None
    if headline_random:
        secs = secs_random
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
            "data": ("synthetic random-init interior, uniform(0, 10), seed 1234 + rank, Dirichlet BCs 0/10/0/10"
                     if headline_random else "synthetic (uniform IC 5.0, Dirichlet BCs 0/10/0/10)"),
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
                "arith": {"fma": "FMA-contracted (<= 10 ULP of exact: 8 at 4000^2 x 10, 7 at 2048^2 x 200 random)",
                          "exact": "exact (no contraction)",
                          "fast": "reassociated (folded CFL weights summing to exactly one, pair sums; <= 10 ULP "
                                  "of exact: 9 at 4000^2 x 10 random, 7 at 2048^2 x 200 random)"}[args.arith],
                "tblock": args.tblock,
                "device": args.device,
                "rehearsal_shared_gpu": bool(args.share_gpu),
                "loop": f"native-{info['transport']}" if use_native else ("torch.distributed" if comm.size > 1
                                                                            else "single (native multi-pass)"),
                "transport": (info["transport"] if use_native else ("torch.distributed" if comm.size > 1 else "none")),
                "schedule": schedule,
                # the native transport chain as tried (rccl -> ipc -> torch.distributed loop)
                "transport_attempts": info.get("attempts", []),
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
        if headline_random:
            rec["ms_per_step_uniform"] = round(secs_uniform * 1e3 / args.steps, 4)
            rec["value_uniform"] = round(pts * bpp * args.steps / secs_uniform / 1e9, 2)
            rec["data_uniform"] = "the reference's uniform IC 5.0, Dirichlet BCs 0/10/0/10"
        for name, sf in secs_cmp.items():
            rec[f"ms_per_step_{name}_{cmp_arith}"] = round(sf * 1e3 / args.steps, 4)
        if secs_dist1 is not None:
            rec["ms_per_step_dist_schedule"] = round(secs_dist1 * 1e3 / args.steps, 4)
        rec.update(prims)
        print(json.dumps(rec), flush=True)
    sim.close_native()
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
