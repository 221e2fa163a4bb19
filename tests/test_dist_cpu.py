"""Multi-process (gloo, CPU) tests of the distributed heat solver and the
communicator layer: the same code path the 8-GPU RCCL run uses."""
import numpy as np
import pytest
import torch

from dist_util import run_ranks


def _heat_rank(rank, world, method, sync, order, tblock=1, fma=False):
    import cme213x
    from cme213x.models.heat2d_dist import DistHeat
    from cme213x.parallel.comm import TorchComm
    from cme213x.utils.params import SimParams

    p = SimParams(nx=70, ny=104, iters=9, order=order, ic=5.0, bc=(1.0, 10.0, 3.0, 7.0), grid_method=method,
                  sync=sync, flavor="hw5")
    sim = DistHeat(p, TorchComm(), torch.float64, "cpu", variant="naive", tblock=tblock, fma=fma)
    # non-uniform initial condition (same on every rank, by global coords)
    for s in sim.subs.values():
        g, b = s.grid, s.blk
        B = g.H
        yy, xx = np.meshgrid(np.arange(b.ny) + b.y0, np.arange(b.nx) + b.x0, indexing="ij")
        ic = torch.from_numpy(np.sin(0.3 * xx) * np.cos(0.2 * yy) + 5.0)
        g.buf[:, B:B + b.ny, B:B + b.nx] = ic
    sim.exchange(sim._cur()).wait()
    sim.run(p.iters)
    s = next(iter(sim.subs.values()))
    B = s.grid.B
    return (s.blk.x0, s.blk.y0, s.grid.state()[B:B + s.blk.ny, B:B + s.blk.nx])


def _single(method, order, sync, fma=False):
    import cme213x
    from cme213x.models.heat2d_dist import DistHeat
    from cme213x.utils.params import SimParams

    p = SimParams(nx=70, ny=104, iters=9, order=order, ic=5.0, bc=(1.0, 10.0, 3.0, 7.0), grid_method=method,
                  sync=sync, flavor="hw5")
    sim = DistHeat(p, None, torch.float64, "cpu", variant="naive", fma=fma)
    g = sim.subs[0].grid
    B = g.B
    yy, xx = np.meshgrid(np.arange(p.ny), np.arange(p.nx), indexing="ij")
    g.buf[:, B:B + p.ny, B:B + p.nx] = torch.from_numpy(np.sin(0.3 * xx) * np.cos(0.2 * yy) + 5.0)
    sim.run(p.iters)
    return g.state()[B:-B, B:-B]


@pytest.mark.parametrize("method,sync,order,world,tblock",
                         [(1, True, 8, 2, 1), (1, False, 4, 2, 1), (2, False, 8, 4, 1), (2, True, 2, 4, 1),
                          (1, False, 8, 3, 2), (1, True, 4, 2, 2), (2, False, 8, 4, 2), (2, True, 2, 4, 2),
                          (2, False, 4, 6, 2), (1, False, 8, 3, 3), (2, True, 4, 4, 3), (1, False, 8, 2, 4),
                          (2, False, 2, 4, 4)])
@pytest.mark.parametrize("fma", [False, True])
def test_dist_heat_matches_single(method, sync, order, world, tblock, fma):
    parts = run_ranks(_heat_rank, world, (method, sync, order, tblock, fma))
    ref = _single(method, order, sync, fma)
    for x0, y0, st in parts:
        np.testing.assert_array_equal(st, ref[y0:y0 + st.shape[0], x0:x0 + st.shape[1]])


@pytest.mark.parametrize("method,world", [(1, 3), (2, 4), (2, 6)])
def test_deep_halo_exchange_fills_corners(method, world):
    """With 2B-deep halos every ghost cell of a subdomain (corners included)
    must hold the neighbouring owner's value after one exchange."""
    from cme213x.models.heat2d_dist import DistHeat
    from cme213x.utils.params import SimParams

    p = SimParams(nx=61, ny=47, order=4, ic=0.0, bc=(-1.0, -2.0, -3.0, -4.0), grid_method=method, flavor="hw5")
    sim = DistHeat(p, None, torch.float64, "cpu", local_ranks=list(range(world)), world=world, tblock=2)
    f = lambda y, x: 1000.0 * y + x  # noqa: E731  global field by global coords
    for s in sim.subs.values():
        g, b = s.grid, s.blk
        H = g.H
        yy, xx = np.meshgrid(np.arange(b.ny) + b.y0, np.arange(b.nx) + b.x0, indexing="ij")
        g.buf[g.cur, H:H + b.ny, H:H + b.nx] = torch.from_numpy(f(yy, xx))
    sim.exchange(sim._cur()).wait()
    for s in sim.subs.values():
        g, b = s.grid, s.blk
        H = g.H
        st = g.buf[g.cur, :g.gy, :g.gx].numpy()
        gy_ = np.arange(g.gy) - H + b.y0
        gx_ = np.arange(g.gx) - H + b.x0
        inside_y = (gy_ >= 0) & (gy_ < p.ny)
        inside_x = (gx_ >= 0) & (gx_ < p.nx)
        m = np.outer(inside_y, inside_x)
        yy, xx = np.meshgrid(gy_, gx_, indexing="ij")
        np.testing.assert_array_equal(st[m], f(yy, xx)[m])


def _collectives(rank, world):
    from cme213x.parallel.comm import TorchComm

    c = TorchComm()
    t = torch.tensor([float(rank + 1)])
    c.allreduce_(t)
    g = c.allgather(torch.tensor([rank]))
    b = c.broadcast_(torch.tensor([rank * 10]), src=1)
    sub = c.split(color=rank % 2)
    s = sub.allreduce_(torch.tensor([1.0]))
    a2a = c.alltoall(torch.arange(world, dtype=torch.float32) + 100 * rank)
    return (t.item(), g.tolist(), b.item(), sub.size, s.item(), a2a.tolist())


def test_collectives_gloo():
    out = run_ranks(_collectives, 4)
    for r, (ar, ag, bc, ssz, ss, a2a) in enumerate(out):
        assert ar == 10.0
        assert ag == [[0], [1], [2], [3]]
        assert bc == 10
        assert ssz == 2 and ss == 2.0
        assert a2a == [float(r + 100 * k) for k in range(4)]


def _dist_spmv_rank(rank, world, mode):
    import cme213x
    from cme213x.models.dist_spmv import RowPartitionedSpMV
    from cme213x.ops.spmv import random_csr, spmv
    from cme213x.parallel.comm import TorchComm

    a = random_csr(3000, 3000, 9, seed=4)
    x = torch.from_numpy(np.random.default_rng(0).standard_normal(3000).astype(np.float32))
    op = RowPartitionedSpMV(a, TorchComm(), "cpu", mode=mode)
    y = op(op.local_slice(x))
    ref = spmv(a, x)
    return (op.lo, op.hi, y.numpy(), ref.numpy()[op.lo:op.hi])


@pytest.mark.parametrize("mode", ["allgather", "halo"])
def test_row_partitioned_spmv_gloo(mode):
    for lo, hi, y, ref in run_ranks(_dist_spmv_rank, 4, (mode,)):
        np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-5)


def _banded_halo_rank(rank, world):
    import cme213x
    from cme213x.models.dist_spmv import RowPartitionedSpMV
    from cme213x.ops.spmv import laplacian, spmv
    from cme213x.parallel.comm import TorchComm

    n = 40
    a = laplacian("5pt", n)
    x = torch.from_numpy(np.random.default_rng(1).standard_normal(a.ncols).astype(np.float32))
    op = RowPartitionedSpMV(a, TorchComm(), "cpu", mode="halo")
    ys = [op(op.local_slice(x)).clone() for _ in range(3)]  # persistent buffers reused across calls
    ref = spmv(a, x).numpy()[op.lo:op.hi]
    return (rank, op.halo_volume, op.recv_peers, op.send_peers, [y.numpy() for y in ys], ref)


def test_row_partitioned_spmv_neighbour_only():
    """5-pt Laplacian, 6 ranks of grid rows: every rank talks to its row
    neighbours only and moves exactly one grid row of x each way (no padded
    all-to-all: the volume is the halo, not P x max halo)."""
    world, n = 6, 40
    for rank, (sent, recvd, peers), rp, sp, ys, ref in run_ranks(_banded_halo_rank, world):
        want = [q for q in (rank - 1, rank + 1) if 0 <= q < world]
        assert rp == want and sp == want
        assert sent == recvd <= 2 * n + 2 and peers == len(want)
        for y in ys:
            np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-5)


def _dense_matvec_rank(rank, world):
    import cme213x
    from cme213x.models.dist_spmv import block2d_matvec, colwise_matvec
    from cme213x.parallel.comm import TorchComm

    c = TorchComm()
    n = 64
    g = torch.Generator().manual_seed(0)
    A = torch.randn(n, n, generator=g, dtype=torch.float64)
    x = torch.randn(n, generator=g, dtype=torch.float64)
    nb = n // world
    ycol = colwise_matvec(c, A[:, rank * nb:(rank + 1) * nb].contiguous(), x[rank * nb:(rank + 1) * nb].contiguous())
    q = 2
    row, col = divmod(rank, q)
    bs = n // q
    Ab = A[row * bs:(row + 1) * bs, col * bs:(col + 1) * bs].contiguous()
    xd = x[row * bs:(row + 1) * bs].clone() if row == col else None
    y2 = block2d_matvec(c, Ab, xd)
    ref = A @ x
    ok_col = torch.allclose(ycol, ref[rank * nb:(rank + 1) * nb])
    ok_2d = (y2 is None) or torch.allclose(y2, ref[row * bs:(row + 1) * bs])
    return ok_col, ok_2d


def test_dense_matvecs_gloo():
    for ok_col, ok_2d in run_ranks(_dense_matvec_rank, 4):
        assert ok_col and ok_2d


def _p2p_collectives_rank(rank, world):
    import cme213x
    from cme213x.parallel.collectives import ring_allgather, tree_broadcast, tree_reduce_sum
    from cme213x.parallel.comm import TorchComm

    c = TorchComm()
    g = ring_allgather(c, torch.tensor([rank * 1.0, rank + 0.5]))
    b = tree_broadcast(c, torch.tensor([float(rank)] * 3), root=2)
    r = tree_reduce_sum(c, torch.tensor([float(rank + 1)]), root=1)
    return g.tolist(), b.tolist(), r.item()


def test_p2p_collectives_gloo():
    world = 5
    out = run_ranks(_p2p_collectives_rank, world)
    for rank, (g, b, r) in enumerate(out):
        assert g == [[k * 1.0, k + 0.5] for k in range(world)]
        assert b == [2.0] * 3
        if rank == 1:
            assert r == sum(range(1, world + 1))


def _dist_scan_rank(rank, world, seed):
    import cme213x
    from cme213x.parallel.comm import TorchComm
    from cme213x.parallel.dist_scan import dist_scan, dist_segmented_scan

    rng = np.random.default_rng(seed)
    n = 10_007
    x = rng.integers(-5, 6, n).astype(np.float32)  # small integers: fp32 sums are exact
    flags = (rng.random(n) < 0.001).astype(np.uint8)
    flags[0] = 1
    cuts = sorted(rng.choice(np.arange(1, n), world - 1, replace=False).tolist())
    bounds = [0] + cuts + [n]
    lo, hi = bounds[rank], bounds[rank + 1]
    c = TorchComm()
    inc = dist_scan(torch.from_numpy(x[lo:hi].copy()), c)
    exc = dist_scan(torch.from_numpy(x[lo:hi].copy()), c, exclusive=True)
    seg = dist_segmented_scan(torch.from_numpy(x[lo:hi].copy()), torch.from_numpy(flags[lo:hi].copy()), c)
    return lo, hi, inc.numpy(), exc.numpy(), seg.numpy()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_dist_scan_gloo(world):
    rng = np.random.default_rng(7)
    n = 10_007
    x = rng.integers(-5, 6, n).astype(np.float32)
    flags = (rng.random(n) < 0.001).astype(np.uint8)
    flags[0] = 1
    inc = np.cumsum(x.astype(np.float64))
    seg = np.empty(n)
    acc = 0.0
    for i in range(n):
        acc = x[i] if flags[i] else acc + x[i]
        seg[i] = acc
    for lo, hi, yi, ye, ys in run_ranks(_dist_scan_rank, world, (7,)):
        np.testing.assert_array_equal(yi, inc[lo:hi])
        np.testing.assert_array_equal(ye, (inc - x)[lo:hi])
        np.testing.assert_array_equal(ys, seg[lo:hi])


def _dist_spmvscan_rank(rank, world):
    import cme213x
    from cme213x.models.spmv_scan import generate
    from cme213x.parallel.comm import TorchComm
    from cme213x.parallel.dist_scan import DistSpmvScan

    prob = generate(20_000, 40, 500, 4, seed=3)  # few long segments: most straddle shards
    a, xx, f = DistSpmvScan.shard(prob, rank, world)
    d = DistSpmvScan(a, xx, f, TorchComm())
    out = d.run(prob.iters)
    n = prob.n
    return n * rank // world, out.numpy()


@pytest.mark.parametrize("world", [2, 4])
def test_dist_spmv_scan_gloo(world):
    from cme213x.models.spmv_scan import errors, generate, reference_solution

    prob = generate(20_000, 40, 500, 4, seed=3)
    ref = reference_solution(prob)
    parts = sorted(run_ranks(_dist_spmvscan_rank, world), key=lambda t: t[0])
    b = np.concatenate([p for _, p in parts])
    e = errors(ref, b)
    assert e["relL2"] < 1e-5, e


def _ckpt_rank(rank, world, directory, tblock, use_async=False):
    import cme213x
    from cme213x.models.heat2d_dist import DistHeat
    from cme213x.parallel.comm import TorchComm
    from cme213x.utils.params import SimParams

    p = SimParams(nx=64, ny=48, iters=8, order=4, ic=5.0, bc=(1.0, 10.0, 3.0, 7.0), grid_method=2, sync=False,
                  flavor="hw5")
    c = TorchComm()
    full = DistHeat(p, c, torch.float64, "cpu", variant="naive", tblock=tblock)
    for s in full.subs.values():
        g, b = s.grid, s.blk
        yy, xx = np.meshgrid(np.arange(b.ny) + b.y0, np.arange(b.nx) + b.x0, indexing="ij")
        g.buf[:, g.H:g.H + b.ny, g.H:g.H + b.nx] = torch.from_numpy(np.sin(0.3 * xx) * np.cos(0.2 * yy) + 5.0)
    full.exchange(full._cur()).wait()
    full.run(5)
    if use_async:  # the run continues while the files are written
        w = full.checkpoint_async(directory)
        full.run(6)
        assert len(w.wait()) == len(full.subs)
    else:
        full.checkpoint(directory)
        full.run(6)
    # a fresh solver resumes from the checkpoint and must land on the same state
    resumed = DistHeat(p, c, torch.float64, "cpu", variant="naive", tblock=tblock)
    resumed.restore(directory)
    assert resumed.iteration == 5
    resumed.run(6)
    a = next(iter(full.subs.values())).grid
    b = next(iter(resumed.subs.values())).grid
    B = a.B
    return bool(np.array_equal(a.state()[B:-B, B:-B], b.state()[B:-B, B:-B]))


@pytest.mark.parametrize("tblock,use_async", [(1, False), (2, False), (4, False), (2, True)])
def test_dist_heat_checkpoint_restart_gloo(tmp_path, tblock, use_async):
    assert all(run_ranks(_ckpt_rank, 4, (str(tmp_path), tblock, use_async)))


def _setup_agreement_rank(rank, world, fail_rank, fail_step):
    import torch.distributed as dist

    from cme213x.models.heat2d_dist import native_setup_agreement

    calls = []

    def agree(ok):
        calls.append(ok)
        t = torch.tensor([1.0 if ok else 0.0])
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item() == 1.0)

    def load_lib():
        if rank == fail_rank and fail_step == "lib":
            raise OSError("faked library-load failure")

    opened = []

    def open_transport():
        if rank == fail_rank and fail_step == "transport":
            raise RuntimeError("faked transport failure")
        opened.append(True)
        return "handle"

    ok, handle = native_setup_agreement(agree, load_lib, open_transport, f"rank {rank}", "ipc")
    # a collective after the setup: a rank left alone in one would hang here
    t = torch.tensor([float(len(calls))])
    dist.all_reduce(t)
    return ok, len(calls), len(opened), float(t.item())


@pytest.mark.parametrize("fail_rank,fail_step", [(1, "lib"), (0, "lib"), (1, "transport"), (-1, "")])
def test_native_setup_every_rank_falls_back_together(fail_rank, fail_step):
    """one rank failing to load the native library (or to open the
    transport) makes EVERY rank fall back, after the same number of
    agreement collectives -- no rank enters the self-test alone."""
    parts = run_ranks(_setup_agreement_rank, 2, (fail_rank, fail_step))
    oks = {p[0] for p in parts}
    assert oks == {fail_rank < 0}
    assert parts[0][1] == parts[1][1]  # same number of agree() calls on both ranks
    if fail_step == "lib":
        assert all(p[2] == 0 for p in parts)  # nobody opened a transport


def _chain_rank(rank, world, scenario):
    """The native transport chain (RCCL -> IPC -> Python loop) with faked
    transports: which kind every rank ends on, and its agreement count."""
    import torch.distributed as dist

    from cme213x.models.heat2d_dist import choose_native_transport

    calls, released = [], []

    def agree(ok):
        calls.append(ok)
        t = torch.tensor([1.0 if ok else 0.0])
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item() == 1.0)

    def open_transport(kind):
        if kind == "rccl" and scenario == "rccl_setup" and rank == 1:
            raise RuntimeError("faked ncclCommInitRank failure")
        if scenario == "all_setup":
            raise RuntimeError("faked transport failure")
        return f"{kind}-handle"

    def selftest(kind, handle, fused):
        if scenario == "rccl_selftest" and kind == "rccl" and rank == 0:
            return False
        if scenario == "ipc_fused" and kind == "ipc" and fused and rank == 1:
            raise TimeoutError("faked gate timeout")
        return True

    def release(kind, handle):
        released.append(kind)

    kind, handle, fused, attempts = choose_native_transport(["rccl", "ipc"], agree, lambda: None, open_transport,
                                                            selftest, release, (True, False), f"rank {rank}")
    t = torch.tensor([float(len(calls))])
    dist.all_reduce(t)  # a rank left alone in a collective would hang here
    return kind, handle, fused, attempts, len(calls), released


@pytest.mark.parametrize("scenario,want,fused", [("none", "rccl", True), ("rccl_setup", "ipc", True),
                                                 ("rccl_selftest", "ipc", True), ("ipc_fused", "rccl", True),
                                                 ("all_setup", None, False)])
def test_native_transport_chain_gloo(scenario, want, fused):
    """RCCL failing its setup (on one rank) or its bitwise
    self-test moves EVERY rank to the IPC transport together, with the same
    number of agreement collectives; a failed self-test releases the RCCL
    handle first; with no transport left every rank ends on the Python
    loop. (ipc_fused: RCCL passes, so IPC is never tried.)"""
    parts = run_ranks(_chain_rank, 2, (scenario,))
    kinds = {p[0] for p in parts}
    assert kinds == {want}, parts
    assert parts[0][4] == parts[1][4]  # same number of agree() calls
    assert parts[0][3] == parts[1][3]  # same attempt record on every rank
    assert parts[0][2] == fused
    if scenario == "rccl_setup":
        assert [a["result"] for a in parts[0][3]] == ["setup", "ok"]
        assert parts[0][1] == "ipc-handle"
        assert parts[0][5] == ["rccl"] and parts[1][5] == []  # rank 0's opened communicator aborted
    if scenario == "rccl_selftest":
        assert [a["result"] for a in parts[0][3]] == ["selftest", "ok"]
        assert all(p[5] == ["rccl"] for p in parts)  # RCCL released on both ranks before IPC opened
    if scenario == "all_setup":
        assert [a["result"] for a in parts[0][3]] == ["setup", "setup"]
