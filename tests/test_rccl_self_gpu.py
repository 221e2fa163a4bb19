"""Real RCCL halo traffic on one GPU: periodic decompositions at world 1.

With a periodic axis and one block along it, every halo piece of the native
loop's RCCL transport is an ``ncclSend``/``ncclRecv`` to the caller's own
rank -- the grouped batch of ``post_exchange_rccl`` (``csrc/hip/
dist_heat.hip``) moves real bytes (rows straight from / into the grid,
column and corner blocks through the packed staging buffer), under schedule
0, the fused gated schedule (RCCL's own kernels on the comm stream beside
the spinning border workgroups) and with ``GPU_MAX_HW_QUEUES=1``. Every
result is compared bit for bit with the periodic CPU oracle (``DistHeat`` on
the OpenMP backend, itself checked against plain-PyTorch fp64 in
``test_periodic.py``). Reference: the halo posting and overlap of
``hw/hw5/2dHeat_solution.cpp:413-465, 537-628``.
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from dist_util import REPO, free_port, init_single_rank, run_ranks


def _setup_single():
    import torch.distributed as dist

    init_single_rank("nccl")


def _params(method, iters=9):
    from cme213x.utils.params import SimParams

    return SimParams(nx=333, ny=270, order=8, iters=iters, sync=False, grid_method=method, ic=5.0,
                     bc=(1.0, 10.0, 3.0, 7.0), flavor="hw5")


def _set_ic(sim, dtype):
    for s in sim.subs.values():
        g, b = s.grid, s.blk
        H = g.H
        yy, xx = np.meshgrid(np.arange(b.ny) + b.y0, np.arange(b.nx) + b.x0, indexing="ij")
        ic = torch.from_numpy(np.sin(0.3 * xx) * np.cos(0.2 * yy) + 5.0).to(dtype)
        g.buf[:, H:H + b.ny, H:H + b.nx] = ic.to(g.device)
    sim.exchange(sim._cur()).wait()


def _owned(sim):
    s = next(iter(sim.subs.values()))
    g, H = s.grid, s.grid.H
    return g.buf[g.cur, H:H + g.ny, H:H + g.nx].cpu().double().numpy()


def _oracle(method, periodic, dtype, fma):
    from cme213x.models.heat2d_dist import DistHeat

    p = _params(method)
    ref = DistHeat(p, None, dtype, "cpu", variant="naive", fma=fma, periodic=periodic)
    _set_ic(ref, dtype)
    ref.run(p.iters)
    return _owned(ref)


# (grid_method, periodic, tblock, fma, dtype, kernel, fused allowed)
CASES = [
    (1, (False, True), 1, False, "float32", "streamn", True),   # rows only, single steps
    (1, (False, True), 4, True, "float32", "pipe", True),       # rows, fused gated schedule
    (1, (False, True), 4, True, "float32", "pipe", False),      # rows, schedule 0
    (2, (True, True), 2, True, "float32", "streamn", True),     # rows + packed columns + corners
    (2, (True, True), 4, True, "float32", "pipe", True),        # ... under the fused schedule
    (2, (True, True), 4, False, "float32", "pipe", False),
    (2, (True, False), 3, True, "float64", "pipe", True),       # columns only, fp64, fused
    (1, (False, True), 4, True, "float64", "pipe", True),
    (1, (False, True), 4, "fast", "float32", "pipe", True),     # reassociated arithmetic, fused
    (2, (True, True), 4, "fast", "float32", "pipe", True),
    (2, (True, True), 3, "fast", "float32", "pipe", False),
]


def _arith_name(fma):
    return "fast" if fma == "fast" else ("fma" if fma else "exact")


def _run_case(case, group=None):
    """One case on an nccl world-1 group (default: the default group):
    (owned state, schedule)."""
    from cme213x.models.heat2d_dist import DistHeat
    from cme213x.parallel.comm import TorchComm
    from cme213x.parallel.rccl import NativeRccl

    method, periodic, tblock, fma, dt, kernel, fused = case
    dtype = getattr(torch, dt)
    p = _params(method)
    sim = DistHeat(p, TorchComm(group), dtype, "cuda:0", tblock=tblock, fma=fma, kernel=kernel, periodic=periodic)
    _set_ic(sim, dtype)
    rc = NativeRccl(group)
    sim.run_native(5, rc, fused=fused)
    sim.run_native(4, rc, fused=fused)  # two calls: halos and gate counters carried across calls
    torch.cuda.synchronize()
    sim.gate_check()
    rc.check()
    sch = DistHeat.schedule()
    rc.close()
    return _owned(sim), sch


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"m{c[0]}-p{int(c[1][0])}{int(c[1][1])}-t{c[2]}-"
                                                         f"{_arith_name(c[3])}-{c[4]}-{c[5]}"
                                                         f"{'-fused' if c[6] else '-sched0'}")
def test_rccl_self_peer_halo_bitwise(gpu, case):
    import torch.distributed as dist

    _setup_single()
    try:
        got, sch = _run_case(case)
    finally:
        dist.destroy_process_group()
    method, periodic, tblock, fma, dt, kernel, fused = case
    want = _oracle(method, periodic, getattr(torch, dt), fma)
    assert np.array_equal(got, want), f"max |diff| {np.abs(got - want).max()} ({sch})"
    if fused and kernel == "pipe" and tblock >= 3:
        assert sch == {"schedule": "fused", "probe": "passed"}, sch
    elif not fused:
        assert sch["schedule"] == "events", sch


def _queue_rank(rank, world, cases):
    import torch.distributed as dist

    torch.cuda.set_device(0)
    g = dist.new_group(backend="nccl")  # the helper's default group is gloo
    return [(_run_case(c, g), os.environ.get("GPU_MAX_HW_QUEUES")) for c in cases]


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_rccl_self_peer_fused_one_hw_queue(gpu, monkeypatch):
    """GPU_MAX_HW_QUEUES=1 in a fresh process (set before its first GPU call):
    RCCL's kernels, the gate signal and the gated pass may share a hardware
    queue; the queue probe decides, and the result stays bitwise either way."""
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "1")
    cases = [c for c in CASES if c[5] == "pipe" and c[6]]
    (out,) = run_ranks(_queue_rank, 1, (cases,), timeout=240)
    for case, ((got, sch), q) in zip(cases, out):
        assert q == "1"
        want = _oracle(case[0], case[1], getattr(torch, case[4]), case[3])
        assert np.array_equal(got, want), f"{case}: max |diff| {np.abs(got - want).max()} ({sch})"
        assert sch["probe"] in ("passed", "failed") and (sch["schedule"] == "fused") == (sch["probe"] == "passed")


@pytest.mark.gpu
def test_native_rccl_p2p_self_sends(gpu):
    """NativeRccl.p2p (the distributed SpMV's halo batch) to the caller's own
    rank: the k-th send meets the k-th receive, byte for byte, for several
    sizes in one group; plus allreduce / allgather on the same communicator."""
    import torch.distributed as dist

    from cme213x.parallel.rccl import NativeRccl

    _setup_single()
    try:
        rc = NativeRccl()
        gen = torch.Generator(device="cuda").manual_seed(5)
        srcs = [torch.rand(n, device="cuda", generator=gen) for n in (1, 777, 65536, 1 << 20)]
        dsts = [torch.full_like(x, -1.0) for x in srcs]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        rc.p2p([("send", x, 0) for x in srcs] + [("recv", y, 0) for y in dsts], stream=side)
        torch.cuda.current_stream().wait_stream(side)
        for x, y in zip(srcs, dsts):
            assert torch.equal(x, y)
        # the same communicator's collectives
        v = torch.arange(6, dtype=torch.float64, device="cuda")
        assert torch.equal(rc.allgather(v)[0], v)
        rc.check()
        rc.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_run_uses_native_rccl_self_peer(gpu):
    """DistHeat.run with native="on" and transport rccl at world 1: the
    enable_native self-test runs the RCCL batch (fused, then schedule 0 if
    needed), then run() takes the native path and checks its waits."""
    import torch.distributed as dist

    from cme213x.models.heat2d_dist import DistHeat
    from cme213x.parallel.comm import TorchComm

    _setup_single()
    try:
        p = _params(1)
        sim = DistHeat(p, TorchComm(), torch.float32, "cuda:0", tblock=4, fma=True, kernel="pipe",
                       periodic=(False, True), native="on")
        _set_ic(sim, torch.float32)
        info = sim.enable_native("rccl")
        assert info["loop"] == "native" and info["transport"] == "rccl" and info["selftest"] is True
        sim.run(p.iters)
        torch.cuda.synchronize()
        assert sim.native_info["schedule"] in ("fused", "events")
        got = _owned(sim)
        sim.close_native()
    finally:
        dist.destroy_process_group()
    assert np.array_equal(got, _oracle(1, (False, True), torch.float32, True))


@pytest.mark.gpu
def test_gate_timeout_raises_from_run(gpu, monkeypatch):
    """A fused border wait that gives up must raise from DistHeat.run (the
    sticky pinned word is read after the final sync), not leave a silently
    wrong state: one poll allowed (tuning knob dist_gate_spins=1) against
    an exchange held back 20 ms (dist_fake_xchg_us)."""
    from cme213x.models.heat2d_dist import DistHeat

    p = _params(1, iters=12)
    sim = DistHeat(p, None, torch.float32, "cuda:0", tblock=4, fma=True, kernel="pipe", periodic=(False, True),
                   native="on")
    _set_ic(sim, torch.float32)
    info = sim.enable_native()
    assert info["loop"] == "native" and info["transport"] == "loopback" and info["fused_allowed"]
    sim.run(8)
    assert sim.native_info["schedule"] == "fused"
    from cme213x.utils import tuning

    with tuning.override(dist_gate_spins=1, dist_fake_xchg_us=20000):
        with pytest.raises(RuntimeError, match="timed out"):
            sim.run(12)
    sim.run(4)  # the sticky word was cleared by the check: later runs report only their own waits


@pytest.mark.gpu
def test_run_hw5_fused_selftest_failure_falls_back_to_schedule0(gpu, tmp_path, monkeypatch, capsys):
    """run_hw5's native setup with the fused gate forced to give up: the
    fused self-test fails (its timed-out wait raises), the retry on schedule
    0 (no in-kernel gate) passes bit for bit, and the run goes on natively
    with the fused schedule off -- the fallback chain that lived in bench.py,
    now in the solver."""
    from cme213x.models.heat2d_dist import run_hw5

    from cme213x.utils import tuning

    prm = tmp_path / "params.in"
    prm.write_text("333 270\n1 1\n1\n12\n8\n5\n1\n0\n1 10 3 7\n")
    monkeypatch.chdir(tmp_path)
    with tuning.override(dist_gate_spins=1, dist_fake_xchg_us=20000):
        res = run_hw5(str(prm), None, torch.float32, "cuda:0", write_files=False, tblock=4, fma=True,
                      kernel="pipe", native="on", periodic=(False, True))
    info = res["sim"].native_info
    assert info["loop"] == "native" and info["fused_allowed"] is False and info["schedule"] == "events", info
    out = capsys.readouterr().out
    assert "self-test raised" in out and "fused schedule off" in out, out


@pytest.mark.gpu
@pytest.mark.parametrize("arith", ["--fma", "--fast"])
def test_heat2d_mpi_ranks_uses_native_loop(gpu, tmp_path, monkeypatch, capsys, arith):
    """heat2d_mpi --ranks 2 on the GPU runs the native loop (loopback
    transport) after its self-test and logs it (FMA-contracted and
    reassociated arithmetic)."""
    from cme213x.__main__ import main

    monkeypatch.chdir(tmp_path)
    (tmp_path / "params.in").write_text("300 200\n1 1\n1\n9\n8\n5\n1\n0\n0 10 0 10\n")
    assert main(["heat2d_mpi", "params.in", "--ranks", "2", "--float", arith, "--tblock", "4",
                 "--kernel", "pipe"]) == 0
    out = capsys.readouterr().out
    assert "time loop: native (loopback transport, bitwise self-test passed" in out, out
    assert "native schedule: events" in out, out  # two subdomains in one process: schedule 0


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_heat2d_mpi_share_gpu_torchrun_ipc(gpu, tmp_path):
    """The reference's `mpirun -np 2 2dHeat params.in` as two torchrun
    processes on one GPU (--share-gpu: gloo control plane, IPC halo
    transport): the native loop runs after its self-test, the per-rank
    dumps equal the single-process run's."""
    (tmp_path / "params.in").write_text("300 200\n1 1\n1\n9\n8\n5\n1\n0\n0 10 0 10\n")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONPATH=REPO)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO, "cme213x_cli.py"), "heat2d_mpi",
           "params.in", "--share-gpu", "--float", "--fma", "--tblock", "4", "--kernel", "pipe"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=tmp_path)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "time loop: native (ipc transport, bitwise self-test passed" in out.stdout, out.stdout
    assert "9 iterations on a 300 by 200 grid took:" in out.stdout
    one = tmp_path / "one"
    one.mkdir()
    (one / "params.in").write_text((tmp_path / "params.in").read_text())
    o2 = subprocess.run([sys.executable, os.path.join(REPO, "cme213x_cli.py"), "heat2d_mpi", "params.in", "--ranks",
                         "2", "--float", "--fma", "--tblock", "1", "--native", "off"], capture_output=True,
                        text=True, timeout=240, env=env, cwd=one)
    assert o2.returncode == 0, o2.stderr[-3000:]
    for r in range(2):
        assert (tmp_path / f"grid{r}_final.txt").read_text() == (one / f"grid{r}_final.txt").read_text()
