"""LDS-resident tile pass for small grids (csrc/hip/heat_tile.hip): N steps
per pass must equal N single steps bit for bit (exact and FMA arithmetic,
fp32 and fp64, orders 2/4/8, grids that are not multiples of the 64 x 64
tile), through one pass and through heat_run's multi-pass driver (with a
shorter tail pass)."""
import numpy as np
import pytest
import torch

from cme213x.models.heat2d import HeatGrid
from cme213x.ops.stencil import heat_run, heat_step, heat_tile
from cme213x.utils.params import SimParams


def _grid(nx, ny, order, dtype, dev, seed=3):
    p = SimParams(nx=nx, ny=ny, order=order, ic=5.0, bc=(1.0, 10.0, 3.0, 7.0))
    g = HeatGrid(p, dtype, dev)
    B = g.B
    gen = torch.Generator().manual_seed(seed)
    ic = (torch.rand((ny, nx), generator=gen, dtype=torch.float64) * 10.0).to(dtype)
    g.buf[:, B:B + ny, B:B + nx] = ic.to(dev)
    return g


def _single_steps(g, n, fma):
    a, b = g.buf[0].clone(), g.buf[1].clone()
    for _ in range(n):
        heat_step(a, b, g.interior, g.order, g.xcfl, g.ycfl, "fma" if fma else "stream")
        a, b = b, a
    return a


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("order", [2, 4, 8])
@pytest.mark.parametrize("ns", [1, 2, 3, 4])
@pytest.mark.parametrize("fma", [False, True])
@pytest.mark.parametrize("shape", [(1000, 1000), (130, 77), (64, 64), (333, 190)])
def test_tile_pass_bitwise(gpu, dtype, order, ns, fma, shape):
    nx, ny = shape
    g = _grid(nx, ny, order, dtype, gpu)
    want = _single_steps(g, ns, fma)
    out = g.buf[1].clone()
    heat_tile(g.buf[0], out, g.interior, g.order, g.xcfl, g.ycfl, ns, fma)
    torch.cuda.synchronize()
    assert torch.equal(out, want), f"max |diff| {(out - want).abs().max().item()}"


@pytest.mark.gpu
@pytest.mark.parametrize("variant,fma", [("tile2", False), ("tile3_fma", True), ("tile4", False),
                                         ("tile4_fma", True)])
@pytest.mark.parametrize("iters", [1, 7, 10])
def test_tile_heat_run_bitwise(gpu, variant, fma, iters):
    g = _grid(1000, 1000, 8, torch.float64, gpu, seed=5)
    want = _single_steps(g, iters, fma)
    a, b = g.buf[0].clone(), g.buf[1].clone()
    out = heat_run(a, b, g.interior, g.order, g.xcfl, g.ycfl, iters, variant)
    torch.cuda.synchronize()
    assert torch.equal(out, want)


def test_tile_variants_refuse_single_step_api():
    g = _grid(40, 30, 8, torch.float64, "cpu")
    with pytest.raises(ValueError):
        heat_step(g.buf[0], g.buf[1], g.interior, 8, g.xcfl, g.ycfl, "tile2")
    assert np.isfinite(g.state()).all()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("fma", [False, True])
def test_hw5_default_path_uses_tile_pass(gpu, fma, dtype):
    """The hw5 driver's automatic choice on a small single-grid run (fp64, and
    fp32 since round 4) is the tile pass (four steps per pass), bitwise equal
    to the CPU oracle's single steps (exact or FMA) -- the reference's 1000^2
    shape, 13 steps (three passes and a one-step tail)."""
    from cme213x.models.heat2d_dist import DistHeat

    p = SimParams(nx=1000, ny=1000, order=8, iters=13, ic=3.0, bc=(0.0, 10.0, 0.0, 10.0), flavor="hw5")
    sim = DistHeat(p, None, dtype, gpu, tblock="auto", kernel="auto", fma=fma)
    assert sim.kernel == "tile" and sim.tblock == 4 and sim.solo()
    ref = DistHeat(p, None, dtype, "cpu", variant="naive", fma=fma)
    for d in (sim, ref):
        (s,) = d.subs.values()
        g, H = s.grid, s.grid.H
        yy, xx = np.meshgrid(np.arange(1000), np.arange(1000), indexing="ij")
        g.buf[:, H:H + 1000, H:H + 1000] = torch.from_numpy(np.sin(0.01 * xx) * np.cos(0.02 * yy) + 3.0).to(
            device=g.device, dtype=dtype)
    sim.run(13)
    ref.run(13)
    torch.cuda.synchronize()
    assert np.array_equal(sim.gather_global(), ref.gather_global())


def test_auto_kernel_small_grids_pick_tile_except_fast():
    from cme213x.models.heat2d_dist import auto_kernel

    for dt in (torch.float32, torch.float64):
        assert auto_kernel(dt, 1000 * 1000, 4, solo=True) == "tile"
        assert auto_kernel(dt, 2000 * 2000, 4, solo=True) == "pipe"
        assert auto_kernel(dt, 1000 * 1000, 4, solo=False) == "pipe"
    assert auto_kernel(torch.float32, 1000 * 1000, 4, solo=True, fast=True) == "pipe"
    assert auto_kernel(torch.float64, 1000 * 1000, 4, solo=True, order=4) == "tile"
    for dt, o in ((torch.float32, 4), (torch.float32, 2), (torch.float64, 2)):
        assert auto_kernel(dt, 1000 * 1000, 4, solo=True, order=o) == "pipe"


def test_auto_tblock_fp32_order8_mid_sizes_take_three_steps():
    from cme213x.models.heat2d_dist import auto_tblock

    f32 = torch.float32
    assert auto_tblock(f32, 2000 * 2000, False, "cuda", True) == 3
    assert auto_tblock(f32, 2000 * 2000, True, "cuda", True) == 3
    assert auto_tblock(f32, 2000 * 2000, "fast", "cuda", True) == 4
    assert auto_tblock(f32, 2000 * 2000, False, "cuda", True, order=4) == 4
    assert auto_tblock(f32, 2000 * 2000, False, "cuda", False) == 4  # distributed: halo cadence unchanged
    assert auto_tblock(f32, 3000 * 3000, False, "cuda", True) == 4
    assert auto_tblock(f32, 1000 * 1000, False, "cuda", True) == 4  # the tile pass
    assert auto_tblock(f32, 2000 * 2000, False, "cpu", True) == 1
    f64 = torch.float64
    for o in (2, 4):  # fp64 low orders between the tile range and 2000^2: the pipelined 4-step pass
        assert auto_tblock(f64, 1500 * 1500, False, "cuda", True, order=o) == 4
    assert auto_tblock(f64, 1500 * 1500, False, "cuda", True, order=8) == 2
    assert auto_tblock(f64, 1500 * 1500, True, "cuda", True, order=8) == 3
    assert auto_tblock(f64, 1500 * 1500, False, "cuda", False, order=2) == 2


def test_deep_passes_only_for_solo_fp32_gpu_pipe():
    from cme213x.models.heat2d_dist import DistHeat, auto_tblock

    f32 = torch.float32
    assert auto_tblock(f32, 4096 * 4096, False, "cuda", True, order=2) == 5
    assert auto_tblock(f32, 4096 * 4096, True, "cuda", True, order=2) == 6
    assert auto_tblock(f32, 4096 * 4096, True, "cuda", False, order=2) == 4
    p = SimParams(nx=100, ny=100, order=2, iters=2, flavor="hw5")
    for kw in ({"local_ranks": [0, 1], "world": 2}, {"periodic": (True, False)}):
        with pytest.raises(ValueError, match="tblock"):
            DistHeat(p, None, f32, "cpu", tblock=6, kernel="pipe", **kw)
    with pytest.raises(ValueError, match="tblock"):
        DistHeat(p, None, torch.float64, "cpu", tblock=5, kernel="pipe")
    # the reassociated pass stops at 4 steps: refused at construction (the
    # check runs before any device allocation, so a CUDA device is fine here)
    p8 = SimParams(nx=100, ny=100, order=8, iters=2, flavor="hw5")
    for tb in (5, 6):
        with pytest.raises(ValueError, match="fast"):
            DistHeat(p8, None, f32, "cuda", tblock=tb, kernel="pipe", fma="fast")


@pytest.mark.gpu
@pytest.mark.parametrize("fma", [False, True])
def test_solo_fp32_order2_deep_passes_gpu(gpu, fma):
    """The automatic choice for a solo fp32 order-2 grid is 5 (exact) or 6
    (FMA) steps per pipelined pass; bitwise equal to the CPU oracle's single
    steps over 13 steps (two deep passes and a tail); the native loop refuses
    such a depth."""
    from cme213x.models.heat2d_dist import DistHeat

    n = 700
    p = SimParams(nx=n, ny=n, order=2, iters=13, ic=3.0, bc=(0.0, 10.0, 0.0, 10.0), flavor="hw5")
    sim = DistHeat(p, None, torch.float32, gpu, tblock="auto", kernel="auto", fma=fma)
    assert sim.kernel == "pipe" and sim.tblock == (6 if fma else 5) and sim.solo()
    ref = DistHeat(p, None, torch.float32, "cpu", variant="naive", fma=fma)
    for d in (sim, ref):
        (s,) = d.subs.values()
        g, H = s.grid, s.grid.H
        yy, xx = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
        g.buf[:, H:H + n, H:H + n] = torch.from_numpy(np.sin(0.01 * xx) * np.cos(0.02 * yy) + 3.0).to(
            device=g.device, dtype=torch.float32)
    sim.run(13)
    ref.run(13)
    torch.cuda.synchronize()
    assert np.array_equal(sim.gather_global(), ref.gather_global())
    with pytest.raises(ValueError, match="native loop"):
        sim.run_native(4, transport=2)


@pytest.mark.gpu
@pytest.mark.parametrize("order", [2, 4])
def test_solo_fp64_low_order_mid_size_pipe4_gpu(gpu, order):
    """fp64 order 2 / 4 grids between the tile range and 2000^2 (solo): the
    automatic choice is the pipelined 4-step pass, bitwise equal to the CPU
    oracle (exact arithmetic, 9 steps: two passes and a tail)."""
    from cme213x.models.heat2d_dist import DistHeat

    n = 1250
    p = SimParams(nx=n, ny=n, order=order, iters=9, ic=3.0, bc=(0.0, 10.0, 0.0, 10.0), flavor="hw5")
    sim = DistHeat(p, None, torch.float64, gpu, tblock="auto", kernel="auto")
    assert sim.kernel == "pipe" and sim.tblock == 4 and sim.solo()
    ref = DistHeat(p, None, torch.float64, "cpu", variant="naive")
    for d in (sim, ref):
        (s,) = d.subs.values()
        g, H = s.grid, s.grid.H
        yy, xx = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
        g.buf[:, H:H + n, H:H + n] = torch.from_numpy(np.sin(0.01 * xx) * np.cos(0.02 * yy) + 3.0).to(g.device)
    sim.run(9)
    ref.run(9)
    torch.cuda.synchronize()
    assert np.array_equal(sim.gather_global(), ref.gather_global())


def test_tile_kernel_only_for_single_grids():
    from cme213x.models.heat2d_dist import DistHeat

    p = SimParams(nx=100, ny=100, order=8, iters=2, flavor="hw5")
    with pytest.raises(ValueError, match="tile"):
        DistHeat(p, None, torch.float64, "cpu", tblock=4, kernel="tile", local_ranks=[0, 1], world=2)
    with pytest.raises(ValueError, match="tile"):
        DistHeat(p, None, torch.float64, "cpu", tblock=4, kernel="tile", periodic=(False, True))
