"""Resident LDS tiles across a whole run (csrc/hip_tune/heat_tile_res.hip,
tuning library only: measured slower than per-pass tile launches,
profiles/heat_tile_res_r5.md; the GPU tests skip without it): one
cooperative launch keeps every 64 x 64 tile in LDS, exchanges only the
NS*B-deep halo ring with its 8 neighbours per pass, and hides the exchange
behind the tile's inner cone.

Parity: bit for bit the CPU oracle's single steps of the same arithmetic
(the reference's 10-ULP check, hw/hw5/2dHeat_solution.cpp, met with zero
ULP), and the per-pass tile launches (production heat_run). Shapes: the hw5
1000^2, grids that are not multiples of the tile (ragged right / bottom
tiles, tiles narrower than the halo), a single tile; orders 2 / 4 / 8,
fp32 / fp64, exact / FMA, 2 and 4 steps per exchange."""
import pytest
import torch

from cme213x.models.heat2d import HeatGrid
from cme213x.ops.stencil import heat_run, heat_step, heat_tile_res, tile_res_timed_out
from cme213x.utils.params import SimParams


def _grid(nx, ny, order, dtype, dev, seed=3):
    p = SimParams(nx=nx, ny=ny, order=order, ic=5.0, bc=(1.0, 10.0, 3.0, 7.0))
    g = HeatGrid(p, dtype, dev)
    B = g.B
    gen = torch.Generator().manual_seed(seed)
    ic = (torch.rand((ny, nx), generator=gen, dtype=torch.float64) * 10.0).to(dtype)
    g.buf[:, B:B + ny, B:B + nx] = ic.to(dev)
    return g


def _cpu_steps(g, n, fma):
    """The CPU oracle: n single steps (exact, or FMA-contracted)."""
    a, b = g.buf[0].cpu().clone(), g.buf[1].cpu().clone()
    for _ in range(n):
        heat_step(a, b, g.interior, g.order, g.xcfl, g.ycfl, "fma" if fma else "naive")
        a, b = b, a
    return a


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("order,ns", [(8, 2), (8, 4), (4, 2), (2, 2)])
@pytest.mark.parametrize("fma", [False, True])
@pytest.mark.parametrize("shape,npass", [((1000, 1000), 3), ((333, 190), 5), ((130, 77), 2), ((64, 64), 4),
                                         ((70, 600), 1)])
def test_resident_equals_cpu_oracle(gpu, tune_lib, dtype, order, ns, fma, shape, npass):
    g = _grid(*shape, order, dtype, gpu, seed=npass)
    want = _cpu_steps(g, ns * npass, fma)
    a, b = g.buf[0].clone(), g.buf[1].clone()
    out = heat_tile_res(a, b, g.interior, order, g.xcfl, g.ycfl, npass, ns=ns, fma=fma)
    assert out.data_ptr() == (b if npass % 2 else a).data_ptr()
    assert torch.equal(out.cpu(), want), f"max |diff| {(out.cpu() - want).abs().max().item()}"


@pytest.mark.gpu
@pytest.mark.parametrize("variant,fma", [("tile4", False), ("tile4_fma", True), ("tile2", False)])
@pytest.mark.parametrize("iters,res_ns", [(13, 2), (13, 4), (100, 2)])
def test_resident_plus_tail_equals_tile_passes(gpu, tune_lib, variant, fma, iters, res_ns):
    """The resident launch over whole exchanges plus a tile-pass tail is
    bitwise the per-pass tile launches of production heat_run."""
    g = _grid(1000, 1000, 8, torch.float64, gpu, seed=iters)
    ref = heat_run(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, iters, variant).clone()
    np_ = iters // res_ns
    a, b = g.buf[0].clone(), g.buf[1].clone()
    mid = heat_tile_res(a, b, g.interior, 8, g.xcfl, g.ycfl, np_, ns=res_ns, fma=fma)
    other = a if mid.data_ptr() == b.data_ptr() else b
    out = heat_run(mid, other, g.interior, 8, g.xcfl, g.ycfl, iters - np_ * res_ns, variant)
    torch.cuda.synchronize()
    assert not tile_res_timed_out(reset=True)
    assert torch.equal(out, ref)


@pytest.mark.gpu
def test_resident_trace_and_schedule(gpu, tune_lib):
    """Every (pass, tile) is stamped in order (start <= inner done <= halo in
    <= outer done <= ring published, the last during the next pass), and a
    tile's halo of pass p + 1 is read only after each of its 8 neighbours
    published its pass-p ring (wall clock)."""
    g = _grid(1000, 1000, 8, torch.float64, gpu, seed=11)
    npass = 6
    want = _cpu_steps(g, 2 * npass, False)
    out, tr, ntiles = heat_tile_res(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, npass,
                                    trace=True)
    assert torch.equal(out.cpu(), want)
    assert ntiles == 256 and tr.shape == (256 * npass, 5) and bool((tr > 0).all())
    t = tr.view(npass, 16, 16, 5)
    for k in range(4):
        assert bool((t[..., k + 1] >= t[..., k]).all()), k
    for p in range(npass - 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                ys, yd = slice(max(0, dy), 16 + min(0, dy)), slice(max(0, -dy), 16 + min(0, -dy))
                xs, xd = slice(max(0, dx), 16 + min(0, dx)), slice(max(0, -dx), 16 + min(0, -dx))
                # tile (y, x) reads neighbour (y + dy, x + dx)
                assert bool((t[p + 1, yd, xd, 2] >= t[p, ys, xs, 4]).all()), (p, dy, dx)


@pytest.mark.gpu
def test_resident_too_large_falls_back(gpu, tune_lib):
    """More tiles than the device holds at once: the call refuses."""
    g = _grid(2200, 2000, 8, torch.float64, gpu, seed=2)  # 35 x 32 tiles > one per CU
    with pytest.raises(ValueError, match="resident"):
        heat_tile_res(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, 2)


@pytest.mark.gpu
def test_resident_timeout_raises_and_drains(gpu, tune_lib):
    """A neighbour wait that gives up (diagnostics: tile 0 never publishes)
    aborts every workgroup and raises; the next call runs."""
    from cme213x.utils import tuning

    g = _grid(1000, 1000, 8, torch.float64, gpu, seed=4)
    with tuning.override(flow_spins=1 << 12, flow_mode=2048):
        with pytest.raises(RuntimeError, match="gave up"):
            heat_tile_res(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, 8)
    assert not tile_res_timed_out()
    want = _cpu_steps(g, 4, False)
    out = heat_tile_res(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, 2)
    assert torch.equal(out.cpu(), want)


def test_resident_refuses_cpu_and_bad_depth():
    g = _grid(100, 100, 8, torch.float64, "cpu")
    with pytest.raises(ValueError, match="GPU"):
        heat_tile_res(g.buf[0], g.buf[1], g.interior, 8, g.xcfl, g.ycfl, 2)
    g4 = _grid(100, 100, 4, torch.float64, "cpu")
    with pytest.raises(ValueError, match="GPU"):
        heat_tile_res(g4.buf[0], g4.buf[1], g4.interior, 4, g4.xcfl, g4.ycfl, 2, ns=4)
