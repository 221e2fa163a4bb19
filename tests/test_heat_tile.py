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
