"""Reassociated ("fast") stencil arithmetic on the GPU (csrc/hip/heat_fast.hip):
folded CFL weights and symmetric pair sums, 17 flop-instructions per point at
order 8. Every path must equal the CPU fast oracle (cme_cpu_heat_step_fast_*)
bit for bit:
* the plain single step, orders 2/4/8, fp32/fp64;
* the wide-lane pipelined 2-4 step passes over several output regions with a
  grown intermediate region (the distributed border-strip pass);
* the whole-interior multi-pass driver with its remainders;
* the distributed solver's Python and native loops over loopback subdomains.
The fast form itself is checked within the reference's 10-ULP criterion of
the exact stencil in test_heat_pipe.py (test_fast_oracle_close_to_exact)."""
import ctypes

import numpy as np
import pytest
import torch

from cme213x.models.heat2d import HeatGrid
from cme213x.ops.stencil import FAST_VARIANTS, arith_code, heat_run, heat_step, heat_stepn
from cme213x.utils.params import SimParams


def _rand_grid(p, dtype, device="cpu", seed=0):
    g = HeatGrid(p, dtype, device)
    gen = torch.Generator().manual_seed(seed)
    r = torch.rand(g.buf[0].shape, generator=gen, dtype=dtype) * 10.0
    g.buf[0].copy_(r.to(device))
    g.buf[1].copy_(r.to(device))
    return g


def _cpu_fast_steps(buf, region, order, xcfl, ycfl, n):
    a, b = buf.clone(), buf.clone()
    for _ in range(n):
        heat_step(a, b, region, order, xcfl, ycfl, "fast")
        a, b = b, a
    return a


def test_arith_codes():
    assert [arith_code(x) for x in (False, True, 0, 1, "exact", "fma", "fast", 2)] == [0, 1, 0, 1, 0, 1, 2, 2]
    with pytest.raises(ValueError):
        arith_code("fastest")
    assert FAST_VARIANTS["pipe4_fast"] == 4 and FAST_VARIANTS["fast"] == 1


def test_fast_refused_outside_fp32_order8_pipe():
    from cme213x.models.heat2d_dist import DistHeat

    p = SimParams(nx=64, ny=64, order=8, flavor="hw5")
    with pytest.raises(ValueError, match="fast"):
        DistHeat(p, None, torch.float64, "cpu", tblock=4, fma="fast")
    with pytest.raises(ValueError, match="fast"):
        DistHeat(SimParams(nx=64, ny=64, order=4, flavor="hw5"), None, torch.float32, "cpu", tblock=2, fma="fast")
    g = HeatGrid(SimParams(nx=40, ny=30, order=4), torch.float32)
    with pytest.raises(ValueError, match="fp32, order 8"):
        heat_stepn(g.buf[0], g.buf[1], g.interior, g.interior, 4, g.xcfl, g.ycfl, 3, fma="fast")


@pytest.mark.parametrize("world,method,tblock", [(4, 1, 1), (4, 2, 2), (2, 1, 4), (8, 1, 4)])
def test_fast_loopback_subdomains_cpu(world, method, tblock):
    """CPU: the distributed solver with reassociated arithmetic over loopback
    subdomains equals the single-grid fast run bit for bit."""
    from cme213x.models.heat2d_dist import DistHeat

    # (8 stripes of 40 rows: the bench's 8-way split, four steps per pass, 16-row halos -- in one process)
    ny = 320 if world == 8 else 83
    p = SimParams(nx=97, ny=ny, order=8, iters=6, ic=5.0, bc=(1.0, 10.0, 3.0, 7.0), grid_method=method,
                  flavor="hw5")
    one = DistHeat(p, None, torch.float32, "cpu", fma="fast")
    many = DistHeat(p, None, torch.float32, "cpu", fma="fast", tblock=tblock, local_ranks=list(range(world)),
                    world=world)
    for d in (one, many):
        _ic(d, torch.float32)
        d.run(p.iters)
    assert np.array_equal(one.gather_global(), many.gather_global())


def _ic(sim, dtype):
    for s in sim.subs.values():
        g, b = s.grid, s.blk
        H = g.H
        yy, xx = np.meshgrid(np.arange(b.ny) + b.y0, np.arange(b.nx) + b.x0, indexing="ij")
        ic = torch.from_numpy(np.sin(0.3 * xx) * np.cos(0.2 * yy) + 5.0 + 0.01 * ((xx * 7 + yy * 3) % 5)).to(dtype)
        g.buf[:, H:H + b.ny, H:H + b.nx] = ic.to(g.device)
    sim.exchange(sim._cur()).wait()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("order", [2, 4, 8])
def test_gpu_fast_single_step_bitwise(gpu, dtype, order):
    p = SimParams(nx=301, ny=173, order=order)
    c = _rand_grid(p, dtype)
    g = _rand_grid(p, dtype, gpu)
    region = (c.B + 3, c.B + 290, c.B + 1, c.B + 170)
    want = _cpu_fast_steps(c.buf[0], region, order, c.xcfl, c.ycfl, 1)
    out = g.buf[0].clone()
    heat_step(g.buf[0], out, region, order, g.xcfl, g.ycfl, "fast")
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), want)


@pytest.mark.gpu
@pytest.mark.parametrize("ns", [2, 3, 4])
def test_gpu_fast_pipe_regions_bitwise(gpu, ns):
    """Three output regions (interior + two border strips) with the
    intermediate steps over a grown region, one launch: equal to ns single
    fast steps over (ext, ..., ext, regions)."""
    p = SimParams(nx=1500, ny=700, order=8)
    c = _rand_grid(p, torch.float32, seed=4)
    g = _rand_grid(p, torch.float32, gpu, seed=4)
    B = c.B
    xb, xe, yb, ye = c.interior
    regions = [(xb, xe, yb + 20, ye - 20), (xb, xe, yb, yb + 20), (xb, xe, ye - 20, ye)]
    ext = (xb, xe, yb, ye)
    src = c.buf[0].clone()
    for _ in range(ns - 1):
        tmp = src.clone()
        heat_step(src, tmp, ext, 8, c.xcfl, c.ycfl, "fast")
        src = tmp
    want = c.buf[0].clone()
    for reg in regions:
        heat_step(src, want, reg, 8, c.xcfl, c.ycfl, "fast")
    out = g.buf[0].clone()
    heat_stepn(g.buf[0], out, regions, ext, 8, g.xcfl, g.ycfl, ns, fma="fast", kernel="pipe")
    torch.cuda.synchronize()
    assert B > 0 and torch.equal(out.cpu(), want)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["pipe4_fast", "pipe3_fast", "pipe2_fast", "fast"])
@pytest.mark.parametrize("iters", [1, 2, 3, 7, 9])
def test_gpu_fast_heat_run_bitwise(gpu, variant, iters):
    p = SimParams(nx=517, ny=263, order=8)
    c = _rand_grid(p, torch.float32, seed=2)
    g = _rand_grid(p, torch.float32, gpu, seed=2)
    want = _cpu_fast_steps(c.buf[0], c.interior, 8, c.xcfl, c.ycfl, iters)
    out = heat_run(g.buf[0], g.buf[1], g.interior, 8, g.xcfl, g.ycfl, iters, variant)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), want)


@pytest.mark.gpu
@pytest.mark.parametrize("method,world", [(1, 4), (2, 4), (1, 3), (1, 8)])
@pytest.mark.parametrize("sync", [False, True])
@pytest.mark.parametrize("tblock", [3, 4])
@pytest.mark.parametrize("native", [True, False])
def test_gpu_fast_subdomains_bitwise(gpu, method, world, sync, tblock, native):
    """The distributed schedule with reassociated arithmetic (deep interior and
    border strips in one pipelined launch, intermediate steps into the
    nB-deep halos, single-step / shorter remainders) through the native loop
    (loopback transport) and the Python loop: equal to the single-grid CPU
    fast oracle bit for bit."""
    from cme213x.models.heat2d_dist import DistHeat

    p = SimParams(nx=333, ny=270, order=8, iters=9, sync=sync, grid_method=method, ic=5.0,
                  bc=(1.0, 10.0, 3.0, 7.0), flavor="hw5")
    ref = DistHeat(p, None, torch.float32, "cpu", fma="fast")
    sim = DistHeat(p, None, torch.float32, gpu, local_ranks=list(range(world)), world=world, tblock=tblock,
                   fma="fast", kernel="pipe")
    assert sim._flags() & 8
    for d in (ref, sim):
        _ic(d, torch.float32)
    ref.run(p.iters)
    if native:
        sim.run_native(5)
        sim.run_native(4)
    else:
        sim.run(p.iters)
    torch.cuda.synchronize()
    assert np.array_equal(sim.gather_global(), ref.gather_global())


@pytest.mark.gpu
def test_gpu_fast_solo_run_uses_pipe_fast(gpu):
    """A single-grid fp32 run (world 1): DistHeat.run hands the loop to the
    native multi-pass driver with the fast 4-step pass."""
    from cme213x.models.heat2d_dist import DistHeat

    p = SimParams(nx=700, ny=500, order=8, iters=11, ic=5.0, bc=(1.0, 10.0, 3.0, 7.0), flavor="hw5")
    sim = DistHeat(p, None, torch.float32, gpu, tblock="auto", kernel="pipe", fma="fast")
    assert sim.solo() and sim.run_variant() == "pipe4_fast"
    ref = DistHeat(p, None, torch.float32, "cpu", fma="fast")
    for d in (sim, ref):
        _ic(d, torch.float32)
    sim.run(11)
    ref.run(11)
    torch.cuda.synchronize()
    assert np.array_equal(sim.gather_global(), ref.gather_global())


@pytest.mark.gpu
def test_gpu_fast_pipe_gated_entry(gpu):
    """The gated form of the fast pass (the fused schedule's launch): with the
    flag already reached it equals the ungated pass, and the timeout word
    stays clear."""
    from cme213x import _ext

    p = SimParams(nx=900, ny=400, order=8)
    g = _rand_grid(p, torch.float32, gpu, seed=6)
    xb, xe, yb, ye = g.interior
    regs = [(xb, xe, yb + 16, ye - 16), (xb, xe, yb, yb + 16), (xb, xe, ye - 16, ye)]
    flat = (ctypes.c_int * 12)(*[v for r in regs for v in r])
    e = (ctypes.c_int * 4)(xb, xe, yb, ye)
    ref = g.buf[0].clone()
    heat_stepn(g.buf[0], ref, regs, (xb, xe, yb, ye), 8, g.xcfl, g.ycfl, 4, fma="fast", kernel="pipe")
    flag = torch.full((1,), 7, dtype=torch.int32, device=gpu)
    tw = torch.zeros(1, dtype=torch.int32, device=gpu)
    out = g.buf[0].clone()
    _ext.call_hip("cme_heat_pipe_fast_f32", g.buf[0].data_ptr(), out.data_ptr(), g.pitch, g.gy,
                  ctypes.addressof(flat), 3, ctypes.addressof(e), 8, 4, g.xcfl, g.ycfl, 0, 1, flag.data_ptr(), 7,
                  tw.data_ptr(), _ext.stream_ptr(g.buf[0].device))
    torch.cuda.synchronize()
    assert torch.equal(out, ref) and int(tw.item()) == 0


# measured max ULP distance from the exact stencil (interior cells). The
# reassociated arithmetic used to random-walk away from the exact trajectory
# (15 ULP at 4000^2 x 10, 39 at 2048^2 x 200 random): its rounded fp32 weights
# summed to 1 + ~1e-8. With weights that sum to exactly one
# (heat_fast_make_consistent) it stays within the reference's 10-ULP criterion:
# 7 / 9 / 7 / 7 ULP at the four shapes below, like the FMA form's <= 8
# (profiles/heat_arith_ulp_r5.md).
_FAST_DRIFT_MAX = {(4000, 10, "uniform"): 7, (4000, 10, "random"): 9, (2048, 40, "random"): 7,
                   (2048, 200, "random"): 7}


@pytest.mark.parametrize("arith", ["fma", "fast"])
@pytest.mark.parametrize("n,steps,flavor,init", [(4000, 10, "hw2", "uniform"), (4000, 10, "hw2", "random"),
                                                 (2048, 40, "hw5", "random"), (2048, 200, "hw5", "random")])
def test_arith_ulp_drift_from_exact_at_scale(n, steps, flavor, init, arith):
    """VERDICT r4 #7a: distance from the exact stencil after the whole run,
    under the reference's 10-ULP criterion (hw/hw2/solution/
    2dHeat_solution.cu:690-710, interior cells), at the hw2 golden shape
    (4000^2, order 8, 10 steps: the reference's uniform IC and a random
    interior) and over 40- and 200-step 2048^2 runs on the bench's hw5 CFL
    numbers -- rounding differences compound with the step count. The
    FMA-contracted arithmetic (what nvcc emits for the reference's GPU kernel)
    and the reassociated one with exactly-consistent weights (the bench
    default) both meet it; the measured fast drift is pinned here. The GPU
    passes equal these CPU oracles bit for bit (test_gpu_fast_heat_run_bitwise,
    the pipe/stream FMA tests), so the numbers carry over to them."""
    from cme213x.utils.ulp import ulp_distance

    p = SimParams(nx=n, ny=n, order=8, iters=steps, ic=5.0, bc=(0.0, 10.0, 0.0, 10.0), flavor=flavor)
    g = _rand_grid(p, torch.float32, seed=11) if init == "random" else HeatGrid(p, torch.float32)
    if init == "random":  # the BCs stay the reference's
        g0 = HeatGrid(p, torch.float32)
        xb, xe, yb, ye = g.interior
        for k in (0, 1):
            keep = g.buf[k, yb:ye, xb:xe].clone()
            g.buf[k].copy_(g0.buf[0])
            g.buf[k, yb:ye, xb:xe] = keep
    if arith == "fast":
        out = _cpu_fast_steps(g.buf[0], g.interior, 8, g.xcfl, g.ycfl, steps)
    else:
        a, b = g.buf[0].clone(), g.buf[0].clone()
        out = heat_run(a, b, g.interior, 8, g.xcfl, g.ycfl, steps, "fma").clone()
    a, b = g.buf[0].clone(), g.buf[0].clone()
    exact = heat_run(a, b, g.interior, 8, g.xcfl, g.ycfl, steps, "naive")
    xb, xe, yb, ye = g.interior
    d = int(ulp_distance(out[yb:ye, xb:xe].numpy(), exact[yb:ye, xb:xe].numpy()).max())
    bound = 10 if arith == "fma" else min(10, _FAST_DRIFT_MAX[(n, steps, init)])
    assert d <= bound, f"{arith}: max {d} ULP"
