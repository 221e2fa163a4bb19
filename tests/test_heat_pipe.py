"""Wave-pipelined NS-step heat pass (csrc/hip/heat_pipe.hip): bitwise equal to
NS single steps (exact and FMA oracles) and to the streamN pass, over full
grids, sub-regions, several output regions with a grown intermediate region
(the distributed border-strip pass), every tuning arm (rows per phase,
prefetch depth, chunking) and 5-6 steps per pass.

Parity: the reference's hw2/hw5 update loops (hw/hw2/solution/2dHeat_solution.cu
:413-530, hw/hw5/2dHeat_solution.cpp:501-628) applied NS times."""
import numpy as np
import pytest
import torch

from cme213x.models.heat2d import HeatGrid
from cme213x.utils.params import SimParams
from cme213x.utils.ulp import ulp_distance


def _rand_grid(p, dtype, device="cpu", seed=0):
    g = HeatGrid(p, dtype, device)
    gen = torch.Generator().manual_seed(seed)
    r = torch.rand(g.buf[0].shape, generator=gen, dtype=dtype)
    g.buf[0].copy_(r)
    g.buf[1].copy_(r)
    return g


def test_pipe_variants_are_multistep_any_dtype():
    from cme213x.ops.stencil import FMA_VARIANTS, FP32_ONLY, MULTISTEP, VARIANTS
    for v in ("pipe3", "pipe3_fma", "pipe4", "pipe4_fma"):
        assert v in VARIANTS and v in MULTISTEP and v not in FP32_ONLY
    assert "pipe4_fma" in FMA_VARIANTS and "pipe4" not in FMA_VARIANTS


def test_pipe56_variants_fp32_only():
    from cme213x.ops.stencil import FMA_VARIANTS, FP32_ONLY, MULTISTEP, heat_run
    for v in ("pipe5", "pipe5_fma", "pipe6", "pipe6_fma"):
        assert v in MULTISTEP and v in FP32_ONLY
    assert {"pipe5_fma", "pipe6_fma"} <= FMA_VARIANTS
    p = SimParams(nx=20, ny=20, order=2)
    g = HeatGrid(p, torch.float64)
    with pytest.raises(ValueError):
        heat_run(g.buf[0], g.buf[1], g.interior, 2, g.xcfl, g.ycfl, 6, "pipe6")


@pytest.mark.gpu
@pytest.mark.parametrize("order", [2, 4, 8])
@pytest.mark.parametrize("ns", [5, 6])
@pytest.mark.parametrize("fma", [False, True])
@pytest.mark.parametrize("iters", [5, 6, 13])
def test_gpu_pipe56_temporal_blocking_bitwise(gpu, order, ns, fma, iters):
    """Five and six steps per pass (fp32; the HBM-bound low orders), remainders
    through two-step and single passes: bitwise equal to single steps."""
    p = SimParams(nx=517, ny=263, order=order)
    c = _rand_grid(p, torch.float32)
    g = _rand_grid(p, torch.float32, gpu)
    c.run(iters, "fma" if fma else "naive")
    g.run(iters, f"pipe{ns}" + ("_fma" if fma else ""))
    torch.cuda.synchronize()
    d = ulp_distance(c.state(), g.state())
    assert int(d.max()) == 0, f"max ulp {int(d.max())}"


def test_pipe_kernel_name_checked():
    from cme213x.ops.stencil import heat_stepn
    p = SimParams(nx=20, ny=20, order=8)
    g = HeatGrid(p, torch.float32)
    with pytest.raises(ValueError):
        heat_stepn(g.buf[0], g.buf[1], g.interior, g.interior, 8, g.xcfl, g.ycfl, 3, kernel="bogus")


@pytest.mark.gpu
@pytest.mark.parametrize("order", [2, 4, 8])
@pytest.mark.parametrize("ns", [3, 4])
@pytest.mark.parametrize("fma", [False, True])
@pytest.mark.parametrize("iters", [1, 4, 7, 9])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_gpu_pipe_temporal_blocking_bitwise(gpu, order, ns, fma, iters, dtype):
    p = SimParams(nx=517, ny=263, order=order)
    c = _rand_grid(p, dtype)
    g = _rand_grid(p, dtype, gpu)
    c.run(iters, "fma" if fma else "naive")
    g.run(iters, f"pipe{ns}" + ("_fma" if fma else ""))
    torch.cuda.synchronize()
    d = ulp_distance(c.state(), g.state())
    assert int(d.max()) == 0, f"max ulp {int(d.max())}"


@pytest.mark.gpu
@pytest.mark.parametrize("region", [(4, 300, 4, 100), (9, 250, 17, 77), (130, 131, 5, 200), (8, 292, 8, 242)])
@pytest.mark.parametrize("chunk", [0, 8, 14, 400])
@pytest.mark.parametrize("ns", [3, 4])
def test_gpu_pipe_subregion(gpu, region, chunk, ns):
    from cme213x.ops.stencil import heat_run
    p = SimParams(nx=300, ny=250, order=8)
    c = _rand_grid(p, torch.float32)
    g = _rand_grid(p, torch.float32, gpu)
    ca, cb = c.buf[0].clone(), c.buf[0].clone()
    ga, gb = g.buf[0].clone(), g.buf[0].clone()
    oc = heat_run(ca, cb, region, 8, c.xcfl, c.ycfl, 2 * ns, "fma")
    og = heat_run(ga, gb, region, 8, g.xcfl, g.ycfl, 2 * ns, f"pipe{ns}_fma", chunk)
    torch.cuda.synchronize()
    assert torch.equal(oc, og.cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("ns", [3, 4])
@pytest.mark.parametrize("fma", [False, True])
def test_gpu_pipe_multi_region_ext(gpu, ns, fma):
    """Several output regions in one launch with an intermediate region grown
    past them (the distributed border-strip pass): equal to the CPU single
    steps and to the streamN pass."""
    from cme213x.ops.stencil import heat_stepn
    p = SimParams(nx=300, ny=250, order=8)
    c = _rand_grid(p, torch.float32)
    g = _rand_grid(p, torch.float32, gpu)
    regs = [(4, 304, 4, 40), (4, 304, 220, 254), (4, 40, 40, 220), (270, 304, 40, 220)]
    ext = (4, 304, 4, 254)
    oc, og, os_ = c.buf[0].clone(), g.buf[0].clone(), g.buf[0].clone()
    heat_stepn(c.buf[0], oc, regs, ext, 8, c.xcfl, c.ycfl, ns, fma=fma)
    heat_stepn(g.buf[0], og, regs, ext, 8, g.xcfl, g.ycfl, ns, fma=fma, kernel="pipe")
    heat_stepn(g.buf[0], os_, regs, ext, 8, g.xcfl, g.ycfl, ns, fma=fma, kernel="streamn")
    torch.cuda.synchronize()
    assert torch.equal(oc, og.cpu())
    assert torch.equal(og, os_)


@pytest.mark.gpu
def test_gpu_pipe_tuning_arms_bitwise(gpu, tune_lib):
    """Every compiled tuning arm (ns 3-6, rows per phase, prefetch depth,
    tasks per CU / explicit chunk) equals ns single FMA steps on an odd-sized
    region of random data."""
    from cme213x import _ext
    from cme213x.ops.stencil import heat_run
    p = SimParams(nx=1500, ny=700, order=8)
    c = _rand_grid(p, torch.float32)
    g = _rand_grid(p, torch.float32, gpu)
    region = (9, 1400, 6, 690)
    xb, xe, yb, ye = region
    oracle = {}
    for ns in (3, 4, 5, 6):
        ca, cb = c.buf[0].clone(), c.buf[0].clone()
        oracle[ns] = heat_run(ca, cb, region, 8, c.xcfl, c.ycfl, ns, "fma").clone()
    s = _ext.stream_ptr(g.buf[0].device)
    arms = [(ns, rb, pd, pc, ch) for ns in (3, 4) for rb in (2, 4, 8) for pd in (1, 2) for pc, ch in ((2, 0), (0, 24))]
    arms += [(ns, 4, pd, 3, 0) for ns in (5, 6) for pd in (1, 2)]
    for ns, rb, pd, pc, ch in arms:
        out = g.buf[0].clone()
        _ext.call_hip("cme_heat_pipe_tune", g.buf[0].data_ptr(), out.data_ptr(), g.pitch, g.gy, xb, xe, yb, ye,
                      g.xcfl, g.ycfl, ch, rb, ns, pd, pc, s)
        torch.cuda.synchronize()
        assert torch.equal(out.cpu(), oracle[ns]), (ns, rb, pd, pc, ch)


@pytest.mark.gpu
@pytest.mark.parametrize("region", [(9, 1400, 6, 690), (130, 131, 5, 200), (4, 484, 4, 100), (600, 1100, 33, 47)])
def test_gpu_pipe_multiwave_roles_bitwise(gpu, tune_lib, region):
    """Two and four waves per timestep role (seam x-neighbours through the LDS
    edge buffer): equal to ns single FMA steps on regions narrower than, equal
    to and wider than one strip, with explicit short chunks and the default
    chunk rule."""
    from cme213x import _ext
    from cme213x.ops.stencil import heat_run
    p = SimParams(nx=1500, ny=700, order=8)
    c = _rand_grid(p, torch.float32, seed=5)
    g = _rand_grid(p, torch.float32, gpu, seed=5)
    xb, xe, yb, ye = region
    oracle = {}
    for ns in (3, 4, 5, 6):
        ca, cb = c.buf[0].clone(), c.buf[0].clone()
        oracle[ns] = heat_run(ca, cb, region, 8, c.xcfl, c.ycfl, ns, "fma").clone()
    s = _ext.stream_ptr(g.buf[0].device)
    arms = [(ns, 21, pc, ch) for ns in (3, 4, 5, 6) for pc, ch in ((2, 0), (0, 12), (0, 0))]
    arms += [(ns, 41, pc, ch) for ns in (3, 4) for pc, ch in ((1, 0), (0, 8), (0, 0))]
    for ns, pd, pc, ch in arms:
        out = g.buf[0].clone()
        _ext.call_hip("cme_heat_pipe_tune", g.buf[0].data_ptr(), out.data_ptr(), g.pitch, g.gy, xb, xe, yb, ye,
                      g.xcfl, g.ycfl, ch, 4, ns, pd, pc, s)
        torch.cuda.synchronize()
        assert torch.equal(out.cpu(), oracle[ns]), (ns, pd, pc, ch)


@pytest.mark.gpu
@pytest.mark.parametrize("region", [(9, 1400, 6, 690), (130, 131, 5, 200), (4, 484, 4, 100), (600, 1100, 33, 47),
                                    (4, 1504, 4, 704), (12, 20, 4, 704)])
def test_gpu_pipe_wide_lanes_bitwise(gpu, tune_lib, region):
    """Wide lanes (8 columns per lane, strips on 8-column boundaries, so edge
    lanes straddle region starts like x = 4, 9, 12): equal to ns single FMA
    steps for ns 3-5, 2 and 4 rows per phase, chain-major (81) and term-major
    (85, production) FMA order, x-neighbours from the LDS ring (86), register
    caps (83/84), short explicit chunks
    and the default chunk rule, on regions narrower than, equal to and wider
    than one strip, up to the whole interior."""
    from cme213x import _ext
    from cme213x.ops.stencil import heat_run
    p = SimParams(nx=1500, ny=700, order=8)
    c = _rand_grid(p, torch.float32, seed=6)
    g = _rand_grid(p, torch.float32, gpu, seed=6)
    xb, xe, yb, ye = region
    oracle = {}
    for ns in (3, 4, 5):
        ca, cb = c.buf[0].clone(), c.buf[0].clone()
        oracle[ns] = heat_run(ca, cb, region, 8, c.xcfl, c.ycfl, ns, "fma").clone()
    s = _ext.stream_ptr(g.buf[0].device)
    arms = [(ns, rb, pd, pc, ch) for ns in (3, 4) for rb in (2, 4) for pd in (81, 85)
            for pc, ch in ((2, 0), (0, 10), (0, 0))]
    arms += [(ns, rb, 86, pc, ch) for ns in (3, 4) for rb in (2, 4) for pc, ch in ((2, 0), (0, 10), (0, 0))]
    arms += [(5, 4, 81, 0, 0), (5, 4, 85, 0, 12), (4, 2, 83, 0, 0), (4, 2, 84, 0, 0)]
    for ns, rb, pd, pc, ch in arms:
        out = g.buf[0].clone()
        _ext.call_hip("cme_heat_pipe_tune", g.buf[0].data_ptr(), out.data_ptr(), g.pitch, g.gy, xb, xe, yb, ye,
                      g.xcfl, g.ycfl, ch, rb, ns, pd, pc, s)
        torch.cuda.synchronize()
        assert torch.equal(out.cpu(), oracle[ns]), (ns, rb, pd, pc, ch)


@pytest.mark.gpu
def test_gpu_pipe_gated_regions(gpu):
    """The fused-schedule entry (cme_heat_pipe_gated_f32): deep interior plus
    gated border strips in one launch, gate already open, equals the plain
    pipelined pass over the same regions."""
    import ctypes

    from cme213x import _ext
    from cme213x.ops.stencil import heat_stepn
    p = SimParams(nx=600, ny=500, order=8)
    g = _rand_grid(p, torch.float32, gpu, seed=4)
    regs = [(4, 604, 40, 464), (4, 604, 4, 40), (4, 604, 464, 504)]  # interior, then two border strips
    ext = (4, 604, 4, 504)
    ref = g.buf[0].clone()
    heat_stepn(g.buf[0], ref, regs, ext, 8, g.xcfl, g.ycfl, 4, fma=True, kernel="pipe")
    flag = torch.full((1,), 7, dtype=torch.int32, device=gpu)
    tw = torch.zeros(1, dtype=torch.int32, device=gpu)  # the timeout word must be device-visible
    flat = (ctypes.c_int * 12)(*[v for r in regs for v in r])
    e = (ctypes.c_int * 4)(*ext)
    out = g.buf[0].clone()
    _ext.call_hip("cme_heat_pipe_gated_f32", g.buf[0].data_ptr(), out.data_ptr(), g.pitch, g.gy,
                  ctypes.addressof(flat), 3, ctypes.addressof(e), 8, 4, g.xcfl, g.ycfl, 1, 1, flag.data_ptr(), 7,
                  tw.data_ptr(), _ext.stream_ptr(g.buf[0].device))
    torch.cuda.synchronize()
    assert torch.equal(out, ref) and int(tw.item()) == 0


def _fast_steps(c, region, ns):
    """ns steps of the reassociated CPU oracle (cme_cpu_heat_step_fast_f32)."""
    from cme213x import _ext
    a, b = c.buf[0].clone(), c.buf[0].clone()
    for _ in range(ns):
        _ext.call_cpu("cme_cpu_heat_step_fast_f32", a.data_ptr(), b.data_ptr(), c.pitch, *region, 8, c.xcfl, c.ycfl)
        a, b = b, a
    return a


def test_fast_oracle_close_to_exact():
    """The reassociated ("fast") stencil is the same FTCS update: within a few
    ULP of the exact oracle over 8 steps (the reference's criterion is 10)."""
    from cme213x.ops.stencil import heat_run
    from cme213x.utils.ulp import ulp_distance
    p = SimParams(nx=300, ny=250, order=8)
    c = _rand_grid(p, torch.float32, seed=7)
    region = c.interior
    fast = _fast_steps(c, region, 8)
    ca, cb = c.buf[0].clone(), c.buf[0].clone()
    exact = heat_run(ca, cb, region, 8, c.xcfl, c.ycfl, 8, "naive")
    assert not torch.equal(fast, exact)
    assert int(ulp_distance(fast.numpy(), exact.numpy()).max()) <= 10


@pytest.mark.gpu
def test_gpu_pipe_fast_arms_bitwise(gpu, tune_lib):
    """The reassociated-arithmetic tuning arms (pd 12: default registers, 13:
    capped at 4 waves/SIMD, 91: wide lanes, 92: capped at 3 waves/SIMD, 95 / 96:
    terms interleaved across the lane's points) equal ns steps of the CPU fast
    oracle bit for bit."""
    from cme213x import _ext
    p = SimParams(nx=1500, ny=700, order=8)
    c = _rand_grid(p, torch.float32, seed=9)
    g = _rand_grid(p, torch.float32, gpu, seed=9)
    region = (9, 1400, 6, 690)
    s = _ext.stream_ptr(g.buf[0].device)
    for ns in (3, 4):
        oracle = _fast_steps(c, region, ns)
        for pd, rb in ((12, 4), (13, 4), (91, 2), (92, 2), (95, 2), (96, 2), (97, 1)):  # 9x: wide lanes
            if pd == 97 and ns != 4:  # one row per phase: four steps only
                continue
            out = g.buf[0].clone()
            _ext.call_hip("cme_heat_pipe_tune", g.buf[0].data_ptr(), out.data_ptr(), g.pitch, g.gy, *region,
                          g.xcfl, g.ycfl, 0, rb, ns, pd, 0, s)
            torch.cuda.synchronize()
            assert torch.equal(out.cpu(), oracle), (ns, pd)


@pytest.mark.gpu
def test_gpu_pipe_long_run_matches_streamn(gpu):
    """A 16384-wide, 2048-row strip (one rank's share of an 8-GPU run) over 24
    steps: pipelined and streamN passes agree bit for bit."""
    from cme213x.ops.stencil import heat_run
    p = SimParams(nx=4096, ny=1024, order=8)
    g = _rand_grid(p, torch.float32, gpu, seed=3)
    a1, b1 = g.buf[0].clone(), g.buf[0].clone()
    a2, b2 = g.buf[0].clone(), g.buf[0].clone()
    o1 = heat_run(a1, b1, g.interior, 8, g.xcfl, g.ycfl, 24, "pipe4_fma")
    o2 = heat_run(a2, b2, g.interior, 8, g.xcfl, g.ycfl, 24, "stream4_fma")
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    assert np.isfinite(o1.cpu().numpy()).all()


def test_dist_heat_kernel_option_cpu():
    """DistHeat validates the pass kernel and, on CPU tensors, runs the
    single-step oracle composition whatever the kernel."""
    from cme213x.models.heat2d_dist import DistHeat
    p = SimParams(nx=80, ny=90, order=8, iters=4, flavor="hw5")
    with pytest.raises(ValueError):
        DistHeat(p, None, torch.float32, "cpu", tblock=4, kernel="bogus")
    a = DistHeat(p, None, torch.float32, "cpu", local_ranks=[0, 1], world=2, tblock=4, kernel="pipe")
    b = DistHeat(p, None, torch.float32, "cpu", local_ranks=[0, 1], world=2, tblock=1)
    assert a._flags() == 2 and b._flags() == 0
    a.run(5)
    b.run(5)
    assert np.array_equal(a.gather_global(), b.gather_global())


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["pipe4_fma", "pipe4_fast", "pipe3_fma"])
@pytest.mark.parametrize("taper", [-1, 7])
def test_gpu_pipe_taper_bitwise(gpu, variant, taper):
    """Tapered chunking (tuning knob pipe_taper: the last chunks of every
    strip at half height, for passes of several rounds of workgroups) only
    moves task boundaries: bitwise equal to the untapered pass."""
    from cme213x.ops.stencil import heat_run
    from cme213x.utils import tuning

    p = SimParams(nx=4000, ny=3000, order=8)
    g = _rand_grid(p, torch.float32, gpu, seed=11)
    outs = []
    for t in (0, taper):
        with tuning.override(pipe_per_cu=16, pipe_taper=t):  # 16 tasks per CU: several rounds
            a, b = g.buf[0].clone(), g.buf[1].clone()
            outs.append(heat_run(a, b, g.interior, 8, g.xcfl, g.ycfl, 9, variant).clone())
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
