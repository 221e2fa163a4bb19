"""Persistent dataflow schedule of the pipelined heat pass (csrc/hip_tune/
heat_flow.hip, tuning library only: measured no faster than per-pass
launches, profiles/heat_flow_r5.md): all four-step passes of a run in ONE
launch, tasks pulled from a ticket, each waiting for its 3 x 3 neighbourhood
of the previous pass. The GPU tests skip without libcme213_tune.so.

Parity: the result must equal, bit for bit, the same passes launched one by
one (production heat_run) and the CPU oracle's single steps of the same
arithmetic (the reference's 10-ULP check, hw/hw2/solution/
2dHeat_solution.cu:690-710, is met with zero ULP). Uneven load: many tiny
tasks (knob flow_per_cu) so dependency waits actually happen, odd region
edges so edge tasks differ in cost."""
import pytest
import torch

from cme213x.models.heat2d import HeatGrid
from cme213x.ops.stencil import flow_timed_out, heat_flow, heat_run, heat_step
from cme213x.utils.params import SimParams

ARITH = {"exact": ("pipe4", "naive"), "fma": ("pipe4_fma", "fma"), "fast": ("pipe4_fast", "fast")}


def _grid(n, m, device, seed):
    p = SimParams(nx=n, ny=m, order=8, flavor="hw5")
    g = HeatGrid(p, torch.float32, device)
    gen = torch.Generator().manual_seed(seed)
    r = torch.rand(g.buf[0].shape, generator=gen) * 10.0
    g.buf[0].copy_(r.to(device))
    g.buf[1].copy_(r.to(device))
    return g


def _per_pass(g, region, npass, arith):
    """npass one-pass launches (production heat_run)."""
    a, b = g.buf[0].clone(), g.buf[1].clone()
    out = heat_run(a, b, region, 8, g.xcfl, g.ycfl, 4 * npass, ARITH[arith][0])
    return out.clone()


@pytest.mark.gpu
@pytest.mark.parametrize("arith", ["fma", "fast", "exact"])
@pytest.mark.parametrize("shape,npass", [((1500, 1100), 2), ((2000, 1703), 5), ((4096, 4096), 3)])
def test_flow_equals_per_pass_launches(gpu, tune_lib, arith, shape, npass):
    g = _grid(*shape, gpu, seed=npass)
    region = g.interior
    ref = _per_pass(g, region, npass, arith)
    a, b = g.buf[0].clone(), g.buf[1].clone()
    out = heat_flow(a, b, region, 8, g.xcfl, g.ycfl, npass, fma=arith)
    assert out.data_ptr() == (b if npass % 2 else a).data_ptr()
    assert torch.equal(out, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("arith", ["fma", "fast"])
def test_flow_equals_cpu_oracle(gpu, tune_lib, arith):
    """Against the CPU oracle's single steps (13 steps = three flow passes
    + a one-step remainder through heat_run)."""
    n, m, iters = 700, 523, 13
    c = _grid(n, m, "cpu", seed=3)
    g = _grid(n, m, gpu, seed=3)
    a, b = c.buf[0].clone(), c.buf[1].clone()
    for i in range(iters):
        src, dst = (a, b) if i % 2 == 0 else (b, a)
        heat_step(src, dst, c.interior, 8, c.xcfl, c.ycfl, ARITH[arith][1])
    ref = a if iters % 2 == 0 else b
    a, b = g.buf[0].clone(), g.buf[1].clone()
    mid = heat_flow(a, b, g.interior, 8, g.xcfl, g.ycfl, 3, fma=arith)
    other = a if mid.data_ptr() == b.data_ptr() else b
    out = heat_run(mid, other, g.interior, 8, g.xcfl, g.ycfl, iters - 12, ARITH[arith][0])
    assert torch.equal(out.cpu(), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("per_cu", [24, 64])
def test_flow_many_small_tasks_uneven(gpu, tune_lib, per_cu):
    """Many short tasks (16-40-row chunks: dependency waits on every pass
    boundary, tasks of unequal cost at the ragged right and bottom edges) and
    a sub-region that is not the whole interior."""
    from cme213x.utils import tuning

    g = _grid(3000, 2500, gpu, seed=9)
    region = (13, 2900, 9, 2411)
    ref = _per_pass(g, region, 6, "fma")
    with tuning.override(flow_per_cu=per_cu):
        for _ in range(2):
            out = heat_flow(g.buf[0].clone(), g.buf[1].clone(), region, 8, g.xcfl, g.ycfl, 6, fma="fma")
            assert torch.equal(out, ref)


@pytest.mark.gpu
def test_flow_trace_and_schedule(gpu, tune_lib):
    """The profiling launch records every ticket once; pass p + 1 of a task
    starts only after its neighbourhood's pass p ended (wall clock)."""
    g = _grid(2048, 2048, gpu, seed=4)
    npass = 4
    ref = _per_pass(g, g.interior, npass, "fma")
    out, tr, tpp = heat_flow(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, npass, fma="fma",
                             trace=True)
    assert torch.equal(out, ref)
    assert tr.shape[0] == tpp * npass and bool((tr[:, 2] > 0).all())
    assert bool((tr[:, 1] >= tr[:, 0]).all()) and bool((tr[:, 2] >= tr[:, 1]).all())
    strips = 5  # ceil(2048 / 480)
    nch = tpp // strips
    for p in range(1, npass):
        for t in range(tpp):
            s, c = t % strips, t // strips
            start = int(tr[p * tpp + t, 1])
            for dc in (-1, 0, 1):
                for ds in (-1, 0, 1):
                    s2, c2 = s + ds, c + dc
                    if 0 <= s2 < strips and 0 <= c2 < nch:
                        assert start >= int(tr[(p - 1) * tpp + c2 * strips + s2, 2])


@pytest.mark.gpu
def test_flow_timeout_raises_and_drains(gpu, tune_lib):
    """A dependency wait that gives up (knob flow_spins = 1) aborts every
    workgroup (the grid drains, no hang) and raises; the next call runs."""
    from cme213x.utils import tuning

    g = _grid(4096, 4096, gpu, seed=5)
    # diagnostics mode 2048: the first task never publishes its completion
    with tuning.override(flow_spins=1 << 12, flow_mode=2048):
        with pytest.raises(RuntimeError, match="gave up"):
            heat_flow(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, 8, fma="fma")
    assert not flow_timed_out()
    ref = _per_pass(g, g.interior, 2, "fma")
    assert torch.equal(heat_flow(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, 2), ref)


def test_flow_refuses_other_shapes():
    g = _grid(100, 100, "cpu", seed=1)
    with pytest.raises(ValueError, match="fp32, order 8"):
        heat_flow(g.buf[0], g.buf[1], g.interior, 8, g.xcfl, g.ycfl, 2)


@pytest.mark.gpu
def test_flow_banded_stress_distinct_buffers(gpu, tune_lib):
    """The XCD-banded hand-off (band-edge rows write-through, no L2 write-
    back) on buffers whose interiors differ, so a task reading a stale or
    wrong buffer shows: 2 and 6 passes, several repetitions (the ticket race
    fixed this round failed about one run in five here)."""
    g = _grid(4096, 4096, gpu, seed=13)
    xb, xe, yb, ye = g.interior
    gen = torch.Generator().manual_seed(14)
    g.buf[1, yb:ye, xb:xe] = (torch.rand((ye - yb, xe - xb), generator=gen) * 10.0).to(gpu)
    for npass in (2, 6):
        ref = _per_pass(g, g.interior, npass, "fma")
        for _ in range(4):
            out = heat_flow(g.buf[0].clone(), g.buf[1].clone(), g.interior, 8, g.xcfl, g.ycfl, npass, fma="fma")
            assert torch.equal(out, ref)
