"""2-D heat stencil: CPU oracle vs plain-PyTorch fp64, HIP kernels vs the CPU
oracle (bitwise / 10 ULP, the reference's checkErrors criterion), reference
I/O formats, checkpoint/restart."""
import os

import numpy as np
import pytest
import torch

from cme213x.models.heat2d import HeatGrid, check_errors, run_hw2
from cme213x.ops.stencil import heat_step_torch
from cme213x.utils.params import SimParams
from cme213x.utils.ulp import ulp_distance

REF_PARAMS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "hw2_params_test.in")


def _rand_grid(p, dtype, device="cpu", seed=0):
    g = HeatGrid(p, dtype, device)
    gen = torch.Generator().manual_seed(seed)
    r = torch.rand(g.buf[0].shape, generator=gen, dtype=dtype)
    g.buf[0].copy_(r)
    g.buf[1].copy_(r)
    return g


@pytest.mark.parametrize("order", [2, 4, 8])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_cpu_oracle_matches_torch(order, dtype):
    p = SimParams(nx=41, ny=23, order=order)
    g = _rand_grid(p, dtype)
    ref = g.buf[0].double().clone()
    for _ in range(3):
        ref = heat_step_torch(ref, g.interior, order, g.xcfl, g.ycfl)
    g.run(3, "naive")
    tol = 1e-5 if dtype == torch.float32 else 1e-12
    assert (g.curr().double() - ref).abs().max().item() < tol


def test_params_cfl_and_banner():
    p = SimParams(nx=2000, ny=2000, order=8, iters=10)
    assert p.gx == 2008 and p.border == 4
    dx2 = p.dx ** 2
    assert abs(p.dt - (0.5 - 0.0001) * (5040 * dx2 * dx2) / (8064 * (2 * dx2))) < 1e-18
    assert "xcfl" in p.banner()


def test_params_file_roundtrip(tmp_path):
    if os.path.exists(REF_PARAMS):
        p = SimParams.from_file(REF_PARAMS)
        assert p.order in (2, 4, 8)
    p = SimParams(nx=50, ny=40, order=4, flavor="hw5", grid_method=2, sync=False)
    f = tmp_path / "params.in"
    p.to_file(str(f))
    q = SimParams.from_file(str(f), flavor="hw5")
    assert (q.nx, q.ny, q.order, q.grid_method, q.sync) == (50, 40, 4, 2, False)


def test_boundary_layout_matches_reference():
    p = SimParams(nx=6, ny=5, order=2, ic=5, bc=(1, 2, 3, 4))
    st = HeatGrid(p).state()
    assert st[0, 3] == 3 and st[-1, 3] == 1  # bottom row 0, top row gy-1
    assert st[0, 0] == 2 and st[-1, -1] == 4  # corners carry left/right
    assert st[3, 3] == 5


def test_grid_text_format(tmp_path):
    p = SimParams(nx=4, ny=3, order=2, ic=5, bc=(0, 10, 0, 10))
    g = HeatGrid(p)
    os.chdir(tmp_path)
    g.save_text("init")
    txt = open(tmp_path / "grid_init.txt").read()
    lines = txt.split("\n")
    assert lines[0] == "   10     0     0     0     0    10 "
    assert lines[2] == "   10     5     5     5     5    10 "
    assert txt.endswith(" \n\n\n")


def test_checkpoint_restart(tmp_path):
    p = SimParams(nx=30, ny=20, order=4)
    a = _rand_grid(p, torch.float64)
    a.run(5, "naive")
    a.checkpoint(str(tmp_path / "ck.safetensors"))
    a.run(4, "naive")
    b = HeatGrid(p, torch.float64)
    b.restore(str(tmp_path / "ck.safetensors"))
    assert b.iteration == 5
    b.run(4, "naive")
    assert np.array_equal(a.state(), b.state())


def test_ulp_compare():
    a = np.array([1.0, -1.0, 0.0, 1e-30], np.float32)
    b = np.nextafter(a, np.float32(np.inf))
    assert ulp_distance(a, b).tolist() == [1, 1, 1, 1]
    a64 = np.array([-2.0, 3.0])
    b64 = np.nextafter(np.nextafter(a64, -np.inf), -np.inf)
    assert ulp_distance(a64, b64).tolist() == [2, 2]


@pytest.mark.gpu
@pytest.mark.parametrize("order", [2, 4, 8])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("variant", ["global", "shared", "lds_nopad", "stream"])
def test_gpu_variants_bitwise(gpu, order, dtype, variant):
    # odd sizes exercise strip/vector edges; random data is sensitive to
    # any neighbour mix-up
    p = SimParams(nx=517, ny=263, order=order)
    c = _rand_grid(p, dtype)
    g = _rand_grid(p, dtype, gpu)
    c.run(3, "naive")
    g.run(3, variant)
    torch.cuda.synchronize()
    d = ulp_distance(c.state(), g.state())
    assert int(d.max()) == 0, f"max ulp {int(d.max())}"


@pytest.mark.gpu
@pytest.mark.parametrize("region", [(4, 300, 4, 100), (9, 250, 17, 77), (130, 131, 5, 200)])
def test_gpu_stream_subregion(gpu, region):
    p = SimParams(nx=300, ny=250, order=8)
    c = _rand_grid(p, torch.float32)
    g = _rand_grid(p, torch.float32, gpu)
    c.step("naive", region)
    g.step("stream", region)
    torch.cuda.synchronize()
    assert np.array_equal(c.state(), g.state())


@pytest.mark.gpu
@pytest.mark.parametrize("order", [2, 4, 8])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("iters", [1, 2, 5])
def test_gpu_stream2_temporal_blocking_bitwise(gpu, order, dtype, iters):
    # two steps per HBM pass must equal two single steps bit for bit
    p = SimParams(nx=517, ny=263, order=order)
    c = _rand_grid(p, dtype)
    g = _rand_grid(p, dtype, gpu)
    c.run(iters, "naive")
    g.run(iters, "stream2")
    torch.cuda.synchronize()
    d = ulp_distance(c.state(), g.state())
    assert int(d.max()) == 0, f"max ulp {int(d.max())}"


@pytest.mark.gpu
@pytest.mark.parametrize("order", [2, 4, 8])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("variant,iters", [("stream_fma", 3), ("stream2_fma", 1), ("stream2_fma", 4), ("stream2_fma", 7)])
def test_gpu_fma_variants_bitwise_vs_fma_oracle(gpu, order, dtype, variant, iters):
    p = SimParams(nx=517, ny=263, order=order)
    c = _rand_grid(p, dtype)
    g = _rand_grid(p, dtype, gpu)
    c.run(iters, "fma")
    g.run(iters, variant)
    torch.cuda.synchronize()
    d = ulp_distance(c.state(), g.state())
    assert int(d.max()) == 0, f"max ulp {int(d.max())}"


def test_fma_oracle_within_reference_tolerance():
    """The FMA-contracted stencil stays within the reference's 10-ULP
    criterion of the exact oracle (hw2 checkErrors)."""
    p = SimParams(nx=120, ny=90, order=8)
    a = _rand_grid(p, torch.float32)
    b = _rand_grid(p, torch.float32)
    a.run(10, "naive")
    b.run(10, "fma")
    assert check_errors(a.state(), b.state(), p.border) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("region", [(4, 300, 4, 100), (9, 250, 17, 77), (130, 131, 5, 200), (8, 292, 8, 242)])
@pytest.mark.parametrize("chunk", [0, 8, 12])
@pytest.mark.parametrize("fma", [False, True])
def test_gpu_stream2_subregion(gpu, region, chunk, fma):
    from cme213x.ops.stencil import heat_run
    p = SimParams(nx=300, ny=250, order=8)
    c = _rand_grid(p, torch.float32)
    g = _rand_grid(p, torch.float32, gpu)
    ca, cb = c.buf[0].clone(), c.buf[0].clone()
    ga, gb = g.buf[0].clone(), g.buf[0].clone()
    oc = heat_run(ca, cb, region, 8, c.xcfl, c.ycfl, 4, "fma" if fma else "naive")
    og = heat_run(ga, gb, region, 8, g.xcfl, g.ycfl, 4, "stream2_fma" if fma else "stream2", chunk)
    torch.cuda.synchronize()
    assert torch.equal(oc, og.cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("order", [2, 4, 8])
@pytest.mark.parametrize("ns", [3, 4])
@pytest.mark.parametrize("fma", [False, True])
@pytest.mark.parametrize("iters", [1, 4, 7, 9])
def test_gpu_streamn_temporal_blocking_bitwise(gpu, order, ns, fma, iters):
    # 3 / 4 steps per HBM pass (+ two-step and single-step tails) must equal
    # single steps bit for bit, exact and FMA
    p = SimParams(nx=517, ny=263, order=order)
    c = _rand_grid(p, torch.float32)
    g = _rand_grid(p, torch.float32, gpu)
    c.run(iters, "fma" if fma else "naive")
    g.run(iters, f"stream{ns}" + ("_fma" if fma else ""))
    torch.cuda.synchronize()
    d = ulp_distance(c.state(), g.state())
    assert int(d.max()) == 0, f"max ulp {int(d.max())}"


@pytest.mark.gpu
@pytest.mark.parametrize("region", [(4, 300, 4, 100), (9, 250, 17, 77), (130, 131, 5, 200), (8, 292, 8, 242)])
@pytest.mark.parametrize("chunk", [0, 8, 14])
@pytest.mark.parametrize("ns", [3, 4])
def test_gpu_streamn_subregion(gpu, region, chunk, ns):
    from cme213x.ops.stencil import heat_run
    p = SimParams(nx=300, ny=250, order=8)
    c = _rand_grid(p, torch.float32)
    g = _rand_grid(p, torch.float32, gpu)
    ca, cb = c.buf[0].clone(), c.buf[0].clone()
    ga, gb = g.buf[0].clone(), g.buf[0].clone()
    oc = heat_run(ca, cb, region, 8, c.xcfl, c.ycfl, 2 * ns, "fma")
    og = heat_run(ga, gb, region, 8, g.xcfl, g.ycfl, 2 * ns, f"stream{ns}_fma", chunk)
    torch.cuda.synchronize()
    assert torch.equal(oc, og.cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("ns", [2, 3, 4])
def test_gpu_stepn_multi_region_ext(gpu, ns):
    """heat_stepn with several output regions in one launch and an
    intermediate region grown past the output (the distributed border-strip
    pass) equals the CPU composition of single steps."""
    from cme213x.ops.stencil import heat_stepn
    p = SimParams(nx=300, ny=250, order=8)
    c = _rand_grid(p, torch.float32)
    g = _rand_grid(p, torch.float32, gpu)
    regs = [(4, 304, 4, 40), (4, 304, 220, 254), (4, 40, 40, 220), (270, 304, 40, 220)]
    ext = (4, 304, 4, 254)
    oc, og = c.buf[0].clone(), g.buf[0].clone()
    heat_stepn(c.buf[0], oc, regs, ext, 8, c.xcfl, c.ycfl, ns, fma=True)
    heat_stepn(g.buf[0], og, regs, ext, 8, g.xcfl, g.ycfl, ns, fma=True)
    torch.cuda.synchronize()
    assert torch.equal(oc, og.cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("order", [2, 4, 8])
@pytest.mark.parametrize("fma", [False, True])
@pytest.mark.parametrize("iters", [3, 7, 8])
def test_gpu_stream3_fp64_matches_single_steps(gpu, order, fma, iters):
    """fp64 three-step passes (one row per register block) + tails equal the
    CPU single steps bit for bit -- the hw5 precision (2dHeat_solution.cpp:63-84)."""
    p = SimParams(nx=517, ny=263, order=order)
    c = _rand_grid(p, torch.float64)
    g = _rand_grid(p, torch.float64, gpu)
    c.run(iters, "fma" if fma else "naive")
    g.run(iters, "stream3" + ("_fma" if fma else ""))
    torch.cuda.synchronize()
    assert np.array_equal(c.state(), g.state())


@pytest.mark.gpu
@pytest.mark.parametrize("region", [(4, 300, 4, 100), (9, 250, 17, 77), (8, 292, 8, 242)])
@pytest.mark.parametrize("chunk", [0, 5])
def test_gpu_stream3_fp64_subregion(gpu, region, chunk):
    from cme213x.ops.stencil import heat_run
    p = SimParams(nx=300, ny=250, order=8)
    c = _rand_grid(p, torch.float64)
    g = _rand_grid(p, torch.float64, gpu)
    ca, cb = c.buf[0].clone(), c.buf[0].clone()
    ga, gb = g.buf[0].clone(), g.buf[0].clone()
    oc = heat_run(ca, cb, region, 8, c.xcfl, c.ycfl, 6, "fma")
    og = heat_run(ga, gb, region, 8, g.xcfl, g.ycfl, 6, "stream3_fma", chunk)
    torch.cuda.synchronize()
    assert torch.equal(oc, og.cpu())


def test_streamn_is_fp32_only():
    from cme213x.ops.stencil import heat_run
    p = SimParams(nx=40, ny=30, order=2)
    c = _rand_grid(p, torch.float64)
    with pytest.raises(ValueError):
        heat_run(c.buf[0], c.buf[1], c.interior, 2, c.xcfl, c.ycfl, 4, "stream4")


def test_stream2_rejected_for_single_step():
    p = SimParams(nx=40, ny=30, order=2)
    c = _rand_grid(p, torch.float32)
    with pytest.raises(ValueError):
        c.step("stream2")


@pytest.mark.gpu
def test_hw2_driver_gpu(gpu, tmp_path):
    p = SimParams(nx=200, ny=150, iters=10, order=8)
    f = tmp_path / "params.in"
    p.to_file(str(f))
    res = run_hw2(str(f), outdir=str(tmp_path))
    for v, r in res["variants"].items():
        assert r["errors"] == 0, v
    assert (tmp_path / "grid_final_gpu.txt").exists()
    assert (tmp_path / "grid_final_cpu.txt").exists()


def test_hw2_driver_cpu(tmp_path):
    p = SimParams(nx=60, ny=40, iters=10, order=4)
    f = tmp_path / "params.in"
    p.to_file(str(f))
    res = run_hw2(str(f), device="cpu", outdir=str(tmp_path))
    assert res["cpu_ms"] >= 0
    assert (tmp_path / "grid_init.txt").exists()


def test_checkpoint_writer_reports_errors(tmp_path):
    """A write error of the background checkpoint writer is raised by wait(),
    and a good writer returns its paths with the files complete."""
    import numpy as np

    from cme213x.models.heat2d_dist import CheckpointWriter
    from cme213x.utils.gridio import load_checkpoint

    t = torch.arange(12, dtype=torch.float32).reshape(3, 4)
    ok = CheckpointWriter(str(tmp_path), [(0, t, {"iteration": 3}, None)])
    paths = ok.wait()
    assert ok.done() and len(paths) == 1
    got, meta = load_checkpoint(paths[0])
    assert np.array_equal(got["interior"], t.numpy()) and meta["iteration"] == "3"
    bad = CheckpointWriter(str(tmp_path / "missing" / "dir"), [(0, t, {"iteration": 3}, None)])
    with pytest.raises(Exception):
        bad.wait()
