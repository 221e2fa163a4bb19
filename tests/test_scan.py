"""Scan / reduce / segmented scan vs numpy fp64 oracles; the final project's
SpMV-scan against the reference checker's small fixture and the fp64
serial algorithm."""
import os

import numpy as np
import pytest
import torch

from cme213x.models.spmv_scan import (SpmvScanSolver, errors, generate, load,
                                      reference_solution, reference_solution_quadratic, run_fp, save)
from cme213x.ops.scan import head_flags_from_offsets, lookback_timed_out, reduce, scan, segmented_scan

SMALL = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def _np_segscan(v, heads):
    out = np.empty_like(v, dtype=np.float64)
    run = 0.0
    for i, x in enumerate(v.astype(np.float64)):
        run = x if (i == 0 or heads[i]) else run + x
        out[i] = run
    return out


@pytest.mark.parametrize("exclusive", [False, True])
@pytest.mark.parametrize("dtype", [torch.int32, torch.float32])
def test_scan_cpu(exclusive, dtype):
    x = torch.randint(-5, 6, (10007,), dtype=torch.int32).to(dtype)
    y = scan(x, exclusive)
    ref = np.cumsum(x.numpy().astype(np.float64))
    if exclusive:
        ref = np.concatenate([[0], ref[:-1]])
    np.testing.assert_array_equal(y.numpy().astype(np.float64), ref)


def test_reduce_cpu():
    x = torch.arange(1000, dtype=torch.int32)
    assert reduce(x).item() == 499500
    assert reduce(x, "max").item() == 999
    assert reduce(x, "min").item() == 0


def test_segscan_cpu_and_flags():
    rng = np.random.default_rng(1)
    n = 5000
    s = np.concatenate([[0], np.sort(rng.choice(np.arange(1, n), 300, replace=False)), [n]]).astype(np.int32)
    heads = np.zeros(n, bool)
    heads[s[:-1]] = True
    v = rng.standard_normal(n).astype(np.float32)
    ref = _np_segscan(v, heads)
    for bitmask in (True, False):
        f = head_flags_from_offsets(torch.from_numpy(s), n, bitmask=bitmask)
        out = segmented_scan(torch.from_numpy(v), f)
        np.testing.assert_allclose(out.numpy(), ref, rtol=1e-4, atol=1e-4)


def test_small_fixture_matches_reference_output():
    a_path, x_path = os.path.join(SMALL, "small_a.txt"), os.path.join(SMALL, "small_x.txt")
    if not os.path.exists(a_path):
        pytest.skip("reference fixture not mounted")
    prob = load(a_path, x_path)
    ref = reference_solution(prob)
    b_ref = np.fromfile(os.path.join(SMALL, "small_b.txt"), sep=" ")
    np.testing.assert_allclose(ref, b_ref, rtol=1e-6)  # small_b.txt is single precision on purpose
    sol = SpmvScanSolver(prob, "cpu")
    out = sol.run().numpy()
    np.testing.assert_allclose(out, b_ref, rtol=1e-6)
    # the older checker's O(len^2) algorithm agrees (aux/CheckOutput/serialMV.cu)
    np.testing.assert_allclose(reference_solution_quadratic(prob), ref, rtol=1e-12)


def test_quadratic_checker_matches_vectorised():
    prob = generate(600, 40, 50, 3, seed=9)
    np.testing.assert_allclose(reference_solution_quadratic(prob), reference_solution(prob), rtol=1e-9, atol=1e-9)


def test_generator_and_io_roundtrip(tmp_path):
    prob = generate(2000, 150, 500, 3, seed=2)
    prob.validate()
    save(prob, str(tmp_path / "a.txt"), str(tmp_path / "x.txt"))
    q = load(str(tmp_path / "a.txt"), str(tmp_path / "x.txt"))
    assert q.iters == 3 and np.array_equal(q.s, prob.s) and np.array_equal(q.k, prob.k)
    np.testing.assert_array_equal(q.a, prob.a)
    os.chdir(tmp_path)
    res = run_fp(str(tmp_path / "a.txt"), str(tmp_path / "x.txt"), cpu_check=True, device="cpu")
    assert res["relL2"] < 1e-5
    assert (tmp_path / "b.txt").exists()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 1000, 4096, 4097, 1 << 20, 3_000_001, 9_000_011])
@pytest.mark.parametrize("dtype", [torch.int32, torch.float32])
@pytest.mark.parametrize("exclusive", [False, True])
@pytest.mark.parametrize("algo", ["lookback", "rts", "blelloch", "hillis"])
def test_scan_single_pass_gpu(gpu, n, dtype, exclusive, algo):
    x = torch.randint(-3, 4, (n,), dtype=torch.int32).to(dtype)
    ref = np.cumsum(x.numpy().astype(np.int64))
    if exclusive:
        ref = np.concatenate([[0], ref[:-1]])
    y = scan(x.to(gpu), exclusive, algo=algo).cpu().numpy().astype(np.int64)
    np.testing.assert_array_equal(y, ref)  # small integers: exact in fp32 too
    if algo == "lookback":
        assert not lookback_timed_out(gpu)


@pytest.mark.gpu
def test_scan_uint32_gpu(gpu):
    x = torch.randint(0, 100, (1 << 18,), dtype=torch.int32)
    y = scan(x.to(gpu).view(torch.uint32), exclusive=True).view(torch.int32).cpu()
    ref = torch.cumsum(x.to(torch.int64), 0) - x
    assert torch.equal(y.to(torch.int64), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["blelloch_mlevel", "hillis_mlevel"])
@pytest.mark.parametrize("n", [5, 512, 513, 262145, 1 << 20])
def test_scan_mlevel_gpu(gpu, algo, n):
    x = torch.randint(-3, 4, (n,), dtype=torch.int32)
    for excl in (True, False):
        ref = np.cumsum(x.numpy().astype(np.int64))
        if excl:
            ref = np.concatenate([[0], ref[:-1]])
        y = scan(x.to(gpu), excl, algo=algo).cpu().numpy()
        np.testing.assert_array_equal(y, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("op", ["sum", "max", "min"])
@pytest.mark.parametrize("algo", ["vector", "tree"])
def test_reduce_gpu(gpu, op, algo):
    if algo == "tree" and op != "sum":
        pytest.skip("tree variant is sum-only")
    x = torch.randint(-1000, 1000, (3_000_017,), dtype=torch.int32)
    ref = {"sum": x.sum(), "max": x.max(), "min": x.min()}[op].item()
    assert reduce(x.to(gpu), op, algo).item() == ref
    xf = torch.randn(1_000_003)
    r = reduce(xf.to(gpu), op, algo).item()
    rf = {"sum": xf.double().sum(), "max": xf.max(), "min": xf.min()}[op].item()
    assert abs(r - rf) <= 1e-3 * max(1.0, abs(rf))


@pytest.mark.gpu
@pytest.mark.parametrize("nseg", [1, 7, 1000, 200000])
@pytest.mark.parametrize("bitmask", [True, False])
def test_segscan_gpu(gpu, nseg, bitmask):
    rng = np.random.default_rng(nseg)
    n = 1_000_003
    s = np.concatenate([[0], np.sort(rng.choice(np.arange(1, n), nseg - 1, replace=False)), [n]]).astype(np.int32)
    v = rng.integers(-4, 5, n).astype(np.float32)  # integers: exact sums
    m = rng.integers(-2, 3, n).astype(np.float32)
    heads = np.zeros(n, bool)
    heads[s[:-1]] = True
    ref = _np_segscan(v * m, heads)
    f = head_flags_from_offsets(torch.from_numpy(s), n, gpu, bitmask)
    out = segmented_scan(torch.from_numpy(v).to(gpu), f, mul=torch.from_numpy(m).to(gpu)).cpu().numpy()
    np.testing.assert_array_equal(out.astype(np.float64), ref)
    assert not lookback_timed_out(gpu)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(37035, 3128, 6), (3_105_536, 1_000_004, 3), (4_000_000, 1999, 3)])
@pytest.mark.parametrize("algo", ["lookback", "wave", "serial"])
def test_spmv_scan_gpu_vs_fp64(gpu, shape, algo):
    n, p, N = shape
    prob = generate(n, p, 10000, N, seed=5)
    sol = SpmvScanSolver(prob, gpu, algo)
    b = sol.run().cpu().numpy()
    e = errors(reference_solution(prob), b)
    assert e["relL2"] < 1e-5, e


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(1_200_000, 200_000, 70), (300_000, 20_000, 130)])
def test_spmv_scan_fused_steps_long_runs(gpu, shape):
    """The one-launch multi-step kernel on the 2-rows-per-lane tiling, with
    more steps than one launch holds (64): the run is split into launches,
    each with its own per-step descriptor sets."""
    n, p, N = shape
    prob = generate(n, p, 10000, N, seed=9)
    sol = SpmvScanSolver(prob, gpu, "lookback")
    b = sol.run().cpu().numpy()
    step = SpmvScanSolver(prob, gpu, "lookback")  # one segmented_scan launch per step
    for _ in range(N):
        step.step()
    e_steps = errors(step.a.cpu().numpy().astype(np.float64), b)
    assert e_steps["relL2"] < 2e-6 * N, e_steps  # same arithmetic; tiling changes the association only
    e = errors(reference_solution(prob), b)
    assert e["relL2"] < 2e-6 * N, e  # fp32 rounding grows with the number of steps
    assert not lookback_timed_out(gpu)


@pytest.mark.gpu
def test_lookback_epochs_reuse_workspace(gpu):
    """Back-to-back look-back scans share one descriptor array with a new
    epoch per launch (no memset): changing inputs, sizes, exclusive/inclusive,
    dtypes and a segmented scan in between must all stay exact; then a
    captured graph (epoch 0, memset inside the graph) replayed on new data,
    followed by more eager scans."""
    g = torch.Generator().manual_seed(7)
    outs = []
    for i in range(12):
        n = [1 << 20, 3 << 18, 12345, 1 << 22][i % 4]
        x = torch.randint(-50, 50, (n,), generator=g, dtype=torch.int32)
        ex = bool(i % 3 == 1)
        y = scan(x.to(gpu), exclusive=ex, algo="lookback")
        ref = torch.cumsum(x.long(), 0)
        if ex:
            ref = ref - x.long()
        outs.append((y, ref))
        if i == 5:
            f = torch.zeros(n, dtype=torch.uint8)
            f[::1000] = 1
            xs = torch.rand(n, generator=g)
            segmented_scan(xs.to(gpu), f.to(gpu))
    for y, ref in outs:
        assert torch.equal(y.cpu().long(), ref)
    x = torch.randint(-9, 9, (1 << 21,), dtype=torch.int32, device=gpu)
    out = torch.empty_like(x)
    scan(x, out=out, algo="lookback")  # warm-up outside the capture
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        scan(x, out=out, algo="lookback")
    for _ in range(3):
        x.copy_(torch.randint(-9, 9, (1 << 21,), dtype=torch.int32, generator=g).to(gpu))
        graph.replay()
        assert torch.equal(out.cpu().long(), torch.cumsum(x.cpu().long(), 0))
        y = scan(x, algo="lookback")
        assert torch.equal(y.cpu().long(), torch.cumsum(x.cpu().long(), 0))
    assert not lookback_timed_out(gpu)
