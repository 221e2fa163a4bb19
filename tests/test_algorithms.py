"""Thrust-equivalent algorithm layer (ops/algorithms.py): GPU kernels vs the
plain-PyTorch CPU oracle; CPU semantics vs numpy."""
import numpy as np
import pytest
import torch

from cme213x.ops import algorithms as A

SIZES = [1, 17, 4096, 4097, 100_003, 1 << 20]


def _data(n, dtype, seed=0, lo=0, hi=50):
    g = torch.Generator().manual_seed(seed)
    if dtype.is_floating_point:
        return torch.randint(lo, hi, (n,), generator=g).to(dtype) * 0.5
    return torch.randint(lo, hi, (n,), generator=g, dtype=torch.int64).to(dtype)


def test_cpu_semantics():
    x = torch.tensor([1, 1, 2, 3, 3, 3, 7], dtype=torch.int32)
    assert A.unique(x).tolist() == [1, 2, 3, 7]
    k, v = A.reduce_by_key(x, torch.arange(7, dtype=torch.float32))
    assert k.tolist() == [1, 2, 3, 7] and v.tolist() == [1.0, 2.0, 12.0, 6.0]
    assert A.histogram_dense(x, 8).tolist() == [0, 2, 1, 3, 0, 0, 0, 1]
    p, c = A.split(x, x > 2)
    assert c == 3 and p.tolist() == [1, 1, 2, 3, 3, 3, 7]
    p, c = A.stable_partition(x, x % 2 == 0)
    assert c == 1 and p.tolist() == [2, 1, 1, 3, 3, 3, 7]
    assert A.max_element(torch.tensor([1.0, 5.0, 5.0, 2.0])) == (5.0, 1)
    assert A.counting_sort(torch.tensor([3, 1, 2, 1]), 4).tolist() == [1, 1, 2, 3]


@pytest.mark.gpu
@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("dtype", [torch.uint8, torch.int32, torch.float32, torch.float64])
def test_select_family_gpu(gpu, n, dtype):
    x = _data(n, dtype)
    fl = _data(n, torch.int32, seed=1, hi=3) == 0
    xg, fg = x.to(gpu), fl.to(gpu)
    assert torch.equal(A.copy_if(xg, fg).cpu(), A.copy_if(x, fl))
    assert torch.equal(A.copy_if(xg, fg, invert=True).cpu(), A.copy_if(x, fl, invert=True))
    v = x[n // 2].item()
    assert torch.equal(A.remove_value(xg, v).cpu(), A.remove_value(x, v))
    pg, cg = A.stable_partition(xg, fg)
    pc, cc = A.stable_partition(x, fl)
    assert cg == cc and torch.equal(pg.cpu(), pc)
    sg, zg = A.split(xg, fg)
    sc, zc = A.split(x, fl)
    assert zg == zc and torch.equal(sg.cpu(), sc)
    assert torch.equal(A.nonzero(fg).cpu(), A.nonzero(fl))
    xs = torch.sort(x).values
    assert torch.equal(A.unique(xs.to(gpu)).cpu(), A.unique(xs))
    assert torch.equal(A.run_starts(xs.to(gpu)).cpu(), A.run_starts(xs))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 4097, 100_003, 3 * (1 << 22) + 5])
@pytest.mark.parametrize("dtype", [torch.int32, torch.float64])
def test_select_lookback_gpu(gpu, dtype, n, monkeypatch):
    """The single-pass look-back select (values, indices, unique; 12.6M items
    = ~3000 tiles = several rounds of the persistent grid) equals the CPU
    backend."""
    monkeypatch.setattr(A, "SELECT_ALGO", "lookback")
    x = _data(n, dtype, hi=1000)
    fl = _data(n, torch.int32, seed=2, hi=5) != 0
    xg, fg = x.to(gpu), fl.to(gpu)
    assert torch.equal(A.copy_if(xg, fg).cpu(), A.copy_if(x, fl))
    assert torch.equal(A.nonzero(fg).cpu(), A.nonzero(fl))
    xs = torch.sort(x).values
    assert torch.equal(A.unique(xs.to(gpu)).cpu(), A.unique(xs))
    from cme213x.ops.scan import lookback_timed_out
    assert not lookback_timed_out(gpu)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.int32, torch.float32, torch.float64, torch.int64, torch.uint32])
@pytest.mark.parametrize("upper", [False, True])
@pytest.mark.parametrize("m", [70_000, 300_000])  # 300K queries take the two-level splitter kernel
def test_search_gpu(gpu, dtype, upper, m):
    s = torch.sort(_data(200_001, torch.int64, hi=10_000)).values  # ~20 copies of each key: splitters inside runs
    q = _data(m, torch.int64, seed=5, lo=-5, hi=10_010)
    if dtype == torch.uint32:
        q = q.clamp(min=0)
    s, q = s.to(dtype), q.to(dtype)
    f = A.upper_bound if upper else A.lower_bound
    ref = torch.from_numpy(np.searchsorted(s.numpy().astype(np.float64), q.numpy().astype(np.float64),
                                           side="right" if upper else "left"))
    assert torch.equal(f(s.to(gpu), q.to(gpu)).cpu(), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.int32, torch.float32, torch.float64])
@pytest.mark.parametrize("op", ["sum", "max", "min"])
def test_reduce_by_key_gpu(gpu, dtype, op):
    keys = torch.sort(_data(300_000, torch.int32, hi=2000)).values
    keys[:5000] = -1  # one long segment
    vals = _data(300_000, dtype, seed=3, lo=-20, hi=20)
    kg, vg = A.reduce_by_key(keys.to(gpu), vals.to(gpu), op)
    kc, vc = A.reduce_by_key(keys, vals, op)
    assert torch.equal(kg.cpu(), kc)
    if dtype == torch.int32 or op != "sum":
        assert torch.equal(vg.cpu(), vc)
    else:
        torch.testing.assert_close(vg.cpu(), vc, rtol=1e-6, atol=1e-4)


@pytest.mark.gpu
def test_histograms_gpu(gpu):
    x = torch.sort(_data(1_000_000, torch.int32, hi=26)).values
    assert torch.equal(A.histogram_dense(x.to(gpu), 26).cpu(), torch.bincount(x, minlength=26))
    v, c = A.histogram_sparse(x.to(gpu))
    vc, cc = A.histogram_sparse(x)
    assert torch.equal(v.cpu(), vc) and torch.equal(c.cpu(), cc)


@pytest.mark.gpu
@pytest.mark.parametrize("num_keys", [2, 26, 256, 4000])
def test_counting_sort_gpu(gpu, num_keys):
    k = _data(500_000, torch.int32, hi=num_keys)
    v = torch.arange(k.numel(), dtype=torch.int32)
    kg, vg = A.counting_sort(k.to(gpu), num_keys, v.to(gpu))
    kc, vc = A.counting_sort(k, num_keys, v)
    assert torch.equal(kg.cpu(), kc) and torch.equal(vg.cpu(), vc)  # stable


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 1000, 3_000_001])
@pytest.mark.parametrize("dtype", [torch.float32, torch.int32, torch.float64])
def test_arg_reduce_gpu(gpu, n, dtype):
    x = _data(n, dtype, hi=1000)
    for f in (A.max_element, A.min_element):
        assert f(x.to(gpu)) == f(x)


@pytest.mark.gpu
def test_inner_product_gpu(gpu):
    a = torch.randn(2_000_003)
    b = torch.randn(2_000_003)
    assert abs(A.inner_product(a.to(gpu), b.to(gpu)) - A.inner_product(a, b)) < 1e-6 * 2e6 ** 0.5
    x = _data(1_000_000, torch.int32, hi=26)
    y = torch.roll(x, 7)
    assert A.inner_product(x.to(gpu), y.to(gpu), "eq") == A.inner_product(x, y, "eq")
