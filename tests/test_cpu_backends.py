"""The OpenMP CPU backends of the text and algorithm ops
(``csrc/cpu/text_cpu.cpp``, ``csrc/cpu/algorithms_cpu.cpp``) against plain
numpy / PyTorch oracles, on sizes that split unevenly over the threads and on
the edge cases (empty inputs, runs across thread boundaries, ties)."""
import numpy as np
import pytest
import torch

import cme213x  # noqa: F401
from cme213x.ops import algorithms as A
from cme213x.ops import text as T

SIZES = [0, 1, 7, 1000, 100_003]


def _text(n, seed=0, letters_only=False):
    rng = np.random.default_rng(seed)
    if letters_only:
        return torch.from_numpy(rng.integers(ord("a"), ord("z") + 1, n, dtype=np.uint8))
    return torch.from_numpy(rng.integers(0, 256, n, dtype=np.uint8))


@pytest.mark.parametrize("n", SIZES)
def test_text_histograms(n):
    raw = _text(n, 1)
    assert torch.equal(T.histogram_u8(raw), T.ref_histogram_u8(raw))
    assert torch.equal(T.histogram_u8(raw, 32, 100), T.ref_histogram_u8(raw, 32, 100))
    clean = _text(n, 2, letters_only=True)
    assert torch.equal(T.letter_histogram(clean), T.ref_histogram_u8(clean, ord("a"), 26))
    assert torch.equal(T.digraph_histogram(clean), T.ref_digraph_histogram(clean))
    for p in (1, 3, 11, 500):
        assert torch.equal(T.residue_histograms(clean, p), T.ref_residue_histograms(clean, p))


@pytest.mark.parametrize("n", SIZES)
def test_text_sanitize_vigenere_match(n):
    raw = _text(n, 3)
    assert torch.equal(T.sanitize(raw), T.ref_sanitize(raw))
    clean = _text(n, 4, letters_only=True)
    key = torch.tensor([3, 25, 0, 14, 1, 7, 9], dtype=torch.int32)
    enc = T.vigenere(clean, key)
    assert torch.equal(enc, T.ref_vigenere(clean, key))
    assert torch.equal(T.vigenere(enc, key, decode=True), clean)
    assert torch.equal(T.match_counts(clean, 1, 20), T.ref_match_counts(clean, 1, 20))
    assert torch.equal(T.match_counts(clean, max(1, n - 5), 10), T.ref_match_counts(clean, max(1, n - 5), 10))


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.int32, torch.int64, torch.uint8, torch.float64])
def test_selection_family(n, dtype):
    g = torch.Generator().manual_seed(n + 5)
    x = torch.randint(0, 4, (n,), generator=g).to(dtype)  # long runs of equal values
    fl = torch.rand(n, generator=g) < 0.4
    assert torch.equal(A.copy_if(x, fl), A.ref_copy_if(x, fl))
    assert torch.equal(A.copy_if(x, fl, invert=True), A.ref_copy_if(x, fl, invert=True))
    assert torch.equal(A.remove_value(x, 2), A.ref_remove_value(x, 2))
    assert torch.equal(A.unique(x), A.ref_unique(x))
    assert torch.equal(A.run_starts(x), A.ref_run_starts(x))
    assert torch.equal(A.nonzero(fl), A.ref_nonzero(fl))
    for f, r in ((A.stable_partition, A.ref_stable_partition), (A.split, A.ref_split)):
        (p, c), (pr, cr) = f(x, fl), r(x, fl)
        assert torch.equal(p, pr) and c == cr


@pytest.mark.parametrize("dtype", [torch.float32, torch.int32, torch.uint32, torch.int64, torch.float64])
@pytest.mark.parametrize("upper", [False, True])
def test_search(dtype, upper):
    g = torch.Generator().manual_seed(7)
    s = torch.sort(torch.randint(0, 1000, (5001,), generator=g))[0].to(dtype)
    q = torch.randint(-5, 1005, (3000,), generator=g).clamp(min=0 if dtype == torch.uint32 else -5).to(dtype)
    f = A.upper_bound if upper else A.lower_bound
    assert torch.equal(f(s, q), A.ref_search(s, q, upper))


@pytest.mark.parametrize("dtype", [torch.float32, torch.int32, torch.int64, torch.float64])
@pytest.mark.parametrize("op", ["sum", "max", "min"])
def test_segment_reduce(dtype, op):
    g = torch.Generator().manual_seed(11)
    lens = torch.randint(0, 9, (4000,), generator=g)
    lens[::17] = 0  # empty segments -> identity
    off = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(lens, 0)])
    vals = torch.randint(-50, 50, (int(off[-1]),), generator=g).to(dtype)
    got, want = A.segment_reduce(vals, off, op), A.ref_segment_reduce(vals, off, op)
    if dtype.is_floating_point and op == "sum":
        torch.testing.assert_close(got, want)
    else:
        assert torch.equal(got, want)


@pytest.mark.parametrize("dtype", [torch.float32, torch.int32, torch.int64, torch.float64])
def test_arg_reduce_first_index_on_ties(dtype):
    g = torch.Generator().manual_seed(13)
    for n in (1, 9, 100_001):
        x = torch.randint(-20, 20, (n,), generator=g).to(dtype)
        assert A.max_element(x) == A.ref_arg(x, True)
        assert A.min_element(x) == A.ref_arg(x, False)


def test_inner_product_and_counting_sort():
    g = torch.Generator().manual_seed(17)
    a, b = torch.rand(100_003, generator=g), torch.rand(100_003, generator=g)
    assert abs(A.inner_product(a, b) - A.ref_inner_product(a, b)) < 1e-9 * 1e5
    x, y = torch.randint(0, 3, (50_001,), generator=g, dtype=torch.int32), \
        torch.randint(0, 3, (50_001,), generator=g, dtype=torch.int32)
    assert A.inner_product(x, y, "eq") == A.ref_inner_product(x, y, "eq")
    k = torch.randint(0, 300, (70_000,), generator=g, dtype=torch.int32)
    v = torch.arange(70_000, dtype=torch.int32)
    ks, vs = A.counting_sort(k, 300, v)
    kr, idx = torch.sort(k, stable=True)
    assert torch.equal(ks, kr) and torch.equal(vs, v[idx])
    assert torch.equal(A.counting_sort(k.long(), 300), kr.long())
