"""SpMV formats vs dense / fp64 oracles; format conversions; generators."""
import numpy as np
import pytest
import torch

from cme213x.ops.spmv import (CSR, hyb_k, laplacian, random_csr, spmv, to_coo, to_csr_aligned, to_csr_colblocked,
                               to_dia, to_ell, to_hyb)


def _ref(a: CSR, x):
    rp = a.rp.numpy().astype(np.int64)
    rows = np.repeat(np.arange(a.nrows), np.diff(rp))
    y = np.zeros(a.nrows)
    np.add.at(y, rows, a.val.numpy().astype(np.float64) * x.numpy().astype(np.float64)[a.col.numpy()])
    return y


@pytest.mark.parametrize("kind,n,deg", [("3pt", 50, 3), ("5pt", 20, 5), ("9pt", 12, 9), ("7pt", 6, 7), ("27pt", 5, 27)])
def test_laplacian_structure(kind, n, deg):
    a = laplacian(kind, n)
    lens = np.diff(a.rp.numpy())
    assert lens.max() == deg
    d = a.to_dense()
    assert torch.allclose(d, d.t())
    assert torch.allclose(d.sum(1)[lens == deg], torch.zeros(int((lens == deg).sum())))


def test_csr_cpu_and_conversions():
    a = random_csr(500, 400, 7, seed=1)
    x = torch.randn(400)
    ref = _ref(a, x)
    np.testing.assert_allclose(spmv(a, x).numpy(), ref, rtol=1e-4, atol=1e-4)
    ell, rest = to_ell(a)
    assert rest.nnz == 0 and ell.K == int(np.diff(a.rp.numpy()).max())
    hyb = to_hyb(a)
    assert hyb.ell.K == hyb_k(a)
    assert to_coo(a).nnz == a.nnz
    lap = laplacian("5pt", 10)
    dia = to_dia(lap)
    assert dia.offsets.tolist() == [-10, -1, 0, 1, 10]


@pytest.mark.gpu
@pytest.mark.parametrize("mat", ["5pt", "27pt", "random", "skew"])
@pytest.mark.parametrize("fmt", ["csr_scalar", "csr_vector", "csr_stream", "csr_short", "csr_wave", "csr_auto",
                                 "csr_aligned", "ell",
                                 "dia", "coo",
                                 "hyb", "csr_cb"])
def test_spmv_gpu(gpu, mat, fmt):
    if mat == "5pt":
        a = laplacian("5pt", 100)
    elif mat == "27pt":
        a = laplacian("27pt", 20)
    elif mat == "random":
        a = random_csr(20000, 15000, 12, seed=2)
    else:
        a = random_csr(20000, 20000, 20, seed=3, skew=True)
    if fmt == "dia" and mat in ("random", "skew"):
        pytest.skip("DIA only for structured matrices")
    x = torch.randn(a.ncols)
    ref = _ref(a, x)
    if fmt == "csr_cb":  # column blocks of 4 KB of x: several blocks even at these sizes
        dev = to_csr_colblocked(a, block_bytes=4096).to(gpu)
        assert len(dev.blocks) > 1 and dev.col0[0] == 0
        y = spmv(dev, x.to(gpu)).cpu().numpy()
        np.testing.assert_allclose(y, ref, rtol=1e-4, atol=1e-3)
        y0 = torch.randn(a.nrows, device=gpu)
        y1 = spmv(dev, x.to(gpu), y0.clone(), beta=0.5).cpu().numpy()
        np.testing.assert_allclose(y1, ref + 0.5 * y0.cpu().numpy(), rtol=1e-4, atol=1e-3)
        return
    dev = {"csr_scalar": a, "csr_vector": a, "csr_stream": a, "csr_short": a, "csr_wave": a, "csr_auto": a,
           "csr_aligned": to_csr_aligned(a) if fmt == "csr_aligned" else None,
           "ell": to_ell(a)[0], "dia": to_dia(a) if fmt == "dia" else None,
           "coo": to_coo(a), "hyb": to_hyb(a)}[fmt].to(gpu)
    kernel = {"csr_scalar": "scalar", "csr_vector": "vector", "csr_stream": "stream", "csr_short": "short",
              "csr_wave": "wave"}.get(fmt, "auto")
    y = spmv(dev, x.to(gpu), kernel=kernel).cpu().numpy()
    np.testing.assert_allclose(y, ref, rtol=1e-4, atol=1e-3)
    # beta accumulate
    y0 = torch.randn(a.nrows, device=gpu)
    y1 = spmv(dev, x.to(gpu), y0.clone(), kernel=kernel, beta=0.5).cpu().numpy()
    np.testing.assert_allclose(y1, ref + 0.5 * y0.cpu().numpy(), rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
def test_spmv_csr_aligned_stream_load_modes_bitwise(gpu):
    """The aligned-CSR stream-load modes (tuning knob spmv_nt: 0 plain, 1
    non-temporal, 2 by matrix size) only change cache hints: bitwise equal."""
    from cme213x.utils import tuning

    a = random_csr(30000, 30000, 16, seed=6)
    dev = to_csr_aligned(a).to(gpu)
    x = torch.randn(a.ncols, device=gpu)
    outs = []
    for mode in (0, 1, 2):
        with tuning.override(spmv_nt=mode):
            outs.append(spmv(dev, x).cpu())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    np.testing.assert_allclose(outs[2].numpy(), _ref(a, x.cpu()), rtol=1e-4, atol=1e-3)


def test_colblocked_format_choice_and_blocks():
    """Column-blocked CSR: block count from the x footprint (2 MB per block),
    block-relative columns, and `auto` choosing it only when x exceeds 2 MB
    (random rows; structured matrices keep DIA / ELL)."""
    from cme213x.ops.spmv import choose_format, to_csr_colblocked

    small = random_csr(300, 4096, 12, seed=4)
    assert choose_format(small) == "csr_aligned"
    big = random_csr(2000, 1 << 20, 12, seed=5)  # x = 4 MB: two 2 MB blocks
    assert choose_format(big) == "csr_cb"
    cb = to_csr_colblocked(big)
    assert cb.col0 == (0, 1 << 19) and all(b.ncols == 1 << 19 for b in cb.blocks)
    for b in cb.blocks:
        assert int(b.col.max()) < b.ncols and int(b.col.min()) >= 0
    # the blocks partition the entries: every (row, global column, value) once (padding has value 0)
    got = sorted((r, c0 + int(c), float(v)) for c0, b in zip(cb.col0, cb.blocks)
                 for r, (s, e) in enumerate(zip(b.rp[:-1].tolist(), b.rp[1:].tolist()))
                 for c, v in zip(b.col[s:e].tolist(), b.val[s:e].tolist()) if v != 0.0)
    rows = np.repeat(np.arange(big.nrows), np.diff(big.rp.numpy()))
    want = sorted(zip(rows.tolist(), big.col.tolist(), big.val.tolist()))
    assert got == want
    assert choose_format(laplacian("5pt", 1100)) == "dia"


def test_colblocked_needs_far_gathers():
    """A large banded matrix that is not DIA-eligible (a random band of +-2000
    columns around the diagonal, 4-20 per row) keeps the single-pass aligned
    CSR: its gathers already stay local, so column blocks would only re-read
    rp and y per block."""
    from cme213x.ops.spmv import CSR, choose_format, matrix_stats

    n = 1 << 20
    rng = np.random.default_rng(6)
    lens = rng.integers(4, 21, n)  # irregular rows (not ELL): 4..20, mean 12
    rows = np.repeat(np.arange(n), lens)
    cols = np.clip(rows + rng.integers(-2000, 2001, rows.size), 0, n - 1)
    order = np.lexsort((cols, rows))
    rp = np.concatenate([[0], np.cumsum(lens)])
    a = CSR(n, n, torch.from_numpy(rp.astype(np.int32)), torch.from_numpy(cols[order].astype(np.int32)),
            torch.ones(rows.size))
    st = matrix_stats(a)
    assert st.far_frac < 0.01 and st.ndiag > 64
    assert choose_format(a, st) == "csr_aligned"
    assert matrix_stats(random_csr(2000, 1 << 20, 12, seed=5)).far_frac > 0.8


@pytest.mark.gpu
@pytest.mark.parametrize("rows_case", ["long_rows", "empty_rows", "tail", "mixed"])
@pytest.mark.parametrize("kernel,rpt", [("stream", 0), ("short", 1), ("short", 2), ("short", 4), ("wave", 0)])
def test_spmv_csr_stream_blocks(gpu, rows_case, kernel, rpt):
    """CSR-stream's row blocks: a block whose nonzeros overflow the 4096-
    product LDS buffer takes the wave-per-row fallback (rows of 3000 and 9000
    entries among short ones), empty rows, a row count that is not a
    multiple of the block, and every block size (64 / 128 / 256 rows by mean
    row length) -- all against the fp64 oracle, with beta. The same matrices
    through CSR-short (rows longer than its 8-entry batch, 1 / 2 / 4 rows per
    lane, a ragged last block)."""
    import contextlib

    from cme213x.ops.spmv import stream_rows
    from cme213x.utils import tuning

    rng = np.random.default_rng(7)
    n = 5003
    if rows_case == "long_rows":
        lens = rng.integers(1, 6, n)
        lens[[17, 300, 301, 4000]] = [3000, 9000, 5000, 4097]
    elif rows_case == "empty_rows":
        lens = rng.integers(0, 3, n)
    elif rows_case == "tail":
        lens = np.full(n, 12)  # mean 12: 256-row blocks, 4-entry pieces all aligned
    else:
        lens = rng.integers(10, 40, n)  # mean ~25: 64-row blocks
    rows = np.repeat(np.arange(n), lens)
    cols = rng.integers(0, 7000, rows.size)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    a = CSR(n, 7000, torch.from_numpy(rp), torch.from_numpy(cols.astype(np.int32)),
            torch.from_numpy(rng.standard_normal(rows.size).astype(np.float32)))
    x = torch.randn(a.ncols)
    ref = _ref(a, x)
    dev = a.to(gpu)
    with tuning.override(spmv_short_rpt=rpt) if rpt else contextlib.nullcontext():
        y = spmv(dev, x.to(gpu), kernel=kernel).cpu().numpy()
        np.testing.assert_allclose(y, ref, rtol=1e-4, atol=1e-3)
        y0 = torch.randn(n, device=gpu)
        y1 = spmv(dev, x.to(gpu), y0.clone(), kernel=kernel, beta=0.5).cpu().numpy()
    np.testing.assert_allclose(y1, ref + 0.5 * y0.cpu().numpy(), rtol=1e-4, atol=1e-3)
    assert stream_rows(a) in (64, 128, 256, 512)


def test_csr_auto_scalar_rule():
    """CSR "auto" takes the lane-per-row kernel for short regular rows only:
    mean <= 8 and no row longer than 16 (one long row would serialise its
    lane); the longest row is cached per row-pointer tensor."""
    from cme213x.ops.spmv import SCALAR_MAX_MEAN, SCALAR_MAX_ROW, max_row_length

    assert (SCALAR_MAX_MEAN, SCALAR_MAX_ROW) == (8, 16)
    a = laplacian("5pt", 50)
    assert max_row_length(a) == 5 and max_row_length(a) == 5
    rp = torch.tensor([0, 2, 40, 41], dtype=torch.int32)
    b = CSR(3, 50, rp, torch.zeros(41, dtype=torch.int32), torch.ones(41))
    assert max_row_length(b) == 38
    rp[1:] = torch.tensor([20, 40, 41], dtype=torch.int32)  # in-place edit: the cached value is dropped
    assert max_row_length(b) == 20


def test_csr_auto_kernel_rule():
    """CSR "auto" takes the stream kernel below a mean of 32 nonzeros per row
    (rows per block from the mean), the vector kernel above."""
    from cme213x.ops.spmv import STREAM_MAX_MEAN, stream_rows

    assert STREAM_MAX_MEAN == 32
    assert stream_rows(laplacian("5pt", 50)) == 512
    assert stream_rows(random_csr(1000, 1000, 8, seed=1)) == 256
    assert stream_rows(random_csr(1000, 1000, 14, seed=1)) == 128
    assert stream_rows(random_csr(1000, 1000, 30, seed=1)) == 64


def test_csr_caches_longest_row_at_build_and_to():
    """a host-built CSR knows its longest row before any capture,
    and .to() carries it to the new row pointers."""
    from cme213x.ops.spmv import _MAX_ROW, laplacian

    a = laplacian("5pt", 30)
    assert id(a.rp) in _MAX_ROW and _MAX_ROW[id(a.rp)][2] == 5
    b = a.to("cpu")
    assert id(b.rp) in _MAX_ROW and _MAX_ROW[id(b.rp)][2] == 5


@pytest.mark.gpu
def test_csr_auto_graph_equals_eager(gpu):
    """The captured graph takes the same "auto" kernel as eager mode (bitwise
    equal outputs); a device-built CSR whose longest row is unknown refuses
    to be captured instead of silently switching kernels."""
    import torch

    from cme213x.ops.spmv import CSR, laplacian, spmv

    a = laplacian("5pt", 300).to(gpu)
    x = torch.rand(a.ncols, device=gpu)
    eager = spmv(a, x)
    y = torch.empty(a.nrows, device=gpu)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        spmv(a, x, y)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(eager, y)
    raw = CSR(a.nrows, a.ncols, a.rp.clone(), a.col, a.val)  # device row pointers, never measured
    g2 = torch.cuda.CUDAGraph()
    with pytest.raises(RuntimeError, match="longest row"):
        with torch.cuda.graph(g2):
            spmv(raw, x, y)
