"""Sparse matrices and SpMV in the Bell & Garland formats (CSR-scalar,
CSR-vector, ELL, DIA, COO, HYB), plus the structured-Laplacian generators
(3/5/7/9/27-point) used in their evaluation (``refs/Bell SC 2009.pdf`` §4.2;
``slides/Lecture22.pdf``).

Conversions run once on the host (numpy, vectorised); the matrices then live
on the device and every multiply is one HIP kernel (two for HYB).
"""
from __future__ import annotations

import weakref
from dataclasses import dataclass

import numpy as np

import torch

from .. import _ext

_ext.proto(_ext.HIP_PROTOS, "cme_spmv_csr", "ipppppifp")
_ext.proto(_ext.HIP_PROTOS, "cme_spmv_ell", "iippppfp")
_ext.proto(_ext.HIP_PROTOS, "cme_spmv_dia", "iiippppfp")
_ext.proto(_ext.HIP_PROTOS, "cme_spmv_coo", "iqpppppfip")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_spmv_csr", "ipppppf")
_ext.proto(_ext.HIP_PROTOS, "cme_spmv_csr_aligned", "iqpppppifp")
_ext.proto(_ext.HIP_PROTOS, "cme_spmv_csr_stream", "ipppppifp")
_ext.proto(_ext.HIP_PROTOS, "cme_spmv_csr_short", "ipppppifp")
_ext.proto(_ext.HIP_PROTOS, "cme_spmv_csr_wave", "ipppppfp")


# ---------------------------------------------------------------- formats
@dataclass
class CSR:
    nrows: int
    ncols: int
    rp: torch.Tensor  # int32 [nrows+1]
    col: torch.Tensor  # int32 [nnz]
    val: torch.Tensor  # float32 [nnz]

    @property
    def nnz(self) -> int:
        return self.col.numel()

    def __post_init__(self):
        # host row pointers: cache the longest row now (spmv "auto" reads it,
        # and a stream capture cannot compute it)
        if not self.rp.is_cuda:
            max_row_length(self)

    def to(self, device) -> "CSR":
        out = CSR(self.nrows, self.ncols, self.rp.to(device), self.col.to(device), self.val.to(device))
        _carry_max_row(self, out)
        return out

    def to_dense(self) -> torch.Tensor:
        rows = torch.repeat_interleave(torch.arange(self.nrows), torch.diff(self.rp.cpu().long()))
        d = torch.zeros(self.nrows, self.ncols)
        d.index_put_((rows, self.col.cpu().long()), self.val.cpu(), accumulate=True)
        return d


@dataclass
class CSRAligned(CSR):
    """CSR whose rows are zero-padded to multiples of 4 nonzeros, so every row
    starts on a 16-B boundary (Baskaran & Bordawekar's alignment + padding,
    ``refs/Baskaran IBM 2009.pdf`` pp.4-8). Padding entries have value 0 and
    repeat the row's last column index (finite ``x`` assumed)."""

    def to(self, device) -> "CSRAligned":
        return CSRAligned(self.nrows, self.ncols, self.rp.to(device), self.col.to(device), self.val.to(device))


def to_csr_aligned(a: CSR) -> CSRAligned:
    rp = a.rp.cpu().long()
    lens = torch.diff(rp)
    plens = (lens + 3) // 4 * 4
    prp = torch.zeros(a.nrows + 1, dtype=torch.long)
    prp[1:] = torch.cumsum(plens, 0)
    nnz = int(prp[-1])
    col = torch.zeros(nnz, dtype=torch.int32)
    val = torch.zeros(nnz, dtype=torch.float32)
    rows = torch.repeat_interleave(torch.arange(a.nrows), lens)
    pos = prp[:-1][rows] + (torch.arange(a.nnz) - rp[:-1][rows])
    col[pos] = a.col.cpu()
    val[pos] = a.val.cpu()
    # padding repeats the last real column (or 0 for empty rows)
    pad_rows = torch.repeat_interleave(torch.arange(a.nrows), plens - lens)
    if pad_rows.numel():
        offs = torch.arange(pad_rows.numel()) - torch.repeat_interleave(
            torch.cumsum(plens - lens, 0) - (plens - lens), plens - lens)
        ppos = prp[:-1][pad_rows] + lens[pad_rows] + offs
        last = torch.where(lens[pad_rows] > 0, a.col.cpu().long()[(rp[1:][pad_rows] - 1).clamp(min=0)],
                           torch.zeros_like(pad_rows))
        col[ppos] = last.to(torch.int32)
    dev = a.rp.device
    return CSRAligned(a.nrows, a.ncols, prp.to(torch.int32).to(dev), col.to(dev), val.to(dev))


@dataclass
class CSRColBlocked:
    """Aligned CSR split into column blocks, multiplied block after block
    (y = A_0 x_0, then y += A_k x_k). Each block's slice of ``x`` is small
    enough (<= ``block_bytes``, half of one XCD's 4 MB L2) to stay L2-resident
    while the block's column / value stream passes through non-temporally, so
    the random gathers hit L2 instead of the Infinity Cache (the x-caching
    idea of ``refs/Baskaran IBM 2009.pdf`` pp.4-8, by column range). The
    row sums are taken per block, then added: the same value up to fp32
    reassociation (within the tolerance of the reference's checks)."""
    nrows: int
    ncols: int
    col0: tuple  # first column of each block
    blocks: tuple  # CSRAligned per block, column indices relative to col0

    @property
    def nnz(self) -> int:
        return sum(b.nnz for b in self.blocks)

    def to(self, device) -> "CSRColBlocked":
        return CSRColBlocked(self.nrows, self.ncols, self.col0, tuple(b.to(device) for b in self.blocks))


def to_csr_colblocked(a: CSR, block_bytes: int = 2 << 20, aligned: bool = True) -> CSRColBlocked:
    """Split ``a`` into ceil(4 * ncols / block_bytes) column blocks of equal
    width (column indices made block-relative), each an aligned CSR (rows
    padded to multiples of 4 entries) or, ``aligned=False``, a plain CSR
    (no padding; CSR-vector kernel)."""
    nb = max(1, -(-4 * a.ncols // block_bytes))
    width = -(-a.ncols // nb)
    rp = a.rp.cpu().long()
    col = a.col.cpu().long()
    val = a.val.cpu()
    rows = torch.repeat_interleave(torch.arange(a.nrows), torch.diff(rp))
    blk = col // width
    blocks, col0 = [], []
    for k in range(nb):
        sel = blk == k
        r, c, v = rows[sel], col[sel] - k * width, val[sel]
        brp = torch.zeros(a.nrows + 1, dtype=torch.long)
        brp[1:] = torch.cumsum(torch.bincount(r, minlength=a.nrows), 0)
        sub = CSR(a.nrows, min(width, a.ncols - k * width), brp.to(torch.int32), c.to(torch.int32), v)
        blocks.append((to_csr_aligned(sub) if aligned else sub).to(a.rp.device))
        col0.append(k * width)
    return CSRColBlocked(a.nrows, a.ncols, tuple(col0), tuple(blocks))


@dataclass
class ELL:
    nrows: int
    ncols: int
    K: int
    col: torch.Tensor  # int32 [K*nrows], column-major, -1 = padding
    val: torch.Tensor  # float32 [K*nrows]

    def to(self, device) -> "ELL":
        return ELL(self.nrows, self.ncols, self.K, self.col.to(device), self.val.to(device))


@dataclass
class DIA:
    nrows: int
    ncols: int
    offsets: torch.Tensor  # int32 [ndiag]
    data: torch.Tensor  # float32 [ndiag*nrows], data[d*nrows + r] = A[r, r+off[d]]

    def to(self, device) -> "DIA":
        return DIA(self.nrows, self.ncols, self.offsets.to(device), self.data.to(device))


@dataclass
class COO:
    nrows: int
    ncols: int
    row: torch.Tensor  # int32 [nnz], sorted
    col: torch.Tensor
    val: torch.Tensor

    @property
    def nnz(self) -> int:
        return self.row.numel()

    def to(self, device) -> "COO":
        return COO(self.nrows, self.ncols, self.row.to(device), self.col.to(device), self.val.to(device))


@dataclass
class HYB:
    ell: ELL
    coo: COO

    def to(self, device) -> "HYB":
        return HYB(self.ell.to(device), self.coo.to(device))


def csr_from_coo_arrays(nrows: int, ncols: int, r: np.ndarray, c: np.ndarray, v: np.ndarray) -> CSR:
    order = np.lexsort((c, r))
    r, c, v = r[order], c[order], v[order]
    rp = np.zeros(nrows + 1, dtype=np.int64)
    np.add.at(rp, r + 1, 1)
    rp = np.cumsum(rp)
    return CSR(nrows, ncols, torch.from_numpy(rp.astype(np.int32)), torch.from_numpy(c.astype(np.int32)),
               torch.from_numpy(v.astype(np.float32)))


def _row_ids(a: CSR) -> np.ndarray:
    return np.repeat(np.arange(a.nrows, dtype=np.int64), np.diff(a.rp.cpu().numpy().astype(np.int64)))


def to_coo(a: CSR) -> COO:
    return COO(a.nrows, a.ncols, torch.from_numpy(_row_ids(a).astype(np.int32)), a.col.cpu().clone(),
               a.val.cpu().clone())


def to_ell(a: CSR, K: int | None = None, max_entries: int = 1 << 27) -> tuple[ELL, COO]:
    """ELL with K columns (default: max row length); entries beyond K go to
    the returned COO remainder (empty when K >= max row length)."""
    rp = a.rp.cpu().numpy().astype(np.int64)
    lens = np.diff(rp)
    K = int(lens.max()) if K is None else int(K)
    if K * a.nrows > max_entries:
        raise ValueError(f"ELL width {K} x {a.nrows} rows exceeds {max_entries} entries: use HYB")
    rows = _row_ids(a)
    pos = np.arange(a.nnz, dtype=np.int64) - rp[rows]
    col = a.col.cpu().numpy()
    val = a.val.cpu().numpy()
    keep = pos < K
    ecol = np.full(K * a.nrows, -1, dtype=np.int32)
    eval_ = np.zeros(K * a.nrows, dtype=np.float32)
    idx = pos[keep] * a.nrows + rows[keep]
    ecol[idx] = col[keep]
    eval_[idx] = val[keep]
    rest = ~keep
    coo = COO(a.nrows, a.ncols, torch.from_numpy(rows[rest].astype(np.int32)),
              torch.from_numpy(col[rest].copy()), torch.from_numpy(val[rest].copy()))
    return ELL(a.nrows, a.ncols, K, torch.from_numpy(ecol), torch.from_numpy(eval_)), coo


def hyb_k(a: CSR) -> int:
    """Bell & Garland's ELL width: the largest K such that at least
    max(4096, nrows/3) rows have >= K nonzeros."""
    lens = np.diff(a.rp.cpu().numpy().astype(np.int64))
    need = max(4096, a.nrows // 3)
    hist = np.bincount(lens)
    rows_ge = np.cumsum(hist[::-1])[::-1]  # rows_ge[k] = #rows with len >= k
    ks = np.nonzero(rows_ge >= need)[0]
    return int(ks.max()) if ks.size else 0


def to_hyb(a: CSR, K: int | None = None) -> HYB:
    ell, coo = to_ell(a, hyb_k(a) if K is None else K)
    return HYB(ell, coo)


def to_dia(a: CSR, max_diags: int = 1024) -> DIA:
    rows = _row_ids(a)
    col = a.col.cpu().numpy().astype(np.int64)
    off = col - rows
    offs = np.unique(off)
    if offs.size > max_diags:
        raise ValueError(f"{offs.size} diagonals: DIA is not suitable for this matrix")
    d_index = np.searchsorted(offs, off)
    data = np.zeros(offs.size * a.nrows, dtype=np.float32)
    np.add.at(data, d_index * a.nrows + rows, a.val.cpu().numpy())
    return DIA(a.nrows, a.ncols, torch.from_numpy(offs.astype(np.int32)), torch.from_numpy(data))


# ---------------------------------------------------------------- generators
def laplacian(kind: str, n: int) -> CSR:
    """Structured Laplacians on an n (1-D), n x n (2-D) or n^3 (3-D) grid:
    "3pt", "5pt", "7pt", "9pt", "27pt" (Bell & Garland Table 2 family).
    Diagonal = number of neighbours, off-diagonals -1."""
    if kind == "3pt":
        dims, stencil = (n,), [(-1,), (0,), (1,)]
    elif kind == "5pt":
        dims, stencil = (n, n), [(0, 0), (-1, 0), (1, 0), (0, -1), (0, 1)]
    elif kind == "9pt":
        dims, stencil = (n, n), [(i, j) for i in (-1, 0, 1) for j in (-1, 0, 1)]
    elif kind == "7pt":
        dims = (n, n, n)
        stencil = [(0, 0, 0), (-1, 0, 0), (1, 0, 0), (0, -1, 0), (0, 1, 0), (0, 0, -1), (0, 0, 1)]
    elif kind == "27pt":
        dims = (n, n, n)
        stencil = [(i, j, k) for i in (-1, 0, 1) for j in (-1, 0, 1) for k in (-1, 0, 1)]
    else:
        raise ValueError(kind)
    N = int(np.prod(dims))
    coords = np.stack(np.unravel_index(np.arange(N, dtype=np.int64), dims), axis=1)
    rs, cs, vs = [], [], []
    ncount = len(stencil) - 1
    for off in stencil:
        nb = coords + np.asarray(off)
        ok = np.all((nb >= 0) & (nb < np.asarray(dims)), axis=1)
        r = np.nonzero(ok)[0]
        c = np.ravel_multi_index(tuple(nb[ok].T), dims)
        rs.append(r)
        cs.append(c)
        vs.append(np.full(r.size, float(ncount) if not any(off) else -1.0, dtype=np.float32))
    return csr_from_coo_arrays(N, N, np.concatenate(rs), np.concatenate(cs), np.concatenate(vs))


def random_csr(nrows: int, ncols: int, avg_nnz: float, seed: int = 0, skew: bool = False) -> CSR:
    """Random sparse matrix; ``skew`` draws power-law row lengths (the
    unstructured corpus' load-imbalance case)."""
    rng = np.random.default_rng(seed)
    if skew:
        lens = np.minimum((rng.pareto(1.5, nrows) + 1) * avg_nnz / 3, ncols).astype(np.int64)
    else:
        lens = rng.poisson(avg_nnz, nrows).astype(np.int64)
    lens = np.maximum(lens, 1)
    r = np.repeat(np.arange(nrows), lens)
    c = rng.integers(0, ncols, r.size)
    v = rng.uniform(-1, 1, r.size).astype(np.float32)
    return csr_from_coo_arrays(nrows, ncols, r, c, v)


# ---------------------------------------------------------------- multiply
def auto_group(a: CSR) -> int:
    """Lanes per row for CSR-vector: next power of two >= mean row length,
    clamped to [2, 64]."""
    mean = a.nnz / max(1, a.nrows)
    g = 2
    while g < mean and g < 64:
        g *= 2
    return g


def stream_rows(a: CSR) -> int:
    """Rows per workgroup of the CSR-stream kernel: 512 / 256 / 128 / 64 for a
    mean row length up to 6 / 12 / 24 / beyond, so a block's nonzeros (R x
    mean) stay inside its 4096-product LDS buffer (a heavier block still
    runs, on the kernel's wave-per-row fallback) while each block carries
    enough entries to amortise its dependent rp -> col/val -> x round trips."""
    from ..utils import tuning

    forced = tuning.get("spmv_stream_rows") if a.rp.is_cuda else 0
    if forced in (64, 128, 256, 512, 1024):
        return forced
    mean = a.nnz / max(1, a.nrows)
    return 512 if mean <= 6 else (256 if mean <= 12 else (128 if mean <= 24 else 64))


# CSR "auto" on short, regular rows (mean <= 8, longest <= 16 entries: the
# 5-point Laplacian of config #4) takes csr_scalar: 13.5 / 11.4 us cold / warm
# on the 1M matrix against 14.9 / 12.2 for CSR-stream; its lane-per-row loop
# would serialise a long row, hence the bound on the longest
# (profiles/spmv_stream_r5.md)
SCALAR_MAX_MEAN, SCALAR_MAX_ROW = 8, 16
# row-pointer tensor (by identity) -> (weak reference, version, longest row):
# one device sync per matrix, then cached; an in-place write to the row
# pointers bumps the tensor's version and invalidates the entry
_MAX_ROW: dict = {}


def _cache_max_row(rp: torch.Tensor, v: int) -> None:
    key = id(rp)
    _MAX_ROW[key] = (weakref.ref(rp, lambda _r, k=key: _MAX_ROW.pop(k, None)), rp._version, v)


def _carry_max_row(src: CSR, dst: CSR) -> None:
    """dst holds src's rows on another device: the cached longest row moves
    with them (computed on the source if need be)."""
    v = max_row_length(src)
    if v is not None:
        _cache_max_row(dst.rp, v)


def max_row_length(a: CSR) -> int | None:
    """Longest row of ``a`` (cached per row-pointer tensor: a CSR built on the
    host caches it at construction and carries it through ``.to()``; None
    only for device row pointers first seen during a stream capture)."""
    hit = _MAX_ROW.get(id(a.rp))
    if hit is not None and hit[0]() is a.rp and hit[1] == a.rp._version:
        return hit[2]
    if a.rp.is_cuda and torch.cuda.is_current_stream_capturing():
        return None
    v = int(torch.diff(a.rp).max().item()) if a.nrows > 0 else 0
    _cache_max_row(a.rp, v)
    return v


# mean row length below which CSR "auto" takes the stream kernel (measured,
# cold / MALL defeated, profiles/spmv_stream_r5.md: 27-pt Laplacian, 26.5 per
# row, stream 1005 vs vector 415 GFLOP/s; random 16 per row 299 vs 248; skewed
# 20 per row 38 vs 15; 5-pt 678 vs 302)
STREAM_MAX_MEAN = 32


def short_rows_per_lane(a: CSR) -> int:
    """Rows per lane of the CSR-short kernel (tuning knob spmv_short_rpt)."""
    from ..utils import tuning

    r = tuning.get("spmv_short_rpt") if a.rp.is_cuda else 1
    return r if r in (1, 2, 4) else 1


def _auto_max_row(a: CSR) -> int:
    """The longest row for the CSR "auto" choice; refuses (instead of
    silently choosing another kernel than eager mode would) when a capture
    meets device row pointers whose longest row was never computed."""
    v = max_row_length(a)
    if v is None:
        raise RuntimeError("spmv(kernel='auto') under stream capture: the longest row of this CSR is unknown -- "
                           "build it on the host and move it with .to(), or call spmv once before capturing")
    return v


def spmv(a, x: torch.Tensor, y: torch.Tensor | None = None, kernel: str = "auto", beta: float = 0.0) -> torch.Tensor:
    """y = A x + beta*y for any of the formats. ``kernel`` (CSR only):
    "scalar", "vector", "stream" (CSR-stream: row blocks staged through LDS),
    "short" (a lane per row, the first 8 entries of a row as one batch of loads),
    or "auto" (scalar for short regular rows -- mean <= 8, longest <= 16 --,
    stream for a mean row length below 32, where CSR-vector idles most of its
    lanes; vector with auto group above). To pick the FORMAT by
    the matrix structure, convert once with :func:`prepare`."""
    if y is None:
        nrows = a.ell.nrows if isinstance(a, HYB) else a.nrows
        y = torch.zeros(nrows, dtype=torch.float32, device=x.device)
    if not x.is_cuda:
        if not isinstance(a, CSR):
            raise TypeError("CPU path supports CSR only")
        _ext.call_cpu("cme_cpu_spmv_csr", a.nrows, a.rp.data_ptr(), a.col.data_ptr(), a.val.data_ptr(),
                      x.data_ptr(), y.data_ptr(), float(beta))
        return y
    s = _ext.stream_ptr(x.device)
    if isinstance(a, CSRColBlocked):
        for k, (c0, b) in enumerate(zip(a.col0, a.blocks)):
            spmv(b, x[c0:c0 + b.ncols], y, kernel=kernel, beta=beta if k == 0 else 1.0)
        return y
    if isinstance(a, CSRAligned):
        g = max(1, auto_group(a) // 4) if kernel != "scalar" else 1
        _ext.call_hip("cme_spmv_csr_aligned", a.nrows, a.nnz, a.rp.data_ptr(), a.col.data_ptr(), a.val.data_ptr(),
                      x.data_ptr(), y.data_ptr(), g, float(beta), s)
    elif isinstance(a, CSR) and kernel == "auto" and a.nnz <= SCALAR_MAX_MEAN * max(1, a.nrows) and \
            _auto_max_row(a) <= SCALAR_MAX_ROW:
        _ext.call_hip("cme_spmv_csr", a.nrows, a.rp.data_ptr(), a.col.data_ptr(), a.val.data_ptr(), x.data_ptr(),
                      y.data_ptr(), 1, float(beta), s)
    elif isinstance(a, CSR) and kernel == "wave":
        _ext.call_hip("cme_spmv_csr_wave", a.nrows, a.rp.data_ptr(), a.col.data_ptr(), a.val.data_ptr(),
                      x.data_ptr(), y.data_ptr(), float(beta), s)
    elif isinstance(a, CSR) and kernel == "short":
        _ext.call_hip("cme_spmv_csr_short", a.nrows, a.rp.data_ptr(), a.col.data_ptr(), a.val.data_ptr(),
                      x.data_ptr(), y.data_ptr(), short_rows_per_lane(a), float(beta), s)
    elif isinstance(a, CSR) and (kernel == "stream" or
                                 (kernel == "auto" and a.nnz < STREAM_MAX_MEAN * max(1, a.nrows))):
        _ext.call_hip("cme_spmv_csr_stream", a.nrows, a.rp.data_ptr(), a.col.data_ptr(), a.val.data_ptr(),
                      x.data_ptr(), y.data_ptr(), stream_rows(a), float(beta), s)
    elif isinstance(a, CSR):
        g = 1 if kernel == "scalar" else auto_group(a)
        _ext.call_hip("cme_spmv_csr", a.nrows, a.rp.data_ptr(), a.col.data_ptr(), a.val.data_ptr(), x.data_ptr(),
                      y.data_ptr(), g, float(beta), s)
    elif isinstance(a, ELL):
        _ext.call_hip("cme_spmv_ell", a.nrows, a.K, a.col.data_ptr(), a.val.data_ptr(), x.data_ptr(), y.data_ptr(),
                      float(beta), s)
    elif isinstance(a, DIA):
        _ext.call_hip("cme_spmv_dia", a.nrows, a.ncols, a.offsets.numel(), a.offsets.data_ptr(), a.data.data_ptr(),
                      x.data_ptr(), y.data_ptr(), float(beta), s)
    elif isinstance(a, COO):
        _ext.call_hip("cme_spmv_coo", a.nrows, a.nnz, a.row.data_ptr(), a.col.data_ptr(), a.val.data_ptr(),
                      x.data_ptr(), y.data_ptr(), float(beta), 0, s)
    elif isinstance(a, HYB):
        spmv(a.ell, x, y, beta=beta)
        if a.coo.nnz:
            _ext.call_hip("cme_spmv_coo", a.coo.nrows, a.coo.nnz, a.coo.row.data_ptr(), a.coo.col.data_ptr(),
                          a.coo.val.data_ptr(), x.data_ptr(), y.data_ptr(), 1.0, 1, s)
    else:
        raise TypeError(type(a))
    return y


# ------------------------------------------------------- format selection
@dataclass
class MatrixStats:
    nrows: int
    nnz: int
    mean_row: float
    max_row: int
    cv_row: float  # coefficient of variation of the row lengths
    ndiag: int  # occupied diagonals
    dia_fill: float  # nnz / (ndiag * nrows)
    ell_fill: float  # nnz / (max_row * nrows)
    far_frac: float = 1.0  # nonzeros more than _CB_NEAR columns off their row's (scaled) diagonal


def matrix_stats(a: CSR) -> MatrixStats:
    lens = np.diff(a.rp.cpu().numpy().astype(np.int64))
    mean = a.nnz / max(1, a.nrows)
    mx = int(lens.max()) if lens.size else 0
    cv = float(lens.std() / mean) if mean > 0 else 0.0
    # occupied diagonals, counted on a sample of rows when the matrix is large
    rows = _row_ids(a)
    off = a.col.cpu().numpy().astype(np.int64) - rows
    if off.size > (1 << 24):
        off = off[np.random.default_rng(0).integers(0, off.size, 1 << 22)]
    ndiag = int(np.unique(off).size)
    # gather locality: how far a row's columns sit from its own position
    # (scaled to the column range for rectangular matrices)
    cols = a.col.cpu().numpy().astype(np.int64)
    rows_s = rows * (a.ncols / max(1, a.nrows))
    if cols.size > (1 << 24):
        pick = np.random.default_rng(1).integers(0, cols.size, 1 << 22)
        cols, rows_s = cols[pick], rows_s[pick]
    far = float(np.mean(np.abs(cols - rows_s) > _CB_NEAR)) if cols.size else 0.0
    return MatrixStats(a.nrows, a.nnz, mean, mx, cv, ndiag, a.nnz / max(1, ndiag * a.nrows),
                       a.nnz / max(1, mx * a.nrows), far)


def choose_format(a: CSR, stats: MatrixStats | None = None) -> str:
    """Bell & Garland's decision rules (``refs/Bell SC 2009.pdf`` §3-4),
    with thresholds set from the MI355X per-format table (profiles/spmv_r2.md):
      * DIA  -- few diagonals, densely filled (structured stencils);
      * ELL  -- regular rows (max row length close to the mean);
      * HYB  -- ELL for the typical rows + COO for a heavy tail (power-law
                rows would serialise CSR lanes on the longest row);
      * CSR-vector (16-B aligned rows) -- everything else, in column blocks of
        2 MB of x when x is larger and most gathers land far from the
        diagonal (one XCD's L2 keeps the block's x slice: random 1M x 1M,
        16/row: 0.0957 vs 0.1038 ms cold, profiles/spmv_cb_r3.jsonl)."""
    st = stats or matrix_stats(a)
    if st.ndiag <= 64 and st.dia_fill >= 0.6:
        return "dia"
    if st.max_row <= 64 and st.ell_fill >= 0.66:
        return "ell"
    if st.max_row > 8 * max(1.0, st.mean_row) or st.cv_row > 1.0:
        return "hyb"
    # column blocks pay only when x outgrows one L2 slice AND the gathers
    # actually roam over it; banded / reordered matrices (most nonzeros near
    # the diagonal) keep their x reuse in one pass of the aligned CSR, which
    # re-reads rp and y once instead of once per block
    if 4 * a.ncols > (2 << 20) and st.far_frac > 0.5:
        return "csr_cb"
    return "csr_aligned"


# |col - row| beyond this (in columns: 256 KB of fp32 x, an eighth of a
# column block) counts as a far gather
_CB_NEAR = 1 << 16


def prepare(a: CSR, fmt: str = "auto", device=None):
    """Convert ``a`` to ``fmt`` ("auto" = :func:`choose_format`) on ``device``;
    returns (format name, matrix) ready for :func:`spmv`."""
    if fmt == "auto":
        fmt = choose_format(a)
    if fmt.startswith("csr_cb_"):  # csr_cb_<KiB of x per block>[_u]: sweep arms of the column-blocked CSR
        parts = fmt.split("_")[2:]
        m = to_csr_colblocked(a, int(parts[0]) << 10, aligned=not (len(parts) > 1 and parts[1] == "u"))
        return fmt, (m.to(device) if device is not None else m)
    conv = {"csr": lambda m: m, "csr_scalar": lambda m: m, "csr_vector": lambda m: m, "csr_stream": lambda m: m,
            "csr_short": lambda m: m, "csr_wave": lambda m: m,
            "csr_aligned": to_csr_aligned,
            "csr_cb": to_csr_colblocked,
            "coo": to_coo, "hyb": to_hyb, "dia": to_dia, "ell": lambda m: to_ell(m)[0]}
    if fmt not in conv:
        raise ValueError(f"unknown SpMV format {fmt!r}")
    m = conv[fmt](a)
    return fmt, (m.to(device) if device is not None else m)


def bytes_per_nnz(fmt: str) -> float:
    """Bell & Garland's fp32 byte model per nonzero (their Table: DIA 4,
    ELL 6... here value + index bytes): for GFLOP/s -> GB/s conversions."""
    return {"dia": 4, "ell": 8, "csr": 8, "coo": 12, "hyb": 8, "csr_cb": 8}[fmt]
