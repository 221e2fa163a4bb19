"""Distributed matrix-vector products (``slides/Lecture20.pdf``), on RCCL:

* :class:`RowPartitionedSpMV` -- rows (and x) block-partitioned, balanced by
  nonzeros. ``halo`` mode (default) splits each rank's rows into an interior
  block (columns it owns) and a compact boundary block (columns owned by
  others); a product packs the x entries each NEIGHBOUR needs with one HIP
  gather, posts one grouped point-to-point batch to exactly the ranks with
  nonzero counts (native RCCL ``ncclGroupStart/End`` on a side stream, or
  torch.distributed), runs the interior SpMV while the halo is in flight, and
  finishes with the boundary rows. Traffic is O(halo), not O(P * max halo):
  a banded matrix talks to its two neighbours only. ``allgather`` mode is
  the lecture's ``MPI_Allgather`` baseline (RCCL ``all_gather_into_tensor``).
* :func:`colwise_matvec` -- dense column blocks, partial products (framework
  GEMV) combined with a reduce-scatter (``MPI_Reduce`` of the lecture,
  distributed result).
* :func:`block2d_matvec` -- dense sqrt(P) x sqrt(P) blocks on a process grid
  with row/column sub-communicators (``MPI_Cart_create``/``Cart_sub`` ->
  ``Comm.split``): x blocks broadcast down columns, partial y (framework
  GEMV) reduced along rows.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _ext
from ..ops.gemm import gemv
from ..ops.spmv import CSR, prepare, spmv, to_csr_aligned, to_ell
from ..parallel.comm import P2P, Comm, Pending

_ext.proto(_ext.HIP_PROTOS, "cme_gather_f32", "ipppp")
_ext.proto(_ext.HIP_PROTOS, "cme_spmv_halo", "ippppppp")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_gather_f32", "ippp")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_spmv_halo", "ipppppp")


def nnz_balanced_bounds(rp: np.ndarray, P: int) -> np.ndarray:
    """Row boundaries giving each rank ~nnz/P nonzeros."""
    nnz = int(rp[-1])
    targets = np.arange(1, P) * nnz / P
    cuts = np.searchsorted(rp, targets)
    return np.concatenate([[0], cuts, [rp.size - 1]]).astype(np.int64)


def _local_format(a: CSR, fmt: str, device):
    """Local block storage. "auto" is the structure-based choice of
    :func:`~cme213x.ops.spmv.choose_format` (DIA for stencils, ELL for regular
    rows, HYB for power-law rows, else aligned CSR); "ell" / "csr_aligned" /
    "csr" / any :func:`prepare` name force one. The CPU backend takes CSR."""
    if fmt == "csr" or torch.device(device).type != "cuda" or a.nrows == 0:
        return a.to(device)
    if fmt == "ell":
        ell, rest = to_ell(a)
        if rest.nnz == 0:
            return ell.to(device)
        return to_csr_aligned(a).to(device)
    if fmt == "csr_aligned":
        return to_csr_aligned(a).to(device)
    return prepare(a, fmt, device)[1]


def _csr_from(nrows: int, ncols: int, rows: np.ndarray, col: np.ndarray, val: torch.Tensor) -> CSR:
    """CSR from row-sorted (row, col, val) triplets."""
    rp = np.zeros(nrows + 1, dtype=np.int64)
    np.cumsum(np.bincount(rows, minlength=nrows), out=rp[1:])
    return CSR(nrows, ncols, torch.from_numpy(rp.astype(np.int32)), torch.from_numpy(col.astype(np.int32)),
               val.contiguous())


class RowPartitionedSpMV:
    def __init__(self, a: CSR, comm: Comm, device, mode: str = "halo", fmt: str = "auto", rccl=None):
        """``a``: the full matrix (every rank builds the same partition).
        ``fmt``: interior block format (see :func:`_local_format`).
        ``rccl``: a :class:`~cme213x.parallel.rccl.NativeRccl` for the halo
        batch (GPU); default is ``comm.exchange`` (torch.distributed / gloo)."""
        self.comm, self.rccl = comm, rccl
        self.P, self.r = comm.size, comm.rank
        self.n = a.nrows
        self.device = torch.device(device)
        rp = a.rp.cpu().numpy().astype(np.int64)
        # x uses the same row partition (square matrix)
        self.bounds = nnz_balanced_bounds(rp, self.P)
        self.blk = int(np.max(np.diff(self.bounds)))
        lo, hi = int(self.bounds[self.r]), int(self.bounds[self.r + 1])
        self.lo, self.hi = lo, hi
        nloc = hi - lo
        col = a.col.cpu().numpy().astype(np.int64)[rp[lo]:rp[hi]]
        val = a.val.cpu()[rp[lo]:rp[hi]]
        rows = np.repeat(np.arange(nloc, dtype=np.int64), np.diff(rp[lo:hi + 1]))
        self.mode = mode
        owner = np.searchsorted(self.bounds, col, side="right") - 1
        if mode == "allgather":
            # equal-size padded blocks make the all-gather a single RCCL call;
            # global column -> padded position (owner*blk + offset)
            gcol = owner * self.blk + (col - self.bounds[owner])
            self.local = _local_format(_csr_from(nloc, self.P * self.blk, rows, gcol, val), fmt, device)
            self._xpad = torch.zeros(self.blk, dtype=torch.float32, device=device)
        elif mode == "halo":
            self._setup_halo(rows, col, val, owner, nloc, fmt)
        else:
            raise ValueError(mode)

    # ------------------------------------------------------------ set-up
    def _setup_halo(self, rows, col, val, owner, nloc, fmt):
        P, r, dev = self.P, self.r, self.device
        mine = owner == r
        self.interior = _local_format(_csr_from(nloc, nloc, rows[mine], col[mine] - self.lo,
                                                val[torch.from_numpy(mine)]), fmt, dev)
        ext = ~mine
        ucol = np.unique(col[ext])  # sorted, hence grouped by owner in rank order
        uown = np.searchsorted(self.bounds, ucol, side="right") - 1
        need = np.bincount(uown, minlength=P).astype(np.int64)  # entries I receive from each rank
        self.recv_off = np.concatenate([[0], np.cumsum(need)]).astype(np.int64)
        # boundary block: rows with off-rank columns, columns index the halo buffer
        erows, ecol = rows[ext], col[ext]
        hpos = np.searchsorted(ucol, ecol)
        brow, inv = np.unique(erows, return_inverse=True)
        b = _csr_from(brow.size, int(ucol.size), inv.astype(np.int64), hpos, val[torch.from_numpy(ext)])
        self.bnd_rows = torch.from_numpy(brow.astype(np.int32)).to(dev)
        self.bnd = b.to(dev)
        # who needs what from me: counts by one all-gather, then the indices
        # themselves by neighbour-only point-to-point
        counts = torch.from_numpy(need)
        if self._nccl():
            counts = counts.to(dev)
        all_counts = self.comm.allgather(counts).cpu().numpy().reshape(P, P)  # [receiver, owner]
        give = all_counts[:, r].astype(np.int64)  # entries each rank receives from me
        give[r] = 0
        self.send_off = np.concatenate([[0], np.cumsum(give)]).astype(np.int64)
        self.recv_peers = [q for q in range(P) if q != r and need[q] > 0]
        self.send_peers = [q for q in range(P) if q != r and give[q] > 0]
        idx_dev = dev if self._nccl() else torch.device("cpu")
        send_idx = torch.empty(int(self.send_off[-1]), dtype=torch.int64, device=idx_dev)
        req = torch.from_numpy(ucol - self.bounds[uown]).to(idx_dev)  # owner-local indices I need
        ops = [P2P("recv", send_idx[self.send_off[q]:self.send_off[q + 1]], q) for q in self.send_peers]
        ops += [P2P("send", req[self.recv_off[q]:self.recv_off[q + 1]], q) for q in self.recv_peers]
        self.comm.exchange(ops).wait()
        self.send_idx = send_idx.to(torch.int32).to(dev)
        self.sendbuf = torch.empty(int(self.send_off[-1]), dtype=torch.float32, device=dev)
        self.halo = torch.empty(int(self.recv_off[-1]), dtype=torch.float32, device=dev)
        self._ops = [P2P("recv", self.halo[self.recv_off[q]:self.recv_off[q + 1]], q) for q in self.recv_peers]
        self._ops += [P2P("send", self.sendbuf[self.send_off[q]:self.send_off[q + 1]], q) for q in self.send_peers]
        if self.rccl is not None:
            self._cstream = torch.cuda.Stream(dev)
            self._ev_packed, self._ev_recv = torch.cuda.Event(), torch.cuda.Event()

    def _nccl(self) -> bool:
        return getattr(self.comm, "backend", None) == "nccl"

    @property
    def halo_volume(self) -> tuple[int, int, int]:
        """(values sent, values received, peers talked to) per product."""
        if self.mode != "halo":
            return (self.hi - self.lo, self.P * self.blk, self.P - 1)
        return (int(self.send_off[-1]), int(self.recv_off[-1]), len(set(self.recv_peers) | set(self.send_peers)))

    def local_slice(self, x_full: torch.Tensor) -> torch.Tensor:
        return x_full[self.lo:self.hi]

    # ------------------------------------------------------------ product
    def _post_halo(self, x_local: torch.Tensor) -> Pending | None:
        """Pack what the neighbours need and post the grouped exchange."""
        if x_local.is_cuda:
            s = _ext.stream_ptr(x_local.device)
            _ext.call_hip("cme_gather_f32", self.send_idx.numel(), x_local.data_ptr(), self.send_idx.data_ptr(),
                          self.sendbuf.data_ptr(), s)
        else:
            _ext.call_cpu("cme_cpu_gather_f32", self.send_idx.numel(), x_local.data_ptr(), self.send_idx.data_ptr(),
                          self.sendbuf.data_ptr())
        if not self._ops:
            return None
        if self.rccl is not None:
            # RCCL batch on a side stream, ordered after the pack; the compute
            # stream runs the interior product meanwhile
            cur = torch.cuda.current_stream(self.device)
            self._ev_packed.record(cur)
            self._cstream.wait_event(self._ev_packed)
            self.rccl.p2p([(o.kind, o.tensor, o.peer) for o in self._ops], stream=self._cstream)
            self._ev_recv.record(self._cstream)
            return None
        return self.comm.exchange(self._ops)

    def __call__(self, x_local: torch.Tensor, y: torch.Tensor | None = None) -> torch.Tensor:
        """y_local = (A x)[lo:hi] given this rank's slice of x."""
        x_local = x_local.contiguous()
        if x_local.dtype != torch.float32 or x_local.numel() != self.hi - self.lo:
            raise ValueError("x_local must be this rank's fp32 slice")
        if self.mode == "allgather":
            self._xpad[:x_local.numel()].copy_(x_local)
            xg = self.comm.allgather(self._xpad).reshape(-1)
            return spmv(self.local, xg, y)
        if y is None:
            y = torch.empty(self.hi - self.lo, dtype=torch.float32, device=x_local.device)
        pending = self._post_halo(x_local)
        spmv(self.interior, x_local, y)  # overlaps the halo traffic
        if pending is not None:
            pending.wait()
        elif self.rccl is not None and self._ops:
            torch.cuda.current_stream(self.device).wait_event(self._ev_recv)
        b = self.bnd
        if y.is_cuda:
            _ext.call_hip("cme_spmv_halo", b.nrows, self.bnd_rows.data_ptr(), b.rp.data_ptr(), b.col.data_ptr(),
                          b.val.data_ptr(), self.halo.data_ptr(), y.data_ptr(), _ext.stream_ptr(y.device))
        elif b.nrows:
            _ext.call_cpu("cme_cpu_spmv_halo", b.nrows, self.bnd_rows.data_ptr(), b.rp.data_ptr(), b.col.data_ptr(),
                          b.val.data_ptr(), self.halo.data_ptr(), y.data_ptr())
        return y


def colwise_matvec(comm: Comm, A_cols: torch.Tensor, x_local: torch.Tensor) -> torch.Tensor:
    """A_cols: this rank's column block (n x n/P) of a dense A; returns this
    rank's n/P slice of y via reduce-scatter."""
    partial = gemv(A_cols, x_local)
    return comm.reduce_scatter(partial)


def block2d_matvec(comm: Comm, A_blk: torch.Tensor, x_blk_diag: torch.Tensor | None) -> torch.Tensor:
    """2-D block matvec on a q x q grid (P = q^2, rank = row*q + col).
    A_blk: block (row, col); x_blk_diag: x block `row`, held by the diagonal
    rank (row == col), None elsewhere. Returns y block `row` on the diagonal
    rank (None elsewhere)."""
    P = comm.size
    q = int(round(P ** 0.5))
    if q * q != P:
        raise ValueError("2-D matvec needs a square process count")
    row, col = divmod(comm.rank, q)
    col_comm = comm.split(color=col, key=row)  # ranks sharing a column
    row_comm = comm.split(color=row, key=col)  # ranks sharing a row
    nb = A_blk.shape[1]
    xb = x_blk_diag if x_blk_diag is not None else torch.empty(nb, dtype=A_blk.dtype, device=A_blk.device)
    # the diagonal rank of column `col` is (row=col): its rank in col_comm is `col`
    col_comm.broadcast_(xb, src=col)
    partial = gemv(A_blk, xb)
    # reduce along the row to the diagonal rank (its rank in row_comm is `row`)
    row_comm.reduce_(partial, dst=row)
    return partial if row == col else None
