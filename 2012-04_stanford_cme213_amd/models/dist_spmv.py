"""Distributed matrix-vector products (``slides/Lecture20.pdf``), on RCCL:

* :class:`RowPartitionedSpMV` -- rows (and x) block-partitioned, balanced by
  nonzeros; each product all-gathers x (``MPI_Allgather`` -> RCCL
  ``all_gather_into_tensor``) then runs the local HIP SpMV. A ``halo`` mode
  gathers only the x entries the local rows reference (one all-to-all of
  index-selected values), which is what scales on xGMI links.
* :func:`colwise_matvec` -- dense column blocks, partial products combined
  with a reduce-scatter (``MPI_Reduce`` of the lecture, distributed result).
* :func:`block2d_matvec` -- dense sqrt(P) x sqrt(P) blocks on a process grid
  with row/column sub-communicators (``MPI_Cart_create``/``Cart_sub`` ->
  ``Comm.split``): x blocks broadcast down columns, partial y reduced along
  rows.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops.spmv import CSR, spmv, to_csr_aligned, to_ell
from ..parallel.comm import Comm


def nnz_balanced_bounds(rp: np.ndarray, P: int) -> np.ndarray:
    """Row boundaries giving each rank ~nnz/P nonzeros."""
    nnz = int(rp[-1])
    targets = np.arange(1, P) * nnz / P
    cuts = np.searchsorted(rp, targets)
    return np.concatenate([[0], cuts, [rp.size - 1]]).astype(np.int64)


def _local_format(a: CSR, fmt: str, device):
    """Local block storage on the GPU: ELL when rows are short (coalesced, no
    row pointers), else zero-padded aligned CSR (16-B vector loads). The CPU
    backend takes CSR."""
    if fmt == "csr" or torch.device(device).type != "cuda":
        return a
    lens = torch.diff(a.rp.cpu().long())
    if fmt == "ell" or (fmt == "auto" and a.nrows and int(lens.max()) <= 32):
        ell, rest = to_ell(a)
        if rest.nnz == 0:
            return ell
    return to_csr_aligned(a)


class RowPartitionedSpMV:
    def __init__(self, a: CSR, comm: Comm, device, mode: str = "allgather", fmt: str = "auto"):
        """``a``: the full matrix (every rank builds the same partition).
        ``fmt``: local block format -- "auto" (ELL for short rows, else
        aligned CSR), "ell", "csr_aligned" or "csr"."""
        self.comm = comm
        self.P, self.r = comm.size, comm.rank
        self.n = a.nrows
        rp = a.rp.cpu().numpy().astype(np.int64)
        # x uses the same row partition (square matrix); equal-size padded
        # blocks make the all-gather a single RCCL call
        self.bounds = nnz_balanced_bounds(rp, self.P)
        self.blk = int(np.max(np.diff(self.bounds)))
        lo, hi = int(self.bounds[self.r]), int(self.bounds[self.r + 1])
        self.lo, self.hi = lo, hi
        col = a.col.cpu().numpy().astype(np.int64)[rp[lo]:rp[hi]]
        val = a.val.cpu()[rp[lo]:rp[hi]]
        lrp = torch.from_numpy((rp[lo:hi + 1] - rp[lo]).astype(np.int32))
        self.mode = mode
        owner = np.searchsorted(self.bounds, col, side="right") - 1
        if mode == "allgather":
            # map global column -> padded-gather position (owner*blk + offset)
            gcol = owner * self.blk + (col - self.bounds[owner])
            self.local = _local_format(
                CSR(hi - lo, self.P * self.blk, lrp, torch.from_numpy(gcol.astype(np.int32)), val), fmt, device).to(device)
        elif mode == "halo":
            uniq = np.unique(col)
            uown = np.searchsorted(self.bounds, uniq, side="right") - 1
            # what I need from each owner, and (after the exchange) what each rank needs from me
            need = [uniq[uown == q] for q in range(self.P)]
            counts = torch.tensor([len(x) for x in need], dtype=torch.int64)
            all_counts = comm.allgather(counts.to(device) if device != "cpu" and torch.device(device).type == "cuda"
                                        else counts).cpu()  # [P(sender), P(receiver)]
            self.send_counts = all_counts[:, self.r].tolist()  # how many each rank needs from me
            self.recv_counts = counts.tolist()
            maxc = int(all_counts.max())
            self.maxc = max(maxc, 1)
            req = torch.zeros((self.P, self.maxc), dtype=torch.int64)
            for q in range(self.P):
                req[q, :len(need[q])] = torch.from_numpy(need[q] - self.bounds[q])
            reqd = req.to(device)
            got = comm.alltoall(reqd.reshape(-1)).reshape(self.P, self.maxc)  # indices others need from me
            self.send_idx = got.to(torch.int64)
            self.send_mask = torch.zeros_like(self.send_idx, dtype=torch.bool)
            for q in range(self.P):
                self.send_mask[q, :self.send_counts[q]] = True
            # local column ids point into the received halo buffer [P, maxc]:
            # uniq is sorted and grouped by owner, so entry k of uniq lands at
            # owner*maxc + (k - first index of that owner's group)
            first = np.searchsorted(uown, np.arange(self.P))
            upos = uown * self.maxc + (np.arange(uniq.size) - first[uown])
            lcol = upos[np.searchsorted(uniq, col)]
            self.local = _local_format(
                CSR(hi - lo, self.P * self.maxc, lrp, torch.from_numpy(lcol.astype(np.int32)), val), fmt,
                device).to(device)
        else:
            raise ValueError(mode)

    def local_slice(self, x_full: torch.Tensor) -> torch.Tensor:
        return x_full[self.lo:self.hi]

    def __call__(self, x_local: torch.Tensor) -> torch.Tensor:
        """y_local = (A x)[lo:hi] given this rank's slice of x."""
        if self.mode == "allgather":
            buf = torch.zeros(self.blk, dtype=x_local.dtype, device=x_local.device)
            buf[:x_local.numel()] = x_local
            xg = self.comm.allgather(buf).reshape(-1)
        else:
            vals = torch.where(self.send_mask, x_local[self.send_idx.clamp(max=max(x_local.numel() - 1, 0))],
                               torch.zeros((), dtype=x_local.dtype, device=x_local.device))
            xg = self.comm.alltoall(vals.reshape(-1).contiguous())
        return spmv(self.local, xg.contiguous())


def colwise_matvec(comm: Comm, A_cols: torch.Tensor, x_local: torch.Tensor) -> torch.Tensor:
    """A_cols: this rank's column block (n x n/P) of a dense A; returns this
    rank's n/P slice of y via reduce-scatter."""
    partial = A_cols @ x_local
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
    partial = A_blk @ xb
    # reduce along the row to the diagonal rank (its rank in row_comm is `row`)
    row_comm.reduce_(partial, dst=row)
    return partial if row == col else None
