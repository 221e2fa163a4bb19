"""Scans across GPUs: each rank scans its contiguous shard, then one
all-gather of per-rank carries fixes the shard prefixes.

This is the cross-device level of the scan hierarchy (SURVEY §5 "segmented
scan with carry-in across blocks and across GPUs"): lane -> wave (DPP) ->
block (LDS) -> device (decoupled look-back / reduce-then-scan) -> GPUs
(RCCL all-gather of one or two scalars per rank). The reference's multi-block
scan-then-add (``my-refs/scan.pdf`` Fig. 5) is the same idea one level down.

* :func:`dist_scan` -- plain (inclusive / exclusive) sum scan of a sharded
  vector.
* :func:`dist_segmented_scan` -- inclusive segmented sum scan with head flags.
  A segment may straddle shards: the carry into rank r is the sum of the
  trailing partial segments of ranks j..r-1, where j is the last rank before
  r that contains a segment head (or 0).
* :class:`DistSpmvScan` -- the final project's iterated ``a <- segscan(a *
  x[k])`` (``hw/hw_final/programming/fp.cu:168-185``) with ``a`` sharded over
  ranks. Per iteration: one fused local segmented scan, one all-gather of
  (tail, has_head) pairs, one masked add -- all enqueued without a host
  synchronisation.

Shards need not be equal; concatenating the shards in rank order gives the
global vector.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops.scan import scan, segmented_scan
from .comm import Comm


def dist_scan(x: torch.Tensor, comm: Comm, exclusive: bool = False) -> torch.Tensor:
    """Global scan of the concatenation of every rank's shard ``x``."""
    if x.numel() == 0:
        y = x.clone()
        total = torch.zeros(1, dtype=x.dtype, device=x.device)
    else:
        y = scan(x, exclusive=exclusive)
        total = x.sum().view(1).to(x.dtype) if exclusive else y[-1:].clone()
    totals = comm.allgather(total).view(-1)
    carry = totals[:comm.rank].sum()
    return y.add_(carry.to(y.dtype))


def _carry_in(tails: torch.Tensor, has_head: torch.Tensor, rank: int) -> torch.Tensor:
    """Device-side carry into ``rank`` from (tail, has_head) of all ranks."""
    if rank == 0:
        return torch.zeros((), dtype=tails.dtype, device=tails.device)
    prev_heads = has_head[:rank]
    idx = torch.arange(rank, device=tails.device)
    # last rank < `rank` with a head (or 0 when none): max over idx * has_head
    j = torch.max(torch.where(prev_heads, idx, torch.zeros_like(idx)))
    mask = idx >= j
    return (tails[:rank] * mask.to(tails.dtype)).sum()


def dist_segmented_scan(x: torch.Tensor, flags: torch.Tensor, comm: Comm,
                        mul: torch.Tensor | None = None) -> torch.Tensor:
    """Inclusive segmented sum scan (``x`` or ``x*mul``) of the sharded vector.
    ``flags``: uint8 per element, 1 at segment heads (global index 0 need not
    be flagged)."""
    y = segmented_scan(x, flags, mul=mul)
    heads = torch.nonzero(flags).view(-1)
    first = int(heads[0]) if heads.numel() else x.numel()
    pair = torch.stack([y[-1] if x.numel() else torch.zeros((), dtype=x.dtype, device=x.device),
                        torch.tensor(float(heads.numel() > 0), dtype=x.dtype, device=x.device)]).view(1, 2)
    allp = comm.allgather(pair).view(-1, 2)
    carry = _carry_in(allp[:, 0], allp[:, 1] > 0, comm.rank)
    if first > 0:
        y[:first] += carry
    return y


class DistSpmvScan:
    """Sharded final-project iteration. ``a_local``/``xx_local``/``flags_local``
    are this rank's contiguous slice (``xx = x[k]`` pre-gathered, as in
    ``fp.cu:124-125``)."""

    def __init__(self, a_local: torch.Tensor, xx_local: torch.Tensor, flags_local: torch.Tensor, comm: Comm):
        self.a = a_local
        self.xx = xx_local
        self.flags = flags_local
        self.comm = comm
        heads = torch.nonzero(flags_local).view(-1)
        self.first = int(heads[0]) if heads.numel() else a_local.numel()
        self.has_head = torch.tensor(float(heads.numel() > 0), dtype=a_local.dtype, device=a_local.device)

    @staticmethod
    def shard(prob, rank: int, world: int, device="cpu"):
        """(a, xx, flags) slices of a :class:`~cme213x.models.spmv_scan.
        SpmvScanProblem` for ``rank`` (near-equal contiguous element ranges)."""
        n = prob.n
        lo, hi = n * rank // world, n * (rank + 1) // world
        flags = np.zeros(n, dtype=np.uint8)
        flags[prob.s[:-1]] = 1
        xx = prob.x[prob.k[lo:hi]]
        return (torch.from_numpy(prob.a[lo:hi].copy()).to(device), torch.from_numpy(xx.copy()).to(device),
                torch.from_numpy(flags[lo:hi].copy()).to(device))

    def step(self) -> None:
        y = segmented_scan(self.a, self.flags, out=self.a, mul=self.xx)
        tail = y[-1:] if y.numel() else torch.zeros(1, dtype=y.dtype, device=y.device)
        pair = torch.cat([tail, self.has_head.view(1)]).view(1, 2)
        allp = self.comm.allgather(pair).view(-1, 2)
        carry = _carry_in(allp[:, 0], allp[:, 1] > 0, self.comm.rank)
        if self.first > 0:
            self.a[:self.first] += carry

    def run(self, iters: int) -> torch.Tensor:
        for _ in range(iters):
            self.step()
        return self.a
