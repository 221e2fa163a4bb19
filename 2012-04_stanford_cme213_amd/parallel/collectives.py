"""Hand-built collectives from point-to-point (the lecture algorithms,
``slides/Lecture18.pdf`` ring all-gather, ``Lecture19.pdf`` trees), next to
the library (RCCL) collectives they are measured against.

On MI355X the xGMI fabric is point-to-point (7 links per GPU), so a ring
all-gather moves (P-1)/P of the data over ONE link per step -- exactly the
per-link-bound pattern the library ring uses. These implementations exist to
teach/measure that; production code calls ``Comm.allgather`` (RCCL).
"""
from __future__ import annotations

import torch

from .comm import P2P, TorchComm


def ring_allgather(comm: TorchComm, t: torch.Tensor) -> torch.Tensor:
    """Non-blocking ring all-gather (Gather_ring): P-1 steps, each rank sends
    the block it received last step to its right neighbour."""
    P, r = comm.size, comm.rank
    out = torch.empty((P,) + tuple(t.shape), dtype=t.dtype, device=t.device)
    out[r].copy_(t)
    right, left = (r + 1) % P, (r - 1) % P
    for step in range(P - 1):
        send_blk = (r - step) % P
        recv_blk = (r - step - 1) % P
        comm.exchange([P2P("send", out[send_blk], right), P2P("recv", out[recv_blk], left)]).wait()
    return out


def tree_broadcast(comm: TorchComm, t: torch.Tensor, root: int = 0) -> torch.Tensor:
    """Binomial-tree broadcast: log2(P) rounds of point-to-point sends."""
    P = comm.size
    rel = (comm.rank - root) % P
    mask = 1
    while mask < P:  # receive phase: find the round in which we get the data
        if rel & mask:
            src = (rel - mask + root) % P
            comm.exchange([P2P("recv", t, src)]).wait()
            break
        mask <<= 1
    mask >>= 1
    while mask > 0:  # forward to the subtree
        if rel + mask < P:
            dst = (rel + mask + root) % P
            comm.exchange([P2P("send", t, dst)]).wait()
        mask >>= 1
    return t


def tree_reduce_sum(comm: TorchComm, t: torch.Tensor, root: int = 0) -> torch.Tensor:
    """Binomial-tree sum reduction to ``root`` (the tree dot-product of the
    iso-efficiency analysis, Lecture20)."""
    P = comm.size
    rel = (comm.rank - root) % P
    acc = t.clone()
    tmp = torch.empty_like(t)
    mask = 1
    while mask < P:
        if rel & mask:
            dst = (rel - mask + root) % P
            comm.exchange([P2P("send", acc, dst)]).wait()
            break
        src_rel = rel + mask
        if src_rel < P:
            comm.exchange([P2P("recv", tmp, (src_rel + root) % P)]).wait()
            acc += tmp
        mask <<= 1
    return acc
