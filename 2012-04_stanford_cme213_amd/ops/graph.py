"""CSR graph propagation (PageRank, hw1 p2).

``propagate(g, x)`` is one sweep ``out[i] = 0.5/N + 0.5*sum_j x[e_j]*inv[e_j]``
(``hw/hw1/programming/pagerank.cu:70-83``); ``iterate`` runs the 20-sweep
ping-pong of ``device_graph_iterate`` (``:86-143``) with the prescaled-gather
kernels and no host synchronisation between sweeps.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from .. import _ext

_ext.proto(_ext.HIP_PROTOS, "cme_pr_prescale", "pppip")
_ext.proto(_ext.HIP_PROTOS, "cme_pr_propagate_ref", "pppppip")
_ext.proto(_ext.HIP_PROTOS, "cme_pr_propagate", "ppppppiip")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_pr_propagate", "pppppi")
_ext.proto(_ext.HIP_PROTOS, "cme_pr_propagate_blocked", "pppppppiiip")


@dataclass
class CSRGraph:
    indices: torch.Tensor  # int32 (n+1,) row offsets (uint32 semantics)
    edges: torch.Tensor  # int32 (nnz,) targets
    inv_deg: torch.Tensor  # float32 (n,)

    @property
    def n(self) -> int:
        return self.inv_deg.numel()

    def to(self, device) -> "CSRGraph":
        return CSRGraph(self.indices.to(device), self.edges.to(device), self.inv_deg.to(device))


def make_graph(n: int = 1 << 21, avg_edges: int = 8, seed: int = 0) -> CSRGraph:
    """The reference generator (``pagerank.cu:185-204``): node i has
    ``(i % (2*avg-1)) + 1`` out-edges to uniformly random targets."""
    rng = np.random.default_rng(seed)
    deg = (np.arange(n, dtype=np.int64) % (2 * avg_edges - 1)) + 1
    idx = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(deg, out=idx[1:])
    if idx[-1] >= n * avg_edges:
        raise ValueError("more edges than we have space for")
    edges = rng.integers(0, n, size=int(idx[-1]), dtype=np.int64)
    inv = (1.0 / deg.astype(np.float32)).astype(np.float32)
    return CSRGraph(torch.from_numpy(idx.astype(np.int32)), torch.from_numpy(edges.astype(np.int32)),
                    torch.from_numpy(inv))


@dataclass
class BlockedGraph:
    """Edges re-sorted by (block of the gathered node, row): ``blocks`` column
    blocks of ``ceil(n / blocks)`` nodes, row offsets ``rp`` of length
    ``blocks*n + 1`` (row i of block b: ``[rp[b*n+i], rp[b*n+i+1])``); within
    a (block, row) the edges keep their CSR order."""
    rp: torch.Tensor
    edges: torch.Tensor
    inv_deg: torch.Tensor
    blocks: int

    @property
    def n(self) -> int:
        return self.inv_deg.numel()


def block_columns(g: CSRGraph, blocks: int = 4) -> BlockedGraph:
    """Column-blocked copy of ``g`` (one-time preprocessing with tensor ops,
    on g's device): a sweep then gathers from one 1/blocks slice of the vector
    at a time (:func:`iterate` with ``blocks``)."""
    n = g.n
    dev = g.edges.device
    deg = (g.indices[1:] - g.indices[:-1]).to(torch.int64)
    row = torch.repeat_interleave(torch.arange(n, device=dev), deg)
    bs = (n + blocks - 1) // blocks
    blk = g.edges.to(torch.int64) // bs
    key = blk * n + row
    order = torch.sort(key, stable=True).indices
    edges = g.edges[order].contiguous()
    counts = torch.bincount(key, minlength=blocks * n)
    rp = torch.zeros(blocks * n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(counts, 0, out=rp[1:])
    return BlockedGraph(rp.to(torch.int32), edges, g.inv_deg, blocks)


def propagate_ref(g: CSRGraph, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """One sweep with the reference's two-gathers-per-edge arithmetic."""
    out = torch.empty_like(x) if out is None else out
    if x.is_cuda:
        _ext.call_hip("cme_pr_propagate_ref", g.indices.data_ptr(), g.edges.data_ptr(), x.data_ptr(),
                      out.data_ptr(), g.inv_deg.data_ptr(), g.n, _ext.stream_ptr(x.device))
    else:
        _ext.call_cpu("cme_cpu_pr_propagate", g.indices.data_ptr(), g.edges.data_ptr(), x.data_ptr(),
                      out.data_ptr(), g.inv_deg.data_ptr(), g.n)
    return out


def iterate(g, x0: torch.Tensor, iters: int = 20, group: int = 1) -> torch.Tensor:
    """``iters`` sweeps (even, like the reference); returns the final vector.
    group = lanes per row on the GPU (1 keeps the CPU summation order).
    ``g`` may be a :class:`BlockedGraph` (GPU): column-blocked sweeps, each
    row summed block by block (same terms, different association order)."""
    if isinstance(g, BlockedGraph):
        return _iterate_blocked(g, x0, iters, group)
    if iters % 2:
        raise ValueError("iters must be even (A/B ping-pong, as in the reference)")
    if not x0.is_cuda:
        a, b = x0.clone(), torch.empty_like(x0)
        for _ in range(iters // 2):
            propagate_ref(g, a, b)
            propagate_ref(g, b, a)
        return a
    s = _ext.stream_ptr(x0.device)
    n = g.n
    out = torch.empty_like(x0)
    ya, yb = torch.empty_like(x0), torch.empty_like(x0)
    _ext.call_hip("cme_pr_prescale", x0.data_ptr(), g.inv_deg.data_ptr(), ya.data_ptr(), n, s)
    for it in range(iters):
        yi, yo = (ya, yb) if it % 2 == 0 else (yb, ya)
        _ext.call_hip("cme_pr_propagate", g.indices.data_ptr(), g.edges.data_ptr(), yi.data_ptr(), out.data_ptr(),
                      yo.data_ptr(), g.inv_deg.data_ptr(), n, group, s)
    return out


def _iterate_blocked(g: BlockedGraph, x0: torch.Tensor, iters: int, group: int) -> torch.Tensor:
    if iters % 2:
        raise ValueError("iters must be even (A/B ping-pong, as in the reference)")
    if not x0.is_cuda:
        raise ValueError("column-blocked sweeps run on the GPU")
    s = _ext.stream_ptr(x0.device)
    n = g.n
    out = torch.empty_like(x0)
    acc = torch.empty_like(x0)
    ya, yb = torch.empty_like(x0), torch.empty_like(x0)
    _ext.call_hip("cme_pr_prescale", x0.data_ptr(), g.inv_deg.data_ptr(), ya.data_ptr(), n, s)
    for it in range(iters):
        yi, yo = (ya, yb) if it % 2 == 0 else (yb, ya)
        _ext.call_hip("cme_pr_propagate_blocked", g.rp.data_ptr(), g.edges.data_ptr(), yi.data_ptr(), acc.data_ptr(),
                      out.data_ptr(), yo.data_ptr(), g.inv_deg.data_ptr(), n, g.blocks, group, s)
    return out


def bytes_model(g: CSRGraph, iters: int = 20) -> int:
    """The student's traffic model (``hw/hw1/programming/analysis/pagerank.cu:
    47-62``): 2 uint per node + (2 float + 2 uint) per edge + 1 float per node,
    per sweep -- used to quote GB/s comparably with BASELINE.md #5."""
    n, nnz = g.n, g.edges.numel()
    return iters * (n * 8 + nnz * 16 + n * 4)
