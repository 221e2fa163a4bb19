"""Cartesian process topologies, blocking point-to-point and derived
datatypes on top of :class:`~cme213x.parallel.comm.Comm` -- the MPI helpers
the lectures teach but the reference's code never calls (SURVEY §2.3:
``MPI_Dims_create``, ``MPI_Cart_create`` / ``Cart_coords`` / ``Cart_rank`` /
``Cart_shift`` / ``Cart_sub``, ``Send`` / ``Recv`` / ``Sendrecv``,
``Type_vector``; ``slides/Lecture18.pdf``, ``slides/Lecture20.pdf``).

MI355X notes: a process grid is bookkeeping only -- every GPU of a node is one
xGMI hop from every other, so a Cartesian neighbour costs the same as any
other peer. What matters is that one exchange's partners are DISTINCT peers,
so its traffic spreads over several of the 7 links instead of queueing on
one; :meth:`CartComm.halo_exchange` posts all faces as one grouped batch for
that reason. Sub-communicators are real process groups (RCCL communicators
for ``nccl``), created collectively through :meth:`Comm.split`.

Ranks are numbered row-major (the last dimension varies fastest), as MPI's
``reorder=0`` numbering.
"""
from __future__ import annotations

import itertools
import math

import torch

from .comm import P2P, Comm, LoopbackComm


def dims_create(nnodes: int, ndims: int, dims: list[int] | None = None) -> list[int]:
    """``MPI_Dims_create``: a balanced factorisation of ``nnodes`` into
    ``ndims`` factors, non-increasing. Entries of ``dims`` > 0 stay fixed;
    zeros are filled."""
    dims = list(dims) if dims is not None else [0] * ndims
    if len(dims) != ndims:
        raise ValueError("len(dims) != ndims")
    fixed = math.prod(d for d in dims if d > 0)
    if fixed <= 0 or nnodes % fixed:
        raise ValueError(f"{nnodes} nodes not divisible by the fixed dims {dims}")
    free = [i for i, d in enumerate(dims) if d <= 0]
    rest = nnodes // fixed
    if not free:
        if rest != 1:
            raise ValueError("dims fully specified but their product != nnodes")
        return dims
    primes, n, p = [], rest, 2
    while p * p <= n:
        while n % p == 0:
            primes.append(p)
            n //= p
        p += 1
    if n > 1:
        primes.append(n)
    slots = [1] * len(free)
    for f in sorted(primes, reverse=True):  # largest factor onto the smallest slot
        slots[slots.index(min(slots))] *= f
    slots.sort(reverse=True)
    for i, v in zip(free, slots):
        dims[i] = v
    return dims


class CartComm:
    """``MPI_Cart_create`` over an existing communicator (no reordering)."""

    def __init__(self, comm: Comm, dims: list[int], periods: list[bool] | None = None):
        self.comm = comm
        self.dims = [int(d) for d in dims]
        self.periods = [bool(p) for p in (periods or [False] * len(self.dims))]
        if len(self.periods) != len(self.dims):
            raise ValueError("periods and dims differ in length")
        if math.prod(self.dims) != comm.size:
            raise ValueError(f"grid {self.dims} does not cover {comm.size} ranks")
        self.ndims = len(self.dims)
        self.rank = comm.rank
        self.size = comm.size
        self.my_coords = self.coords(self.rank)

    # -- rank <-> coordinates ---------------------------------------------
    def coords(self, rank: int) -> list[int]:
        """``MPI_Cart_coords``."""
        if not 0 <= rank < self.size:
            raise ValueError(f"rank {rank} outside the grid")
        out = []
        for d in reversed(self.dims):
            out.append(rank % d)
            rank //= d
        return out[::-1]

    def rank_of(self, coords) -> int:
        """``MPI_Cart_rank``; periodic dimensions wrap, out-of-range
        coordinates of a non-periodic dimension give -1 (``MPI_PROC_NULL``)."""
        r = 0
        for c, d, per in zip(coords, self.dims, self.periods):
            if per:
                c %= d
            elif not 0 <= c < d:
                return -1
            r = r * d + c
        return r

    def shift(self, direction: int, disp: int = 1) -> tuple[int, int]:
        """``MPI_Cart_shift``: (source, dest) for a shift of ``disp`` along
        ``direction``; -1 past a non-periodic edge."""
        src, dst = list(self.my_coords), list(self.my_coords)
        src[direction] -= disp
        dst[direction] += disp
        return self.rank_of(src), self.rank_of(dst)

    def neighbours(self) -> dict[tuple[int, int], int]:
        """The 2*ndims face neighbours ``{(dim, -1 | +1): rank}``, -1 at edges."""
        out = {}
        for d in range(self.ndims):
            lo, hi = self.shift(d, 1)
            out[(d, -1)], out[(d, +1)] = lo, hi
        return out

    def sub(self, remain_dims: list[bool]) -> "CartComm":
        """``MPI_Cart_sub``: keep the dimensions flagged in ``remain_dims``;
        ranks that agree on every dropped coordinate form one sub-grid.
        Collective over the parent communicator."""
        if len(remain_dims) != self.ndims:
            raise ValueError("remain_dims length != ndims")
        color = key = 0
        kdims, kper = [], []
        for c, d, per, keep in zip(self.my_coords, self.dims, self.periods, remain_dims):
            if keep:
                key = key * d + c
                kdims.append(d)
                kper.append(per)
            else:
                color = color * d + c
        sub = self.comm.split(color, key)
        if not kdims:  # every dimension dropped: a one-rank grid
            return CartComm(sub, [1], [False])
        return CartComm(sub, kdims, kper)

    def halo_exchange(self, sends: dict[tuple[int, int], torch.Tensor],
                      recvs: dict[tuple[int, int], torch.Tensor]):
        """Post every face exchange as ONE grouped batch: ``sends[(d, s)]``
        goes to the neighbour on side ``s`` of dimension ``d`` and
        ``recvs[(d, s)]`` is filled from it; missing neighbours are skipped.
        Returns a :class:`~cme213x.parallel.comm.Pending`. A periodic
        dimension of extent 2 makes both faces the same peer; RCCL
        point-to-point has no tags to tell them apart, so it is rejected."""
        for d, (n, per) in enumerate(zip(self.dims, self.periods)):
            if per and n == 2 and any(k[0] == d for k in list(sends) + list(recvs)):
                raise ValueError(f"dimension {d}: periodic extent 2 -- both faces are one peer")
        nb = self.neighbours()
        ops = [P2P("send", t, nb[k]) for k, t in sends.items() if nb[k] >= 0]
        ops += [P2P("recv", t, nb[k]) for k, t in recvs.items() if nb[k] >= 0]
        return self.comm.exchange(ops)


def cart_create(comm: Comm, dims: list[int] | None = None, periods: list[bool] | None = None,
                ndims: int = 2) -> CartComm:
    """``MPI_Dims_create`` (for zero / missing entries) + ``MPI_Cart_create``."""
    if dims is None:
        dims = dims_create(comm.size, ndims)
    elif any(d <= 0 for d in dims):
        dims = dims_create(comm.size, len(dims), dims)
    return CartComm(comm, dims, periods)


# -- blocking point-to-point -------------------------------------------------
def send(comm: Comm, t: torch.Tensor, dest: int) -> None:
    """Blocking ``MPI_Send`` (returns when ``t`` may be reused)."""
    comm.exchange([P2P("send", t, dest)]).wait()


def recv(comm: Comm, t: torch.Tensor, source: int) -> torch.Tensor:
    """Blocking ``MPI_Recv`` into ``t``."""
    comm.exchange([P2P("recv", t, source)]).wait()
    return t


def sendrecv(comm: Comm, sendbuf: torch.Tensor, dest: int, recvbuf: torch.Tensor, source: int) -> torch.Tensor:
    """``MPI_Sendrecv``: both directions posted in one group, so a ring shift
    in which every rank sends first cannot deadlock (the Lecture18 pitfall of
    blocking ``Send`` before ``Recv``). -1 (``MPI_PROC_NULL``) skips a side."""
    if isinstance(comm, LoopbackComm):
        if dest == 0 and source == 0:
            recvbuf.copy_(sendbuf)
        return recvbuf
    ops = []
    if dest >= 0:
        ops.append(P2P("send", sendbuf, dest))
    if source >= 0:
        ops.append(P2P("recv", recvbuf, source))
    comm.exchange(ops).wait()
    return recvbuf


# -- derived datatypes ---------------------------------------------------------
class VectorType:
    """``MPI_Type_vector(count, blocklength, stride)`` over a flat buffer:
    ``count`` blocks of ``blocklength`` elements whose starts are ``stride``
    apart (the column-halo type of a row-major grid). RCCL moves contiguous
    bytes only, so on the GPU a strided view is packed into a staging buffer by
    one copy kernel (the distributed heat loop does exactly this for its
    column halos, ``csrc/hip/dist_heat.hip`` ``pack_block_kernel``)."""

    def __init__(self, count: int, blocklength: int, stride: int):
        if count < 1 or blocklength < 1:
            raise ValueError("count and blocklength must be positive")
        if blocklength > stride:
            raise ValueError("blocklength > stride (overlapping blocks)")
        self.count, self.blocklength, self.stride = count, blocklength, stride

    @property
    def size(self) -> int:
        return self.count * self.blocklength

    def view(self, base: torch.Tensor, offset: int = 0) -> torch.Tensor:
        """Strided ``(count, blocklength)`` view of contiguous ``base`` at
        element ``offset``."""
        if not base.is_contiguous():
            raise ValueError("base buffer must be contiguous")
        flat = base.reshape(-1)
        if offset + (self.count - 1) * self.stride + self.blocklength > flat.numel():
            raise ValueError("vector type runs past the end of the buffer")
        return flat.as_strided((self.count, self.blocklength), (self.stride, 1), flat.storage_offset() + offset)

    def pack(self, base: torch.Tensor, offset: int = 0, out: torch.Tensor | None = None) -> torch.Tensor:
        v = self.view(base, offset)
        if out is None:
            return v.contiguous().reshape(-1)
        out.view(self.count, self.blocklength).copy_(v)
        return out

    def unpack(self, packed: torch.Tensor, base: torch.Tensor, offset: int = 0) -> None:
        self.view(base, offset).copy_(packed.reshape(self.count, self.blocklength))


def all_coords(dims: list[int]) -> list[list[int]]:
    """Every coordinate of a grid, in rank order."""
    return [list(c) for c in itertools.product(*[range(d) for d in dims])]
