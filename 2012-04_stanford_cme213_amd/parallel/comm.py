"""Communicators: RCCL over xGMI (via ``torch.distributed``, backend ``nccl``
== RCCL on ROCm), gloo for CPU tensors, and an in-process loopback.

This replaces the reference's host-MPI layer (hw5: ``MPI_Isend``/``MPI_Irecv``/
``MPI_Waitall``, ``hw/hw5/2dHeat_solution.cpp:394-465``) and the
lecture collectives (Bcast / Reduce / Gather / Scatter / Allgather / Alltoall,
``slides/Lecture19.pdf``; ``Comm_split`` / ``Cart_sub``, ``slides/Lecture20.pdf``).

Design (MI355X-first): one process per GPU; point-to-point traffic is posted
as ONE grouped batch per exchange (``batch_isend_irecv`` -> ncclGroupStart/End)
on RCCL's own stream, so it overlaps kernels on the compute stream; completion
is a stream-side wait, never a host sync. Ranks that are co-located in one
process (:class:`LoopbackComm`) exchange by device copies -- this is the fake
backend the reference never had, used to test decomposition logic
on one GPU or on CPU.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class P2P:
    kind: str  # "send" | "recv"
    tensor: torch.Tensor
    peer: int


class Pending:
    """Handle for posted point-to-point traffic."""

    def __init__(self, works=()):
        self._works = list(works)

    def wait(self) -> None:
        for w in self._works:
            w.wait()
        self._works.clear()


class Comm:
    rank: int = 0
    size: int = 1

    def exchange(self, ops: list[P2P]) -> Pending:  # pragma: no cover - interface
        raise NotImplementedError

    def allreduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:  # pragma: no cover
        raise NotImplementedError

    def allgather(self, t: torch.Tensor) -> torch.Tensor:  # pragma: no cover
        raise NotImplementedError

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:  # pragma: no cover
        raise NotImplementedError

    def barrier(self) -> None:  # pragma: no cover
        raise NotImplementedError


_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
        "prod": dist.ReduceOp.PRODUCT}


class TorchComm(Comm):
    """torch.distributed process group (RCCL for cuda tensors, gloo for cpu)."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)
        self.backend = dist.get_backend(group)

    def _global(self, r: int) -> int:
        return r if self.group is None else dist.get_global_rank(self.group, r)

    def exchange(self, ops: list[P2P]) -> Pending:
        if not ops:
            return Pending()
        if any(self._staged(o.tensor) for o in ops):
            return self._exchange_host_staged(ops)
        p2p = [dist.P2POp(dist.isend if o.kind == "send" else dist.irecv, o.tensor, self._global(o.peer),
                          group=self.group) for o in ops]
        return Pending(dist.batch_isend_irecv(p2p))

    def _exchange_host_staged(self, ops: list[P2P]) -> Pending:
        """gloo moves host memory only: device tensors are staged through
        host copies (control-plane use, e.g. the initial halo fill of ranks
        whose data plane is :class:`~cme213x.parallel.ipc.NativeIpc`)."""
        host, back = [], []
        for o in ops:
            if o.kind == "send":
                host.append(o.tensor.detach().to("cpu", copy=True).contiguous())
            else:
                h = torch.empty(o.tensor.shape, dtype=o.tensor.dtype)
                host.append(h)
                back.append((o.tensor, h))
        p2p = [dist.P2POp(dist.isend if o.kind == "send" else dist.irecv, h, self._global(o.peer),
                          group=self.group) for o, h in zip(ops, host)]
        works = dist.batch_isend_irecv(p2p)

        class _Staged(Pending):
            def wait(self_inner):
                for w in works:
                    w.wait()
                for dst, h in back:
                    dst.copy_(h)

        return _Staged()

    def allreduce_(self, t, op="sum"):
        if self._staged(t):
            h = t.cpu()
            dist.all_reduce(h, _OPS[op], group=self.group)
            t.copy_(h)
            return t
        dist.all_reduce(t, _OPS[op], group=self.group)
        return t

    def _staged(self, t: torch.Tensor) -> bool:
        """gloo moves host memory only: device tensors go through host copies
        (control plane of shared-GPU rehearsals)."""
        return self.backend == "gloo" and t.is_cuda

    def allgather(self, t):
        if self._staged(t):
            return self.allgather(t.cpu()).to(t.device)
        flat = t.contiguous().reshape(-1)
        out = torch.empty(self.size * flat.numel(), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, flat, group=self.group)
        return out.view((self.size,) + tuple(t.shape))

    def reduce_scatter(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self._staged(t):
            return self.reduce_scatter(t.cpu(), op).to(t.device)
        out = torch.empty((t.shape[0] // self.size,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.reduce_scatter_tensor(out, t.contiguous(), _OPS[op], group=self.group)
        return out

    def alltoall(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty_like(t)
        dist.all_to_all_single(out, t.contiguous(), group=self.group)
        return out

    def broadcast_(self, t, src=0):
        if self._staged(t):
            h = t.cpu()
            dist.broadcast(h, self._global(src), group=self.group)
            t.copy_(h)
            return t
        dist.broadcast(t, self._global(src), group=self.group)
        return t

    def reduce_(self, t: torch.Tensor, dst: int = 0, op: str = "sum") -> torch.Tensor:
        dist.reduce(t, self._global(dst), _OPS[op], group=self.group)
        return t

    def gather(self, t: torch.Tensor, dst: int = 0):
        lst = [torch.empty_like(t) for _ in range(self.size)] if self.rank == dst else None
        dist.gather(t.contiguous(), lst, self._global(dst), group=self.group)
        return lst

    def scatter(self, chunks, out: torch.Tensor, src: int = 0) -> torch.Tensor:
        dist.scatter(out, chunks if self.rank == src else None, self._global(src), group=self.group)
        return out

    def barrier(self):
        if self.backend == "nccl":
            dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier(group=self.group)

    def split(self, color: int, key: int | None = None) -> "TorchComm":
        """MPI_Comm_split: ranks with equal ``color`` form a sub-communicator,
        ordered by ``key`` (default: parent rank). Collective over the group."""
        key = self.rank if key is None else key
        mine = torch.tensor([color, key, self.rank], dtype=torch.int64)
        if self.backend == "nccl":
            mine = mine.cuda()
        allv = self.allgather(mine).cpu().tolist()
        groups: dict[int, list] = {}
        for c, k, r in allv:
            groups.setdefault(c, []).append((k, r))
        mine_group = None
        for c in sorted(groups):  # every rank creates every group in the same order
            members = [self._global(r) for _, r in sorted(groups[c])]
            g = dist.new_group(members)
            if c == color:
                mine_group = g
        return TorchComm(mine_group)


class LoopbackComm(Comm):
    """Single-process communicator of size 1: every peer is ourselves. Used
    when all subdomains of a decomposition live in one process (exchanges
    are performed by the caller as direct copies)."""

    def __init__(self):
        self.rank, self.size = 0, 1

    def exchange(self, ops):
        if ops:
            raise RuntimeError("LoopbackComm has no remote peers")
        return Pending()

    def allreduce_(self, t, op="sum"):
        return t

    def allgather(self, t):
        return t.unsqueeze(0).clone()

    def broadcast_(self, t, src=0):
        return t

    def reduce_scatter(self, t, op="sum"):
        return t.clone()

    def alltoall(self, t):
        return t.clone()

    def reduce_(self, t, dst=0, op="sum"):
        return t

    def gather(self, t, dst=0):
        return [t.clone()]

    def scatter(self, chunks, out, src=0):
        out.copy_(chunks[0])
        return out

    def split(self, color, key=None):
        return self

    def barrier(self):
        pass


def init_from_env(device_type: str | None = None, backend: str | None = None, share_gpu: bool = False) -> Comm:
    """torchrun-style bootstrap (RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT).
    Returns :class:`LoopbackComm` when WORLD_SIZE is unset or 1.
    ``share_gpu``: every rank on device 0 (rehearsing a multi-rank run on one
    GPU; RCCL refuses that, so pair it with ``backend="gloo"``)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return LoopbackComm()
    if not dist.is_initialized():
        if device_type is None:
            device_type = "cuda" if torch.cuda.is_available() else "cpu"
        backend = backend or ("nccl" if device_type == "cuda" else "gloo")
        if device_type == "cuda":
            torch.cuda.set_device(0 if share_gpu else int(os.environ.get("LOCAL_RANK", "0")))
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group(backend=backend, **kw)
    return TorchComm()
