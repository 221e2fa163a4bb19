"""Native RCCL communicator (``ncclCommInitRank`` from C++), bootstrapped
over an existing torch.distributed group: rank 0 draws the unique id and
broadcasts it. Used where per-call Python overhead matters (the distributed
stencil's K-step loop runs entirely in ``cme_heat_dist_run``)."""
from __future__ import annotations

import ctypes
import os

import torch
import torch.distributed as dist

from .. import _ext

_ext.proto(_ext.HIP_PROTOS, "cme_rccl_unique_id", "p")
_ext.proto(_ext.HIP_PROTOS, "cme_rccl_init", "pipi")
_ext.proto(_ext.HIP_PROTOS, "cme_rccl_destroy", "p")
_ext.proto(_ext.HIP_PROTOS, "cme_rccl_allreduce", "pppqiip")
_ext.proto(_ext.HIP_PROTOS, "cme_rccl_allgather", "pppqip")
_ext.proto(_ext.HIP_PROTOS, "cme_rccl_p2p", "pippppip")
_ext.proto(_ext.HIP_PROTOS, "cme_rccl_async_error", "pp")
_ext.proto(_ext.HIP_PROTOS, "cme_rccl_abort", "p")

_DT = {torch.float32: 0, torch.float64: 1, torch.int32: 2, torch.int64: 3, torch.uint8: 4}
_OP = {"sum": 0, "max": 1, "min": 2, "prod": 3}


class NativeRccl:
    def __init__(self, group=None):
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed must be initialised first")
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)
        if os.environ.get("CME_FAULT_RCCL_INIT", "0") not in ("", "0"):
            # fault injection (tests of the transport chain): every rank that
            # sees it fails here, before the collective ncclCommInitRank
            raise RuntimeError("RCCL init failed (CME_FAULT_RCCL_INIT)")
        dev = torch.device("cuda", torch.cuda.current_device())
        uid = torch.zeros(128, dtype=torch.uint8)
        if self.rank == 0:
            buf = ctypes.create_string_buffer(128)
            _ext.call_hip("cme_rccl_unique_id", ctypes.addressof(buf))
            uid = torch.frombuffer(bytearray(buf.raw), dtype=torch.uint8).clone()
        uid_d = uid.to(dev)
        dist.broadcast(uid_d, dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        raw = bytes(uid_d.cpu().numpy().tobytes())
        self._id = ctypes.create_string_buffer(raw, 128)
        h = ctypes.c_void_p()
        _ext.call_hip("cme_rccl_init", ctypes.addressof(h), self.size, ctypes.addressof(self._id), self.rank)
        self.handle = h.value

    def allreduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        _ext.call_hip("cme_rccl_allreduce", self.handle, t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype], _OP[op],
                      _ext.stream_ptr(t.device))
        return t

    def allgather(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty((self.size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        _ext.call_hip("cme_rccl_allgather", self.handle, t.data_ptr(), out.data_ptr(), t.numel(), _DT[t.dtype],
                      _ext.stream_ptr(t.device))
        return out

    def p2p(self, ops, stream: torch.cuda.Stream | None = None) -> None:
        """ops: list of (kind, tensor, peer) in one ncclGroupStart/End, on
        ``stream`` (default: the current stream). All tensors share a dtype."""
        n = len(ops)
        if n == 0:
            return
        peers = (ctypes.c_int * n)(*[o[2] for o in ops])
        sends = (ctypes.c_int * n)(*[1 if o[0] == "send" else 0 for o in ops])
        ptrs = (ctypes.c_void_p * n)(*[o[1].data_ptr() for o in ops])
        cnts = (ctypes.c_longlong * n)(*[o[1].numel() for o in ops])
        _ext.call_hip("cme_rccl_p2p", self.handle, n, ctypes.addressof(peers), ctypes.addressof(sends),
                      ctypes.addressof(ptrs), ctypes.addressof(cnts), _DT[ops[0][1].dtype],
                      stream.cuda_stream if stream is not None else _ext.stream_ptr(ops[0][1].device))

    def check(self) -> None:
        """Raise if the communicator reported an asynchronous error (and
        abort it, so no collective can hang on a dead peer)."""
        err = ctypes.c_int(0)
        _ext.call_hip("cme_rccl_async_error", self.handle, ctypes.addressof(err))
        if err.value != 0:
            self.abort()
            raise RuntimeError(f"RCCL asynchronous error {err.value}; communicator aborted")

    def abort(self) -> None:
        if self.handle:
            _ext.call_hip("cme_rccl_abort", self.handle)
            self.handle = None

    def close(self) -> None:
        if self.handle:
            _ext.call_hip("cme_rccl_destroy", self.handle)
            self.handle = None
