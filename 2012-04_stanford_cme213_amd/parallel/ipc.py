"""IPC peer communicator: zero-copy access to other processes' device memory
(SURVEY §2.6 "IpcPeerComm": ``hipIpcGetMemHandle`` / peer loads).

Each process exports device tensors with :meth:`NativeIpc.export` (an IPC
handle of the allocation base + the tensor's offset in it), the descriptors
are all-gathered over any torch.distributed group (gloo is enough -- this is
control-plane traffic only), and every process maps the tensors of the peers
it needs with :meth:`NativeIpc.open`. Kernels then read the peers' memory
directly: over xGMI between MI355X devices, or plain HBM when several ranks
share one GPU -- which is what makes a real multi-process halo exchange
testable on a single device (RCCL refuses two ranks on one GPU).

The distributed heat loop uses it as transport 3 of ``cme_heat_dist_run``
(``csrc/hip/dist_heat.hip``): the same pack / staging / unpack plan as the
RCCL transport, the "move" done by a pull kernel, cross-process order kept
by epoch words in mapped memory. This mirrors the async overlap of
``hw/hw5/2dHeat_solution.cpp:537-628`` with no host in the loop.
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from .. import _ext

_ext.proto(_ext.HIP_PROTOS, "cme_ipc_export", "ppp")
_ext.proto(_ext.HIP_PROTOS, "cme_ipc_open", "pp")
_ext.proto(_ext.HIP_PROTOS, "cme_ipc_close", "p")

HANDLE_BYTES = 64


class NativeIpc:
    """Bootstrap + bookkeeping for IPC-mapped peer memory. ``group``: the
    torch.distributed group the descriptors are exchanged over."""

    def __init__(self, group=None):
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed must be initialised first")
        self.group = group
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)
        self._opened: list[int] = []
        self._keep: list = []  # exported tensors and host words the kernels point into

    @staticmethod
    def export(t: torch.Tensor) -> tuple[bytes, int]:
        """(handle of t's allocation base, byte offset of t in it)."""
        if not t.is_cuda:
            raise ValueError("only device tensors can be exported")
        h = ctypes.create_string_buffer(HANDLE_BYTES)
        off = ctypes.c_longlong(0)
        _ext.call_hip("cme_ipc_export", t.data_ptr(), ctypes.addressof(h), ctypes.addressof(off))
        return bytes(h.raw), int(off.value)

    def open(self, handle: bytes, offset: int) -> int:
        """Map a peer's exported allocation; returns the device address of the
        exported tensor in THIS process (base + offset)."""
        buf = ctypes.create_string_buffer(handle, HANDLE_BYTES)
        base = ctypes.c_void_p()
        _ext.call_hip("cme_ipc_open", ctypes.addressof(buf), ctypes.addressof(base))
        self._opened.append(base.value)
        return base.value + offset

    def allgather_object(self, obj):
        out = [None] * self.size
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def barrier(self) -> None:
        if dist.get_backend(self.group) == "nccl":
            dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier(group=self.group)

    def keep(self, *objs) -> None:
        self._keep.extend(objs)

    def close(self) -> None:
        """Unmap every peer allocation. Collective: no rank frees what it
        exported before every peer has unmapped it."""
        torch.cuda.synchronize()
        self.barrier()
        for base in self._opened:
            _ext.call_hip("cme_ipc_close", base)
        self._opened.clear()
        self.barrier()
        self._keep.clear()
