"""Streaming element-wise ops: Caesar shift cipher (1/4/8/16 B per lane),
16-B copy (HBM calibration) and in-place multiply.

Parity: ``shift_cypher`` / ``shift_cypher_int`` / ``shift_cypher_int2`` and the
Thrust ``transform`` variant (``hw/hw1/programming/cipher.cu:64-92``,
``hw/hw1/solution/cipher_solution.cu:234-245``).
"""
from __future__ import annotations

import torch

from .. import _ext

_ext.proto(_ext.HIP_PROTOS, "cme_shift_cipher", "ppqiiip")
_ext.proto(_ext.HIP_PROTOS, "cme_copy_bytes", "ppqp")
_ext.proto(_ext.HIP_PROTOS, "cme_mul_f32", "ppqp")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_shift_cipher", "ppqi")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_mul_f32", "ppq")

WIDTHS = {"char": 1, "uint": 4, "uint2": 8, "uint4": 16, 1: 1, 4: 4, 8: 8, 16: 16}


def shift_cipher(x: torch.Tensor, shift: int, out: torch.Tensor | None = None, width="uint4",
                 block: int = 256) -> torch.Tensor:
    """out[i] = (x[i] + shift) mod 256 over a uint8 tensor."""
    if x.dtype != torch.uint8 or not x.is_contiguous():
        raise TypeError("shift_cipher expects a contiguous uint8 tensor")
    out = torch.empty_like(x) if out is None else out
    n = x.numel()
    if x.is_cuda:
        w = WIDTHS[width]
        if (x.data_ptr() % w) or (out.data_ptr() % w):
            w = 1
        _ext.call_hip("cme_shift_cipher", x.data_ptr(), out.data_ptr(), n, int(shift), w, block,
                      _ext.stream_ptr(x.device))
    else:
        _ext.call_cpu("cme_cpu_shift_cipher", x.data_ptr(), out.data_ptr(), n, int(shift))
    return out


def copy_(dst: torch.Tensor, src: torch.Tensor) -> torch.Tensor:
    """Byte copy with 16-B lanes, non-temporal (HBM bandwidth calibration)."""
    nb = src.numel() * src.element_size()
    assert dst.numel() * dst.element_size() == nb and src.is_cuda and dst.is_cuda
    _ext.call_hip("cme_copy_bytes", src.data_ptr(), dst.data_ptr(), nb, _ext.stream_ptr(src.device))
    return dst


def mul_(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a *= b (float32, same shape)."""
    assert a.dtype == b.dtype == torch.float32 and a.numel() == b.numel()
    if a.is_cuda:
        _ext.call_hip("cme_mul_f32", a.data_ptr(), b.data_ptr(), a.numel(), _ext.stream_ptr(a.device))
    else:
        _ext.call_cpu("cme_cpu_mul_f32", a.data_ptr(), b.data_ptr(), a.numel())
    return a
