"""Matrix transpose ladder (Lecture06/07, Ruetsch & Micikevicius
``my-refs/MatrixTranspose.pdf``): copy / naive / LDS tile / +1 pad / XOR
swizzle / diagonal reorder / XCD remap / 16-B vectorised. CPU: OpenMP blocked.

Effective bandwidth convention (the paper's): 2 x bytes / time.
"""
from __future__ import annotations

import torch

from .. import _ext

_ext.proto(_ext.HIP_PROTOS, "cme_transpose_f32", "ppiiip")
_ext.proto(_ext.HIP_PROTOS, "cme_transpose_reps_f32", "ppiiip")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_transpose_f32", "ppiii")

VARIANTS = {"copy": 0, "naive": 1, "lds": 2, "lds_pad": 3, "lds_swizzle": 4, "diagonal": 5, "xcd": 6, "vec": 7,
            "vec_xcd": 8, "naive_1d": 9}
# the paper's diagnostic kernels (square matrices; NOT transposes):
# "coarse" moves tiles without transposing their elements, "fine" transposes
# elements inside tiles that stay in place
DIAGNOSTICS = {"coarse": 10, "fine": 11}


def transpose(x: torch.Tensor, variant: str = "vec", out: torch.Tensor | None = None) -> torch.Tensor:
    """Transpose a 2-D contiguous float32 tensor (``variant="copy"`` returns a
    same-shape copy -- the bandwidth upper bound)."""
    if x.dim() != 2 or x.dtype != torch.float32:
        raise TypeError("transpose expects a 2-D float32 tensor")
    x = x.contiguous()
    rows, cols = x.shape
    if out is None:
        out = torch.empty((rows, cols) if variant == "copy" else (cols, rows), dtype=x.dtype, device=x.device)
    if x.is_cuda:
        _ext.call_hip("cme_transpose_f32", x.data_ptr(), out.data_ptr(), rows, cols, VARIANTS[variant],
                      _ext.stream_ptr(x.device))
    else:
        if variant == "copy":
            out.copy_(x)
        else:
            _ext.call_cpu("cme_cpu_transpose_f32", x.data_ptr(), out.data_ptr(), rows, cols,
                          0 if variant == "naive" else 1)
    return out


def diagnostic(x: torch.Tensor, kind: str, out: torch.Tensor | None = None) -> torch.Tensor:
    """The paper's coarse-/fine-grained diagnostic kernels (square, GPU):
    ``coarse`` = tiles moved to their transposed position, elements kept in
    tile order; ``fine`` = elements transposed inside tiles kept in place."""
    if x.dim() != 2 or x.shape[0] != x.shape[1] or not x.is_cuda:
        raise ValueError("diagnostics take a square cuda matrix")
    out = torch.empty_like(x) if out is None else out
    _ext.call_hip("cme_transpose_f32", x.data_ptr(), out.data_ptr(), x.shape[0], x.shape[1], DIAGNOSTICS[kind],
                  _ext.stream_ptr(x.device))
    return out


def transpose_reps(x: torch.Tensor, reps: int, out: torch.Tensor | None = None) -> torch.Tensor:
    """lds_pad transpose performed ``reps`` times inside ONE kernel launch --
    the paper's second timing methodology (launch overhead excluded)."""
    if not x.is_cuda:
        raise ValueError("GPU only")
    rows, cols = x.shape
    out = torch.empty((cols, rows), dtype=x.dtype, device=x.device) if out is None else out
    _ext.call_hip("cme_transpose_reps_f32", x.data_ptr(), out.data_ptr(), rows, cols, reps,
                  _ext.stream_ptr(x.device))
    return out
