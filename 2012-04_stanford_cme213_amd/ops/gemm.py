"""SGEMM ladder (Lecture09): naive / LDS-tiled VALU / MFMA f32 matrix cores.
Reference numbers (GTX 480): naive ~80, tiled 235.9, CUBLAS 784.6 GFLOP/s.
GEMV (fp32/fp64) for the distributed dense matvecs of Lecture20."""
from __future__ import annotations

import torch

from .. import _ext

_ext.proto(_ext.HIP_PROTOS, "cme_sgemm", "iiifppfpip")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_sgemm", "iiifppfp")
_ext.proto(_ext.HIP_PROTOS, "cme_gemv", "iidppdpip")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_gemv", "iidppdpi")

VARIANTS = {"naive": 0, "lds": 1, "mfma": 2}


def sgemm(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor | None = None, alpha: float = 1.0, beta: float = 0.0,
          variant: str = "mfma") -> torch.Tensor:
    if A.dtype != torch.float32 or B.dtype != torch.float32:
        raise TypeError("sgemm is fp32")
    A, B = A.contiguous(), B.contiguous()
    M, K = A.shape
    K2, N = B.shape
    if K != K2:
        raise ValueError("inner dimensions differ")
    if C is None:
        C = torch.zeros(M, N, dtype=torch.float32, device=A.device)
    if A.is_cuda:
        _ext.call_hip("cme_sgemm", M, N, K, float(alpha), A.data_ptr(), B.data_ptr(), float(beta), C.data_ptr(),
                      VARIANTS[variant], _ext.stream_ptr(A.device))
    else:
        _ext.call_cpu("cme_cpu_sgemm", M, N, K, float(alpha), A.data_ptr(), B.data_ptr(), float(beta), C.data_ptr())
    return C


_GEMV_DT = {torch.float32: 0, torch.float64: 4}


def gemv(A: torch.Tensor, x: torch.Tensor, y: torch.Tensor | None = None, alpha: float = 1.0,
         beta: float = 0.0) -> torch.Tensor:
    """y = alpha*A x + beta*y for a row-major A [M, K] (fp32 or fp64):
    ``cme_gemv`` (HBM-streaming HIP kernel, ``csrc/hip/gemm.hip``) on the GPU,
    ``cme_cpu_gemv`` (OpenMP) on the CPU."""
    if A.dim() != 2 or x.dim() != 1 or A.shape[1] != x.numel():
        raise ValueError(f"gemv shapes {tuple(A.shape)} x {tuple(x.shape)}")
    if A.dtype not in _GEMV_DT or x.dtype != A.dtype:
        raise TypeError("gemv is fp32 or fp64 with matching x")
    A, x = A.contiguous(), x.contiguous()
    M, K = A.shape
    if y is None:
        y = torch.empty(M, dtype=A.dtype, device=A.device)
        beta = 0.0
    elif y.numel() != M or y.dtype != A.dtype or not y.is_contiguous():
        raise ValueError("gemv output must be a contiguous [M] tensor of A's dtype")
    if A.is_cuda:
        _ext.call_hip("cme_gemv", M, K, float(alpha), A.data_ptr(), x.data_ptr(), float(beta), y.data_ptr(),
                      _GEMV_DT[A.dtype], _ext.stream_ptr(A.device))
    else:
        _ext.call_cpu("cme_cpu_gemv", M, K, float(alpha), A.data_ptr(), x.data_ptr(), float(beta), y.data_ptr(),
                      _GEMV_DT[A.dtype])
    return y
