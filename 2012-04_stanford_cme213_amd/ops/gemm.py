"""SGEMM ladder (Lecture09): naive / LDS-tiled VALU / MFMA f32 matrix cores.
Reference numbers (GTX 480): naive ~80, tiled 235.9, CUBLAS 784.6 GFLOP/s."""
from __future__ import annotations

import torch

from .. import _ext

_ext.proto(_ext.HIP_PROTOS, "cme_sgemm", "iiifppfpip")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_sgemm", "iiifppfp")

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
