"""Lecture micro-studies: branch divergence and memory coalescing
(``slides/Lecture04.pdf`` 4-20) and floating-point summation accuracy
(``slides/Lecture11.pdf``, "Reductions and Floating Point").

GPU kernels: ``csrc/hip/studies.hip``; host summation variants:
``csrc/cpu/sum_cpu.cpp``; the GPU tree/vector reductions are
:func:`cme213x.ops.scan.reduce`.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _ext

_ext.proto(_ext.HIP_PROTOS, "cme_divergence", "pqiip")
_ext.proto(_ext.HIP_PROTOS, "cme_strided_copy", "ppqiip")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_sum_f32", "pqip")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_omp_schedule", "qiiiipp")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_omp_sum", "pqiqpp")

OMP_SCHEDULES = {"static": 0, "static_chunk": 1, "dynamic": 2, "guided": 3}

SUM_ALGOS = {"serial": 0, "pairwise": 1, "kahan": 2}


def divergence(out: torch.Tensor, stride: int, work: int = 256) -> torch.Tensor:
    """Each lane runs one of two FMA chains picked by (lane / stride) & 1; the
    chains diverge inside a wave for stride < 64."""
    if not out.is_cuda or out.dtype != torch.float32:
        raise ValueError("float32 cuda output expected")
    _ext.call_hip("cme_divergence", out.data_ptr(), out.numel(), stride, work, _ext.stream_ptr(out.device))
    return out


def divergence_reference(n: int, stride: int, work: int = 256) -> np.ndarray:
    """Host fp32 replay of :func:`divergence` (FMA via fp64 then rounding is
    exact for these small chains only approximately -- use a tolerance)."""
    i = np.arange(n)
    x = ((i & 1023).astype(np.float32) * np.float32(1e-3)).astype(np.float64)
    odd = ((i % 256) // stride) & 1
    a = np.where(odd == 1, 1.0001, 0.9999).astype(np.float32).astype(np.float64)
    b = np.where(odd == 1, 0.5, -0.25)
    for _ in range(work):
        x = (x * a + b).astype(np.float32).astype(np.float64)
    return x.astype(np.float32)


def strided_copy(src: torch.Tensor, n: int, stride: int, offset: int = 0) -> torch.Tensor:
    """out[i] = src[i * stride + offset] for i < n."""
    if (n - 1) * stride + offset >= src.numel():
        raise ValueError("source too small for n / stride / offset")
    out = torch.empty(n, dtype=torch.float32, device=src.device)
    _ext.call_hip("cme_strided_copy", src.data_ptr(), out.data_ptr(), n, stride, offset, _ext.stream_ptr(src.device))
    return out


def sum_f32(x: torch.Tensor, algo: str = "serial") -> float:
    """fp32 host summation: serial left-to-right, pairwise, or Kahan."""
    x = x.detach().to("cpu", torch.float32).contiguous()
    out = np.zeros(1, dtype=np.float32)
    _ext.call_cpu("cme_cpu_sum_f32", x.data_ptr(), x.numel(), SUM_ALGOS[algo], out.ctypes.data)
    return float(out[0])


def summation_study(sizes=(1 << 10, 1 << 14, 1 << 18, 1 << 22, 1 << 24), seed: int = 0,
                    device: str | None = None) -> list[dict]:
    """Relative error vs the fp64 sum for serial / pairwise / Kahan (host, fp32)
    and the GPU wave-tree reduction, on U(0,1) data: serial error grows ~n*eps,
    tree/pairwise ~log(n)*eps, Kahan ~eps."""
    from .scan import reduce

    rows = []
    g = torch.Generator().manual_seed(seed)
    for n in sizes:
        x = torch.rand(n, generator=g, dtype=torch.float32)
        exact = float(x.double().sum())
        row = {"n": n}
        for a in SUM_ALGOS:
            row[a] = abs(sum_f32(x, a) - exact) / exact
        if device is not None:
            xd = x.to(device)
            for algo in ("vector", "tree"):
                row[f"gpu_{algo}"] = abs(float(reduce(xd, "sum", algo)) - exact) / exact
        rows.append(row)
    return rows


def omp_schedule_study(n: int = 200_000, work: int = 200, chunk: int = 64, threads: int = 0) -> list[dict]:
    """OpenMP loop schedules on a triangular (imbalanced) iteration space
    (slides/Lecture14-15): static blocks leave the last thread with the most
    work; cyclic chunks, dynamic and guided rebalance."""
    rows = []
    for name, code in OMP_SCHEDULES.items():
        sec = np.zeros(1)
        chk = np.zeros(1)
        _ext.call_cpu("cme_cpu_omp_schedule", n, work, code, chunk, threads, sec.ctypes.data, chk.ctypes.data)
        rows.append({"schedule": name, "chunk": chunk if code else None, "seconds": float(sec[0]),
                     "checksum": float(chk[0])})
    return rows


def omp_sum(x: np.ndarray, mode: str = "for", cutoff: int = 1 << 16) -> tuple[float, float]:
    """(sum, seconds) of a float64 array by a parallel-for reduction
    (``mode="for"``) or recursive OpenMP tasks (``mode="task"``)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.zeros(1)
    sec = np.zeros(1)
    _ext.call_cpu("cme_cpu_omp_sum", x.ctypes.data, x.size, 0 if mode == "for" else 1, cutoff, out.ctypes.data,
                  sec.ctypes.data)
    return float(out[0]), float(sec[0])
