"""Atomics demos from the lectures: Monte-Carlo pi with a hierarchical
reduction (Lecture05), hierarchical global max and an atomic work queue
(Lecture21). Histograms live in :mod:`.text`."""
from __future__ import annotations

import struct

import numpy as np
import torch

from .. import _ext

_ext.proto(_ext.HIP_PROTOS, "cme_monte_carlo_pi", "qQpp")
_ext.proto(_ext.HIP_PROTOS, "cme_global_max", "pqpp")
_ext.proto(_ext.HIP_PROTOS, "cme_workqueue_segment_sums", "pipppp")


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def monte_carlo_pi(samples: int, seed: int = 1, device="cuda") -> tuple[float, int]:
    """Estimate pi from `samples` points; returns (pi_estimate, hits). The CPU
    path evaluates the SAME counter-based sample stream (bitwise-equal hits)."""
    dev = torch.device(device)
    if dev.type == "cuda":
        hits = torch.empty(1, dtype=torch.int64, device=dev)
        _ext.call_hip("cme_monte_carlo_pi", samples, seed, hits.data_ptr(), _ext.stream_ptr(dev))
        h = int(hits.item())
    else:
        h = 0
        for b in range(0, samples, 1 << 22):
            i = np.arange(b, min(samples, b + (1 << 22)), dtype=np.uint64)
            with np.errstate(over="ignore"):
                r = _splitmix64(np.uint64(seed) ^ (i * np.uint64(0xD1B54A32D192ED03)))
            x = (r & np.uint64(0xFFFFFFFF)).astype(np.float32) * np.float32(2.3283064365386963e-10)
            y = (r >> np.uint64(32)).astype(np.float32) * np.float32(2.3283064365386963e-10)
            h += int(np.count_nonzero(x * x + y * y <= np.float32(1.0)))
    return 4.0 * h / samples, h


def global_max(x: torch.Tensor) -> float:
    if not x.is_cuda:  # OpenMP reduction (csrc/cpu/scan_cpu.cpp)
        from .scan import reduce as _reduce

        return float(_reduce(x.reshape(-1).contiguous(), "max"))
    out = torch.empty(1, dtype=torch.int32, device=x.device)
    _ext.call_hip("cme_global_max", x.data_ptr(), x.numel(), out.data_ptr(), _ext.stream_ptr(x.device))
    i = int(out.item())
    if i < 0:
        i ^= 0x7FFFFFFF
    return struct.unpack("<f", struct.pack("<i", i))[0]


def segment_sums_workqueue(offsets: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """out[s] = sum(v[offsets[s]:offsets[s+1]]), segments dequeued atomically."""
    nseg = offsets.numel() - 1
    out = torch.empty(nseg, dtype=torch.float32, device=v.device)
    if not v.is_cuda:  # OpenMP segmented reduction (csrc/cpu/algorithms_cpu.cpp)
        from .algorithms import segment_reduce

        return segment_reduce(v.contiguous(), offsets.to(torch.int64), "sum")
    head = torch.empty(1, dtype=torch.int32, device=v.device)
    _ext.call_hip("cme_workqueue_segment_sums", offsets.data_ptr(), nseg, v.data_ptr(), out.data_ptr(),
                  head.data_ptr(), _ext.stream_ptr(v.device))
    return out
