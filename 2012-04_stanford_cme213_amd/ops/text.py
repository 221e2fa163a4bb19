"""Histograms and text kernels (hw3 Vigenere; Lecture12/21 histograms).

GPU tensors run the HIP kernels in ``csrc/hip/text.hip``; CPU tensors the
OpenMP backend in ``csrc/cpu/text_cpu.cpp`` (per-thread privatised
histograms, count-scan-write compaction). The ``ref_*`` functions are plain
numpy oracles, used only by the tests.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from .. import _ext

_ext.proto(_ext.HIP_PROTOS, "cme_histogram_u8", "pqiipp")
_ext.proto(_ext.HIP_PROTOS, "cme_digraphs", "pqpp")
_ext.proto(_ext.HIP_PROTOS, "cme_residue_hist", "pqipp")
_ext.proto(_ext.HIP_PROTOS, "cme_match_count", "pqiipp")
_ext.proto(_ext.HIP_PROTOS, "cme_sanitize", "pqpppp")
_ext.proto(_ext.HIP_PROTOS, "cme_vigenere", "pqpiipp")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_histogram_u8", "pqiip")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_digraphs", "pqp")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_residue_hist", "pqip")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_match_count", "pqiip")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_sanitize", "pqpp")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_vigenere", "pqpiip")


def _bytes(x: torch.Tensor) -> torch.Tensor:
    if x.dtype != torch.uint8:
        raise TypeError("uint8 text expected")
    return x.contiguous().view(-1)


def histogram_u8(x: torch.Tensor, lo: int = 0, nbins: int = 256) -> torch.Tensor:
    """Counts of byte values lo..lo+nbins-1 (int32)."""
    x = _bytes(x)
    out = torch.empty(nbins, dtype=torch.int32, device=x.device)
    if x.is_cuda:
        _ext.call_hip("cme_histogram_u8", x.data_ptr(), x.numel(), lo, nbins, out.data_ptr(),
                      _ext.stream_ptr(x.device))
    else:
        _ext.call_cpu("cme_cpu_histogram_u8", x.data_ptr(), x.numel(), lo, nbins, out.data_ptr())
    return out


def letter_histogram(text: torch.Tensor) -> torch.Tensor:
    return histogram_u8(text, ord("a"), 26)


def digraph_histogram(text: torch.Tensor) -> torch.Tensor:
    """26x26 counts of the non-overlapping pairs (t[2i], t[2i+1])."""
    text = _bytes(text)
    out = torch.empty(676, dtype=torch.int32, device=text.device)
    if text.is_cuda:
        _ext.call_hip("cme_digraphs", text.data_ptr(), text.numel(), out.data_ptr(), _ext.stream_ptr(text.device))
    else:
        _ext.call_cpu("cme_cpu_digraphs", text.data_ptr(), text.numel(), out.data_ptr())
    return out.view(26, 26)


def residue_histograms(text: torch.Tensor, period: int) -> torch.Tensor:
    """[period, 26] letter counts of text[r::period]."""
    text = _bytes(text)
    out = torch.empty(period * 26, dtype=torch.int32, device=text.device)
    if text.is_cuda:
        _ext.call_hip("cme_residue_hist", text.data_ptr(), text.numel(), period, out.data_ptr(),
                      _ext.stream_ptr(text.device))
    else:
        _ext.call_cpu("cme_cpu_residue_hist", text.data_ptr(), text.numel(), period, out.data_ptr())
    return out.view(period, 26)


def match_counts(text: torch.Tensor, s0: int, ns: int) -> torch.Tensor:
    """counts[k] = #{i : t[i] == t[i + s0 + k]}, k in [0, ns)."""
    text = _bytes(text)
    out = torch.empty(ns, dtype=torch.int64, device=text.device)
    if text.is_cuda:
        _ext.call_hip("cme_match_count", text.data_ptr(), text.numel(), s0, ns, out.data_ptr(),
                      _ext.stream_ptr(text.device))
    else:
        _ext.call_cpu("cme_cpu_match_count", text.data_ptr(), text.numel(), s0, ns, out.data_ptr())
    return out


def sanitize(raw: torch.Tensor) -> torch.Tensor:
    """Lower-case and keep only a-z (stream compaction)."""
    raw = _bytes(raw)
    out = torch.empty_like(raw)
    if raw.is_cuda:
        part = torch.empty(1025, dtype=torch.int32, device=raw.device)
        cnt = torch.empty(1, dtype=torch.int32, device=raw.device)
        _ext.call_hip("cme_sanitize", raw.data_ptr(), raw.numel(), out.data_ptr(), part.data_ptr(), cnt.data_ptr(),
                      _ext.stream_ptr(raw.device))
        return out[:int(cnt.item())]
    cnt = ctypes.c_longlong(0)
    _ext.call_cpu("cme_cpu_sanitize", raw.data_ptr(), raw.numel(), out.data_ptr(), ctypes.addressof(cnt))
    return out[:cnt.value].clone()


def vigenere(text: torch.Tensor, shifts: torch.Tensor, decode: bool = False) -> torch.Tensor:
    """out[i] = a + (t[i] - a +/- shifts[i % period]) mod 26 (lower-case text)."""
    text = _bytes(text)
    period = shifts.numel()
    out = torch.empty_like(text)
    sh = shifts.to(device=text.device, dtype=torch.int32).contiguous()
    if text.is_cuda:
        _ext.call_hip("cme_vigenere", text.data_ptr(), text.numel(), sh.data_ptr(), period, -1 if decode else 1,
                      out.data_ptr(), _ext.stream_ptr(text.device))
    else:
        _ext.call_cpu("cme_cpu_vigenere", text.data_ptr(), text.numel(), sh.data_ptr(), period, -1 if decode else 1,
                      out.data_ptr())
    return out


# ------------------------------------------------------------------ oracles
def ref_histogram_u8(x: torch.Tensor, lo: int = 0, nbins: int = 256) -> torch.Tensor:
    v = x.numpy().astype(np.int64) - lo
    v = v[(v >= 0) & (v < nbins)]
    return torch.from_numpy(np.bincount(v, minlength=nbins).astype(np.int32))


def ref_digraph_histogram(text: torch.Tensor) -> torch.Tensor:
    t = text.numpy().astype(np.int64) - ord("a")
    m = (t.size // 2) * 2
    a, b = t[0:m:2], t[1:m:2]
    ok = (a >= 0) & (a < 26) & (b >= 0) & (b < 26)
    return torch.from_numpy(np.bincount(a[ok] * 26 + b[ok], minlength=676).astype(np.int32)).view(26, 26)


def ref_residue_histograms(text: torch.Tensor, period: int) -> torch.Tensor:
    t = text.numpy().astype(np.int64) - ord("a")
    idx = np.arange(t.size) % period
    ok = (t >= 0) & (t < 26)
    return torch.from_numpy(np.bincount(idx[ok] * 26 + t[ok], minlength=period * 26).astype(np.int32)).view(period, 26)


def ref_match_counts(text: torch.Tensor, s0: int, ns: int) -> torch.Tensor:
    t = text.numpy()
    return torch.tensor([int(np.count_nonzero(t[s:] == t[:t.size - s])) if s < t.size else 0
                         for s in range(s0, s0 + ns)], dtype=torch.int64)


def ref_sanitize(raw: torch.Tensor) -> torch.Tensor:
    t = raw.numpy().copy()
    up = (t >= ord("A")) & (t <= ord("Z"))
    t[up] += 32
    return torch.from_numpy(t[(t >= ord("a")) & (t <= ord("z"))].copy())


def ref_vigenere(text: torch.Tensor, shifts: torch.Tensor, decode: bool = False) -> torch.Tensor:
    period = shifts.numel()
    t = text.numpy().astype(np.int64) - ord("a")
    s = shifts.numpy().astype(np.int64)[np.arange(t.size) % period]
    return torch.from_numpy(((t + (-s if decode else s)) % 26 + ord("a")).astype(np.uint8))
