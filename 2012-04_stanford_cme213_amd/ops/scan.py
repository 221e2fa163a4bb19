"""Scan / reduction / segmented-scan ops.

* :func:`scan` -- single-pass decoupled look-back (default) or the lecture's
  multi-level scan-then-add with a Blelloch or Hillis-Steele block algorithm
  (``slides/Lecture16.pdf``; ``my-refs/scan.pdf`` Fig. 5).
* :func:`reduce` -- sum / max / min; the lecture's shared-memory tree
  (``slides/Lecture05.pdf`` 15-16) as ``algo="tree"``.
* :func:`segmented_scan` -- inclusive, head-flag segmented scan (Lecture21;
  nvr-2008-003), optionally fused with an element-wise multiply: the final
  project's ``a *= x[k]; b = segscan(a)`` step (``hw/hw_final/programming/
  fp.cu:168-185``) in one pass.

CPU tensors use the OpenMP oracles in ``csrc/cpu/scan_cpu.cpp``.
"""
from __future__ import annotations

import torch

from .. import _ext

_ext.proto(_ext.HIP_PROTOS, "cme_scan", "ppqiipup")
_ext.proto(_ext.HIP_PROTOS, "cme_scan_rts", "ppqiipp")
_ext.proto(_ext.HIP_PROTOS, "cme_scan_mlevel", "ppqiiipp")
_ext.proto(_ext.HIP_PROTOS, "cme_scan_tree", "ppqiiipp")
_ext.proto(_ext.HIP_PROTOS, "cme_reduce", "pqiiippp")
_ext.proto(_ext.HIP_PROTOS, "cme_segscan", "ppppiqpup")
_ext.proto(_ext.HIP_PROTOS, "cme_spmv_scan_run", "pppqipp")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_scan", "ppqii")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_reduce", "pqiip")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_segscan", "ppppiq")

_DT = {torch.float32: 0, torch.int32: 1}
_DT_SCAN = {torch.float32: 0, torch.int32: 1, torch.uint32: 2}
_OPS = {"sum": 0, "max": 1, "min": 2}
TILE = 4096

_ws_cache: dict = {}


def workspace(device: torch.device, nbytes: int, key: str = "lookback") -> torch.Tensor:
    """Per-device scratch, grown on demand (never allocated inside a launch)."""
    k = (key, device.index)
    t = _ws_cache.get(k)
    if t is None or t.numel() < nbytes:
        t = torch.empty(max(nbytes, 1 << 16), dtype=torch.uint8, device=device)
        _ws_cache[k] = t
    return t


_epochs: dict = {}
_EPOCH_LIMIT = 1 << 24  # lookback.h: status word = (epoch << 8) | bits, 32 bits


def _lookback_ws(x: torch.Tensor) -> tuple[torch.Tensor, int]:
    """Descriptor array of a look-back launch and the epoch to run it with.
    Keyed by (device, STREAM): two scans enqueued on different streams must
    not overwrite each other's descriptors. The array is zeroed once when it
    is (re)allocated; every launch then gets the next epoch, so stale
    descriptors of earlier launches never match and no per-launch memset is
    needed. Under stream capture the epoch is 0 (the native side zeroes the
    array inside the graph), because a replayed graph repeats its arguments."""
    tiles = (x.numel() + TILE - 1) // TILE  # >= the launch's tile count (its tiles are >= TILE elements)
    nbytes = 16 * tiles + 16 * (tiles // 64 + 1) + 64  # lookback.h lb2_ws_bytes (>= the one-level layout)
    k = (f"lookback:{_ext.stream_ptr(x.device)}", x.device.index)
    t = _ws_cache.get(k)
    if t is None or t.numel() < nbytes:
        t = torch.zeros(max(nbytes, 1 << 16), dtype=torch.uint8, device=x.device)
        _ws_cache[k] = t
        _epochs[k] = 0
    if torch.cuda.is_current_stream_capturing():
        # the graph zeroes the array at replay and writes epoch-0 words, which
        # later epochs (>= 1) ignore; the count is NOT restarted: before a
        # replay, words of the earlier epochs are still there
        return t, 0
    e = _epochs[k] + 1
    if e >= _EPOCH_LIMIT:
        t.zero_()
        e = 1
    _epochs[k] = e
    return t, e


def _run_ws(x: torch.Tensor) -> torch.Tensor:
    """Descriptors for launches that zero them natively and number their own
    epochs (spmv_scan_run, tuning arms): kept apart from :func:`_lookback_ws`,
    whose epoch count their words would otherwise collide with."""
    import ctypes

    nbytes = ctypes.c_longlong(0)
    _ext.call_hip("cme_spmv_scan_ws_bytes", x.numel(), ctypes.addressof(nbytes))
    return workspace(x.device, nbytes.value, f"lookback-run:{_ext.stream_ptr(x.device)}")


_ext.proto(_ext.HIP_PROTOS, "cme_spmv_scan_ws_bytes", "qp")
_ext.proto(_ext.HIP_PROTOS, "cme_lookback_timeout_word", "p")
_timeout_words: dict = {}


def _tw(device: torch.device | str | None = None):
    """The look-back give-up word of ``device`` (default: the current one):
    pinned host memory the kernels store to (lookback.h), one word per
    device, readable without a device synchronisation."""
    import ctypes

    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    w = _timeout_words.get(idx)
    if w is None:
        p = ctypes.c_void_p()
        with torch.cuda.device(idx):
            _ext.call_hip("cme_lookback_timeout_word", ctypes.addressof(p))
        w = ctypes.c_uint.from_address(p.value)
        _timeout_words[idx] = w
    return w


def lookback_timed_out(device: torch.device | str = "cuda") -> bool:
    """True if a look-back launch on ``device`` (since the last check) hit its
    bounded-spin limit -- its result is wrong. Synchronises the device."""
    torch.cuda.synchronize(torch.device(device))
    return _tw(device).value != 0


def check_lookback(device: torch.device | str = "cuda") -> None:
    """Synchronise and raise if any look-back launch gave up (then clear)."""
    if lookback_timed_out(device):
        _tw(device).value = 0
        raise RuntimeError("look-back scan spin limit exceeded: a result since the last check is invalid")


def _check_lookback(x: torch.Tensor, before: bool = False) -> None:
    """Called around every look-back launch. Before one: the give-up word of
    EARLIER launches is read without a sync (it is sticky host memory) and
    raised. After one: only under CME_SYNC_CHECK (which synchronises)."""
    w = _tw(x.device)
    if before:
        if w.value != 0:
            w.value = 0
            raise RuntimeError("an earlier look-back scan hit its spin limit (its result was invalid)")
    elif _ext.SYNC_CHECK:
        check_lookback(x.device)


def scan(x: torch.Tensor, exclusive: bool = False, out: torch.Tensor | None = None,
         algo: str = "auto") -> torch.Tensor:
    """Prefix sum of a 1-D contiguous float32/int32/uint32 tensor.
    algo: "auto" ("lookback" for integers, whose sums are exact in any order;
    "rts" for float32, whose fixed summation tree is bitwise reproducible --
    look-back's float prefixes depend on which predecessor had published its
    inclusive value), "lookback" (single pass), "rts" (reduce-then-scan with DPP wave
    scans, deterministic), "blelloch" / "hillis" (reduce-then-scan whose block
    level is the lecture's LDS tree algorithm), "blelloch_mlevel" /
    "hillis_mlevel" (the recursive scan-then-add of my-refs/scan.pdf Fig. 5)."""
    if not x.is_contiguous():
        x = x.contiguous()
    out = torch.empty_like(x) if out is None else out
    n = x.numel()
    if algo == "auto":
        algo = "rts" if x.dtype == torch.float32 else "lookback"
    if x.is_cuda:
        s = _ext.stream_ptr(x.device)
        if algo == "lookback":
            _check_lookback(x, before=True)
            ws, epoch = _lookback_ws(x)
            _ext.call_hip("cme_scan", x.data_ptr(), out.data_ptr(), n, _DT_SCAN[x.dtype], int(exclusive),
                          ws.data_ptr(), epoch, s)
            _check_lookback(x)
        elif algo == "rts":
            _ext.call_hip("cme_scan_rts", x.data_ptr(), out.data_ptr(), n, _DT_SCAN[x.dtype], int(exclusive),
                          workspace(x.device, 8192, "rts").data_ptr(), s)
        elif algo in ("blelloch", "hillis"):
            # one 4-B sum / prefix per 4096-element tile
            ws = workspace(x.device, 4 * ((n + 4095) // 4096) + 256, "tree")
            _ext.call_hip("cme_scan_tree", x.data_ptr(), out.data_ptr(), n, _DT_SCAN[x.dtype],
                          0 if algo == "blelloch" else 1, int(exclusive), ws.data_ptr(), s)
        elif algo in ("blelloch_mlevel", "hillis_mlevel"):
            if out.data_ptr() == x.data_ptr() and not exclusive:
                raise ValueError("in-place inclusive multi-level scan is not supported")
            levels, b = 0, (n + 511) // 512
            while b > 1:
                levels += b
                b = (b + 511) // 512
            ws = workspace(x.device, (levels + 1) * 4, "mlevel")
            _ext.call_hip("cme_scan_mlevel", x.data_ptr(), out.data_ptr(), n, _DT[x.dtype],
                          0 if algo == "blelloch_mlevel" else 1, int(exclusive), ws.data_ptr(), s)
        else:
            raise ValueError(f"unknown scan algo {algo!r}")
    else:
        _ext.call_cpu("cme_cpu_scan", x.data_ptr(), out.data_ptr(), n, _DT_SCAN[x.dtype], int(exclusive))
    return out


def reduce(x: torch.Tensor, op: str = "sum", algo: str = "vector") -> torch.Tensor:
    """Full reduction of a float32/int32 tensor; returns a 0-d tensor on x's device."""
    x = x.contiguous()
    out = torch.empty((), dtype=x.dtype, device=x.device)
    if x.is_cuda:
        part = workspace(x.device, 2048 * 4, "reduce")
        _ext.call_hip("cme_reduce", x.data_ptr(), x.numel(), _DT[x.dtype], _OPS[op], 0 if algo == "vector" else 1,
                      part.data_ptr(), out.data_ptr(), _ext.stream_ptr(x.device))
    else:
        _ext.call_cpu("cme_cpu_reduce", x.data_ptr(), x.numel(), _DT[x.dtype], _OPS[op], out.data_ptr())
    return out


def head_flags_from_offsets(s: torch.Tensor, n: int, device=None, bitmask: bool = True) -> torch.Tensor:
    """Segment heads from the final project's offset array ``s`` (s[0] = 0,
    s[p-1] = n, strictly increasing; segment i = [s[i-1], s[i])). Returns a
    bitmask (int32 words, bit i%32 of word i/32) or a uint8 per element."""
    heads = s[:-1].to(torch.int64)
    if bitmask:
        words = torch.zeros((n + 31) // 32, dtype=torch.int64)
        w = heads // 32
        bit = torch.ones_like(heads) << (heads % 32)
        words.index_add_(0, w, bit)  # heads are distinct: add == or
        words = torch.where(words >= 2**31, words - 2**32, words).to(torch.int32)
        return words.to(device) if device is not None else words
    f = torch.zeros(n, dtype=torch.uint8)
    f[heads] = 1
    return f.to(device) if device is not None else f


def segmented_scan(x: torch.Tensor, flags: torch.Tensor, out: torch.Tensor | None = None,
                   mul: torch.Tensor | None = None) -> torch.Tensor:
    """Inclusive segmented sum scan of float32 ``x`` (optionally ``x*mul``).
    ``flags``: uint8 per element (0/1) or int32 bitmask words."""
    out = torch.empty_like(x) if out is None else out
    n = x.numel()
    mode = 0 if flags.dtype == torch.uint8 else 1
    mp = mul.data_ptr() if mul is not None else None
    if x.is_cuda:
        _check_lookback(x, before=True)
        ws, epoch = _lookback_ws(x)
        _ext.call_hip("cme_segscan", x.data_ptr(), mp, out.data_ptr(), flags.data_ptr(), mode, n, ws.data_ptr(),
                      epoch, _ext.stream_ptr(x.device))
        _check_lookback(x)
    else:
        _ext.call_cpu("cme_cpu_segscan", x.data_ptr(), mp, out.data_ptr(), flags.data_ptr(), mode, n)
    return out


def spmv_scan_run(a: torch.Tensor, xx: torch.Tensor, flags: torch.Tensor, iters: int) -> torch.Tensor:
    """``iters`` in-place steps ``a <- segscan(a * xx)`` (bitmask heads): one
    descriptor memset + one kernel per step, no host synchronisation."""
    if not a.is_cuda:
        for _ in range(iters):
            segmented_scan(a, flags, out=a, mul=xx)
        return a
    assert flags.dtype == torch.int32, "bitmask flags expected"
    _check_lookback(a, before=True)
    _ext.call_hip("cme_spmv_scan_run", a.data_ptr(), xx.data_ptr(), flags.data_ptr(), a.numel(), iters,
                  _run_ws(a).data_ptr(), _ext.stream_ptr(a.device))
    _check_lookback(a)
    return a
