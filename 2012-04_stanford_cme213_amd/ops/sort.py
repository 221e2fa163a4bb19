"""Sorting: GPU LSD radix sort (8-bit digits, stable, key-value), GPU
merge-path merge sort, and the hw4 OpenMP radix / merge sorts.

Keys: uint32 natively; int32 and float32 are mapped to order-preserving
uint32 codes (sign-bit flip / IEEE total-order trick) and back -- inside the
onesweep kernels (first pass loads, last pass stores), elsewhere by tensor ops.

GPU radix algorithms: "radix" = reduce-then-scan (``csrc/hip/sort.hip``:
upsweep + one-launch count scan + downsweep per 8-bit digit), "onesweep"
(``csrc/hip/radix.hip``: one histogram read for every pass, then one read +
one write of the keys per digit with decoupled look-back across tiles). Both
are stable and exact; reduce-then-scan is the default because it measures
faster on MI355X (16M keys: profiles/sort_r3.md).
"""
from __future__ import annotations

import torch

from .. import _ext

_ext.proto(_ext.HIP_PROTOS, "cme_radix_sort_u32", "ppppqiipp")
_ext.proto(_ext.HIP_PROTOS, "cme_radix_sort", "ppppppqiiipp")
_ext.proto(_ext.HIP_PROTOS, "cme_radix_onesweep", "ppppppqiiipqp")
_ext.proto(_ext.HIP_PROTOS, "cme_radix_lane_order", "i")
_ext.proto(_ext.HIP_PROTOS, "cme_merge_sort_u32", "ppppqp")
_ext.proto(_ext.HIP_PROTOS, "cme_merge_sort", "ppppppqip")
_ext.proto(_ext.HIP_PROTOS, "cme_merge_sort_ws", "ppppppqipp")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_radix_sort_u32", "ppqii")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_radix_sort_serial_u32", "ppqi")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_merge_sort_i32", "ppqqqp")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_radix_sort_kv_u32", "ppppqii")


def _to_u32(k: torch.Tensor) -> torch.Tensor:
    if k.dtype == torch.uint32:
        return k.clone()
    if k.dtype == torch.int32:
        return (k.view(torch.int32) ^ torch.tensor(-(2 ** 31), dtype=torch.int32, device=k.device)).view(torch.uint32)
    if k.dtype == torch.float32:
        i = k.view(torch.int32)
        mask = torch.where(i < 0, torch.tensor(-1, dtype=torch.int32, device=k.device),
                           torch.tensor(-(2 ** 31), dtype=torch.int32, device=k.device))
        return (i ^ mask).view(torch.uint32)
    raise TypeError(f"unsupported key dtype {k.dtype}")


def _from_u32(u: torch.Tensor, dtype) -> torch.Tensor:
    if dtype == torch.uint32:
        return u
    i = u.view(torch.int32)
    if dtype == torch.int32:
        return i ^ torch.tensor(-(2 ** 31), dtype=torch.int32, device=u.device)
    mask = torch.where(i >= 0, torch.tensor(-1, dtype=torch.int32, device=u.device),
                       torch.tensor(-(2 ** 31), dtype=torch.int32, device=u.device))
    return (i ^ mask).view(torch.float32)


_ws: dict = {}
_os_ws: dict = {}
_os_epochs: dict = {}
_OS_TILE = 8192
_OS_EPOCH_LIMIT = 1 << 27  # radix.hip: granule tag = epoch * 4 + pass, 30 bits
_MODES = {torch.uint32: 0, torch.int32: 1, torch.float32: 2}


def _onesweep_ws(keys: torch.Tensor) -> tuple[torch.Tensor, int]:
    """Workspace + call epoch of a onesweep sort (cf. ops/scan.py
    _lookback_ws): zeroed once when (re)allocated, then every call gets the
    next epoch, so granules of earlier calls never match and no memset runs.
    Keyed by (device, stream); under stream capture a separate workspace with
    epoch 0, which the launcher zeroes inside the graph at every replay."""
    n = keys.numel()
    tiles = (n + _OS_TILE - 1) // _OS_TILE
    nbytes = 2 * 4 * 256 * 4 + tiles * 8 + 2 * tiles * 256 * 8 + 256  # = cme_radix_onesweep_ws_bytes
    capturing = torch.cuda.is_current_stream_capturing()
    k = (f"os:{'cap:' if capturing else ''}{_ext.stream_ptr(keys.device)}", keys.device.index)
    t = _os_ws.get(k)
    if t is None or t.numel() < nbytes:
        t = torch.zeros(max(nbytes, 1 << 16), dtype=torch.uint8, device=keys.device)
        _os_ws[k] = t
        _os_epochs[k] = 0
    if capturing:
        return t, 0
    e = _os_epochs[k] + 1
    if e >= _OS_EPOCH_LIMIT:
        t.zero_()
        e = 1
    _os_epochs[k] = e
    return t, e


def radix_lane_order(check: bool = True) -> bool:
    """Whether the current device resolves the same-address lanes of one
    returning LDS atomic in lane order -- the property the radix downsweep's
    lane-atomic ranks rely on (``csrc/hip/sort.hip`` kRankLanes). ``check``
    runs the library's one-time probe kernel if this device has not been
    checked yet; the radix sort falls back to ballot-match ranks otherwise."""
    return bool(_ext._fn("hip", "cme_radix_lane_order")(1 if check else 0))


def _merge(keys: torch.Tensor, values: torch.Tensor | None):
    """GPU merge sort (csrc/hip/sort.hip cme_merge_sort_ws): stable; 8192-key
    block sorts, then one LDS-staged merge-path pass per doubling of the run
    length; from 8M keys each pass first finds every tile's merge-path split
    in one launch (tuning knob merge_part), below that each merge block
    searches its own; key transforms fused into the first and last kernels.
    Keys-only and key-value tiles are block-sorted by an LDS radix sort
    (tuning knob merge_block_sort). A 4-way pass schedule lives in the tuning
    library (cme_merge_sort4_tune; measured slower: profiles/sort_r6.md)."""
    if keys.dtype not in _MODES:
        raise TypeError(f"unsupported key dtype {keys.dtype}")
    k = keys.contiguous()
    out, tmp = torch.empty_like(k), torch.empty_like(k)
    vp = vo = vt = None
    if values is not None:
        if values.element_size() != 4 or values.numel() != k.numel():
            raise TypeError("values: one 32-bit value per key")
        v = values.contiguous()
        vout, vtmp = torch.empty_like(v), torch.empty_like(v)
        vp, vo, vt = v.data_ptr(), vout.data_ptr(), vtmp.data_ptr()
    ws = _workspace(keys.device, (k.numel() + 4095) // 4096 * 48 + 256)  # = cme_merge_ws_bytes
    _ext.call_hip("cme_merge_sort_ws", k.data_ptr(), out.data_ptr(), tmp.data_ptr(), vp, vo, vt, k.numel(),
                  _MODES[keys.dtype], ws.data_ptr(), _ext.stream_ptr(keys.device))
    return (out, vout) if values is not None else out


def _rts(keys: torch.Tensor, values: torch.Tensor | None, key_bits: int):
    """Reduce-then-scan LSD radix sort (cme_radix_sort): key transforms fused
    into the first and last passes, input untouched."""
    n = keys.numel()
    dtype = keys.dtype
    if dtype not in _MODES:
        raise TypeError(f"unsupported key dtype {dtype}")
    if key_bits < 32 and dtype not in (torch.int32, torch.uint32):
        raise TypeError("key_bits < 32 needs non-negative integer keys")
    mode = 0 if key_bits < 32 else _MODES[dtype]
    bits = 32 if key_bits >= 32 else max(1, int(key_bits))
    k = keys.contiguous()
    out, tmp = torch.empty_like(k), torch.empty_like(k)
    vp = vo = vt = None
    if values is not None:
        if values.element_size() != 4 or values.numel() != n:
            raise TypeError("values: one 32-bit value per key")
        v = values.contiguous()
        vout, vtmp = torch.empty_like(v), torch.empty_like(v)
        vp, vo, vt = v.data_ptr(), vout.data_ptr(), vtmp.data_ptr()
    tiles = (n + 4095) // 4096
    ws = _workspace(keys.device, min(tiles, 4096) * 256 * 4 + 256 * 4 + 256)  # = cme_radix_ws_bytes
    _ext.call_hip("cme_radix_sort", k.data_ptr(), out.data_ptr(), tmp.data_ptr(), vp, vo, vt, n, mode, 0, bits,
                  ws.data_ptr(), _ext.stream_ptr(keys.device))
    return (out, vout) if values is not None else out


def _onesweep(keys: torch.Tensor, values: torch.Tensor | None, key_bits: int):
    from .scan import _check_lookback

    n = keys.numel()
    dtype = keys.dtype
    if dtype not in _MODES:
        raise TypeError(f"unsupported key dtype {dtype}")
    if key_bits < 32 and dtype not in (torch.int32, torch.uint32):
        raise TypeError("key_bits < 32 needs non-negative integer keys")
    mode = 0 if key_bits < 32 else _MODES[dtype]
    bits = 32 if key_bits >= 32 else max(1, int(key_bits))
    k = keys.contiguous()
    out = torch.empty_like(k)
    tmp = torch.empty_like(k)
    vp = vo = vt = None
    if values is not None:
        if values.element_size() != 4 or values.numel() != n:
            raise TypeError("values: one 32-bit value per key")
        v = values.contiguous()
        vout, vtmp = torch.empty_like(v), torch.empty_like(v)
        vp, vo, vt = v.data_ptr(), vout.data_ptr(), vtmp.data_ptr()
    ws, epoch = _onesweep_ws(k)
    _check_lookback(k, before=True)
    _ext.call_hip("cme_radix_onesweep", k.data_ptr(), out.data_ptr(), tmp.data_ptr(), vp, vo, vt, n, mode, 0, bits,
                  ws.data_ptr(), epoch, _ext.stream_ptr(keys.device))
    _check_lookback(k)
    return (out, vout) if values is not None else out


def _workspace(dev: torch.device, nbytes: int) -> torch.Tensor:
    """Scratch of the reduce-then-scan sort (tile counts and totals; every
    call rewrites what it reads). Eager calls share one buffer per (device,
    stream): sorts on different streams never race on it. Under stream
    capture every call gets its own buffer from the graph's private pool, so
    a replay never writes into memory an eager call has since replaced and
    freed."""
    if torch.cuda.is_current_stream_capturing():
        return torch.empty(nbytes, dtype=torch.uint8, device=dev)
    key = (dev.index, _ext.stream_ptr(dev))
    t = _ws.get(key)
    if t is None or t.numel() < nbytes:
        t = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        _ws[key] = t
    return t


def sort(keys: torch.Tensor, values: torch.Tensor | None = None, algo: str = "radix", num_bits: int = 8,
         key_bits: int = 32):
    """Sort a 1-D tensor (optionally carrying int32/uint32/float32 values).
    GPU algos: "radix" (reduce-then-scan, stable; "radix_rts" is an alias),
    "onesweep" (decoupled look-back, stable), "merge" (stable). CPU algos: "radix" (OpenMP,
    ``num_bits`` per pass), "radix_serial", "merge" (OpenMP tasks, keys only).
    ``key_bits`` < 32 (GPU radix, non-negative integer keys below
    ``2**key_bits``) runs only the passes covering those bits -- a counting
    sort when ``key_bits <= 8``. Returns sorted keys (and values)."""
    if keys.dim() != 1:
        raise ValueError("1-D keys expected")
    n = keys.numel()
    dtype = keys.dtype
    if keys.is_cuda and algo in ("radix", "radix_rts", "onesweep"):
        if n <= 1:
            return (keys.clone(), values.clone()) if values is not None else keys.clone()
        if algo == "onesweep":
            return _onesweep(keys, values, key_bits)
        return _rts(keys, values, key_bits)
    if keys.is_cuda and algo == "merge":
        return _merge(keys, values)
    if keys.is_cuda:
        raise ValueError(f"unknown GPU sort algo {algo!r}")
    if values is not None:
        if algo != "radix":
            raise NotImplementedError("CPU key-value sort: algo='radix'")
        if values.element_size() != 4 or values.numel() != n:
            raise TypeError("values: one 32-bit value per key")
        if key_bits < 32 and dtype not in (torch.int32, torch.uint32):
            raise TypeError("key_bits < 32 needs non-negative integer keys")
        k = keys.contiguous().clone().view(torch.uint32) if key_bits < 32 else _to_u32(keys.contiguous())
        v = values.contiguous().clone().view(torch.uint32)
        kt, vt = torch.empty_like(k), torch.empty_like(v)
        _ext.call_cpu("cme_cpu_radix_sort_kv_u32", k.data_ptr(), kt.data_ptr(), v.data_ptr(), vt.data_ptr(), n,
                      num_bits, min(32, max(1, int(key_bits))))
        out = k.view(dtype) if key_bits < 32 else _from_u32(k, dtype)
        return out, v.view(values.dtype)
    if algo == "merge":
        if dtype != torch.int32:
            raise TypeError("CPU merge sort takes int32 keys (the hw4 driver's type)")
        a = keys.clone()
        tmp = torch.empty_like(a)
        st = torch.zeros(1, dtype=torch.int32)
        _ext.call_cpu("cme_cpu_merge_sort_i32", a.data_ptr(), tmp.data_ptr(), n, 2048, 2048, st.data_ptr())
        return a if st.item() == 1 else tmp
    k = _to_u32(keys.contiguous())
    tmp = torch.empty_like(k)
    if algo == "radix":
        _ext.call_cpu("cme_cpu_radix_sort_u32", k.data_ptr(), tmp.data_ptr(), n, num_bits, 0)
    elif algo == "radix_serial":
        _ext.call_cpu("cme_cpu_radix_sort_serial_u32", k.data_ptr(), tmp.data_ptr(), n, num_bits)
    else:
        raise ValueError(algo)
    return _from_u32(k, dtype)


def merge_sort_cpu(keys: torch.Tensor, sort_threshold: int, merge_threshold: int) -> tuple[torch.Tensor, int]:
    """The hw4 driver's merge sort with explicit thresholds; returns (sorted,
    status) where status 1/-1 says which ping-pong buffer held the result."""
    a = keys.clone()
    tmp = torch.empty_like(a)
    st = torch.zeros(1, dtype=torch.int32)
    _ext.call_cpu("cme_cpu_merge_sort_i32", a.data_ptr(), tmp.data_ptr(), a.numel(), sort_threshold,
                  merge_threshold, st.data_ptr())
    return (a if st.item() == 1 else tmp), int(st.item())
