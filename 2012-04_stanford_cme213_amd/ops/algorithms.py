"""Data-parallel algorithms: the Thrust calls of the reference, native on MI355X.

================================  ===========================================
reference (Thrust 1.x)            here
================================  ===========================================
``remove_copy_if`` / ``copy_if``  :func:`copy_if` (``invert=True`` = remove)
``remove_copy`` (value)           :func:`remove_value`
``unique`` (sorted)               :func:`unique`
``stable_partition`` / split      :func:`stable_partition`, :func:`split`
index of set flags                :func:`nonzero`
``lower_bound``/``upper_bound``   :func:`lower_bound`, :func:`upper_bound`
``reduce_by_key`` (sorted keys)   :func:`reduce_by_key`
dense / sparse histogram          :func:`histogram_dense`, :func:`histogram_sparse`
counting sort (Lecture16)         :func:`counting_sort`
``max_element``/``min_element``   :func:`max_element`, :func:`min_element`
``inner_product``                 :func:`inner_product` (``op="mul"|"eq"``)
================================  ===========================================

Call sites in the reference: ``hw/hw3/programming/create_cipher.cu:111-113``
(remove_copy_if), ``hw/hw3/programming/solve_cipher.cu:136-154`` (sort +
upper_bound dense histogram), ``hw/hw3/solution/solve_cipher_solution.cu:
131-200`` (reduce_by_key, sort_by_key, max_element, inner_product); the scan
applications are ``slides/Lecture16.pdf`` 2-19.

GPU tensors run ``csrc/hip/algorithms.hip`` (deterministic reduce-then-scan
compaction, stable); CPU tensors the OpenMP backend
``csrc/cpu/algorithms_cpu.cpp`` (count -> scan -> write, stable). The
``ref_*`` functions are plain-PyTorch oracles, used only by the tests.
"""
from __future__ import annotations

import ctypes
import math

import torch

from .. import _ext
from .sort import sort as _sort

_ext.proto(_ext.HIP_PROTOS, "cme_select", "ppqiiQiipppp")
_ext.proto(_ext.HIP_PROTOS, "cme_search", "pqpqiipp")
_ext.proto(_ext.HIP_PROTOS, "cme_seg_reduce", "ppqiipp")
_ext.proto(_ext.HIP_PROTOS, "cme_arg_reduce", "pqiipppp")
_ext.proto(_ext.HIP_PROTOS, "cme_inner_product", "ppqippp")

_ext.proto(_ext.CPU_PROTOS, "cme_cpu_select", "ppqiiQiipp")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_search", "pqpqiip")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_seg_reduce", "ppqiip")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_arg_reduce", "pqiipp")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_inner_product", "ppqip")

_SEARCH_DT = {torch.float32: 0, torch.int32: 1, torch.uint32: 2, torch.int64: 3, torch.float64: 4}
_RED_DT = {torch.float32: 0, torch.int32: 1, torch.float64: 4}
_RED_DT_CPU = {torch.float32: 0, torch.int32: 1, torch.int64: 3, torch.float64: 4}
_OPS = {"sum": 0, "max": 1, "min": 2}
_PRED = {"flags": 0, "neq": 1, "head": 2}
_TILE = 4096  # kTile in algorithms.hip


# GPU select algorithm for values / indices: "rts" (reduce-then-scan, two
# reads of the input; default, faster at 2^26) or "lookback" (one pass with a
# two-level decoupled look-back; csrc/hip/algorithms.hip select_lookback_kernel)
SELECT_ALGO = "rts"


def _select_ws_bytes(n: int) -> int:  # = cme_select_ws_bytes
    t = (n + _TILE - 1) // _TILE
    return 16 * t + 16 * ((t + 63) // 64) + 4096 + 64


_ws: dict = {}


def _workspace(dev: torch.device, nbytes: int) -> torch.Tensor:
    t = _ws.get(dev.index)
    if t is None or t.numel() < nbytes:
        t = torch.empty(max(nbytes, 1 << 16), dtype=torch.uint8, device=dev)
        _ws[dev.index] = t
    return t


def _esize(x: torch.Tensor) -> int:
    e = x.element_size()
    if e not in (1, 4, 8):
        raise TypeError(f"unsupported element size {e} ({x.dtype})")
    return e


def _bits(x: torch.Tensor, value) -> int:
    """Raw bit pattern of a scalar in x's dtype (predicates compare bitwise)."""
    t = torch.tensor([value], dtype=x.dtype)
    u = {1: torch.uint8, 4: torch.int32, 8: torch.int64}[x.element_size()]
    v = int(t.view(u).item())
    return v & ((1 << (8 * x.element_size())) - 1)


def _select(x: torch.Tensor, flags: torch.Tensor | None, pred: str, value=0, invert: bool = False,
            mode: int = 0) -> tuple[torch.Tensor, int]:
    x = x.contiguous().view(-1)
    n = x.numel()
    if flags is not None:
        flags = flags.contiguous().view(-1)
        if flags.numel() != n:
            raise ValueError("flags must match x")
        flags = flags.view(torch.uint8) if flags.dtype == torch.bool else flags.to(torch.uint8)
    out = torch.empty(n, dtype=torch.int64 if mode == 1 else x.dtype, device=x.device)
    if not x.is_cuda:
        cnt = ctypes.c_longlong(0)
        _ext.call_cpu("cme_cpu_select", x.data_ptr(), flags.data_ptr() if flags is not None else None, n, _esize(x),
                      _PRED[pred], _bits(x, value) if pred == "neq" else 0, int(invert), mode, out.data_ptr(),
                      ctypes.addressof(cnt))
        return out, cnt.value
    from .scan import _check_lookback

    lookback = SELECT_ALGO == "lookback" and mode != 2
    cnt = torch.zeros(1, dtype=torch.int64, device=x.device)
    ws = _workspace(x.device, _select_ws_bytes(n))
    if lookback:
        _check_lookback(x, before=True)
    _ext.call_hip("cme_select", x.data_ptr(), flags.data_ptr() if flags is not None else None, n, _esize(x),
                  _PRED[pred], _bits(x, value) if pred == "neq" else 0, int(invert), mode | (8 if lookback else 0),
                  out.data_ptr(), cnt.data_ptr(), ws.data_ptr(), _ext.stream_ptr(x.device))
    if lookback:
        _check_lookback(x)
    return out, int(cnt.item())


def copy_if(x: torch.Tensor, flags: torch.Tensor, invert: bool = False) -> torch.Tensor:
    """Stable stream compaction: elements whose flag is set (``invert``: not
    set -- ``remove_copy_if``)."""
    out, c = _select(x, flags, "flags", invert=invert)
    return out[:c]


def remove_value(x: torch.Tensor, value) -> torch.Tensor:
    """``thrust::remove_copy``: every element not equal (bitwise) to value."""
    out, c = _select(x, None, "neq", value)
    return out[:c]


def unique(x: torch.Tensor) -> torch.Tensor:
    """First element of every run of equal values (``thrust::unique`` on
    sorted input = dedup via head flags, Lecture16)."""
    out, c = _select(x, None, "head")
    return out[:c]


def run_starts(x: torch.Tensor) -> torch.Tensor:
    """int64 indices where a new run of equal values begins."""
    out, c = _select(x, None, "head", mode=1)
    return out[:c]


def nonzero(flags: torch.Tensor) -> torch.Tensor:
    """int64 indices of the set flags (stable)."""
    out, c = _select(flags.to(torch.uint8) if flags.dtype != torch.bool else flags, flags, "flags", mode=1)
    return out[:c]


def stable_partition(x: torch.Tensor, flags: torch.Tensor) -> tuple[torch.Tensor, int]:
    """Selected elements first, then the rest, both in input order; returns
    (permuted, number selected)."""
    return _select(x, flags, "flags", mode=2)


def split(x: torch.Tensor, flags: torch.Tensor) -> tuple[torch.Tensor, int]:
    """Lecture16 ``split``: flag-0 elements first, then flag-1 (the radix
    sort step); returns (permuted, number of zeros)."""
    return _select(x, flags, "flags", invert=True, mode=2)


def _search(sorted_: torch.Tensor, q: torch.Tensor, upper: bool) -> torch.Tensor:
    if sorted_.dtype != q.dtype:
        raise TypeError("sorted and queries must share a dtype")
    s, qq = sorted_.contiguous().view(-1), q.contiguous().view(-1)
    out = torch.empty(qq.numel(), dtype=torch.int64, device=q.device)
    if not sorted_.is_cuda:
        _ext.call_cpu("cme_cpu_search", s.data_ptr(), s.numel(), qq.data_ptr(), qq.numel(), _SEARCH_DT[s.dtype],
                      int(upper), out.data_ptr())
        return out
    _ext.call_hip("cme_search", s.data_ptr(), s.numel(), qq.data_ptr(), qq.numel(), _SEARCH_DT[s.dtype], int(upper),
                  out.data_ptr(), _ext.stream_ptr(q.device))
    return out


def lower_bound(sorted_: torch.Tensor, q: torch.Tensor) -> torch.Tensor:
    """First index i with sorted[i] >= q, per query (vectorised)."""
    return _search(sorted_, q, False)


def upper_bound(sorted_: torch.Tensor, q: torch.Tensor) -> torch.Tensor:
    """First index i with sorted[i] > q, per query (vectorised)."""
    return _search(sorted_, q, True)


def segment_reduce(vals: torch.Tensor, offsets: torch.Tensor, op: str = "sum") -> torch.Tensor:
    """out[s] = op(vals[offsets[s]:offsets[s+1]]); offsets int64 (nseg + 1).
    Empty segments give the op's identity."""
    nseg = offsets.numel() - 1
    if not vals.is_cuda:
        v = vals.contiguous().view(-1)
        off = offsets.to(torch.int64).contiguous()
        out = torch.empty(nseg, dtype=v.dtype)
        _ext.call_cpu("cme_cpu_seg_reduce", v.data_ptr(), off.data_ptr(), nseg, _RED_DT_CPU[v.dtype], _OPS[op],
                      out.data_ptr())
        return out
    v = vals.contiguous().view(-1)
    off = offsets.to(torch.int64).contiguous()
    out = torch.empty(nseg, dtype=v.dtype, device=v.device)
    _ext.call_hip("cme_seg_reduce", v.data_ptr(), off.data_ptr(), nseg, _RED_DT[v.dtype], _OPS[op], out.data_ptr(),
                  _ext.stream_ptr(v.device))
    return out


def reduce_by_key(keys: torch.Tensor, vals: torch.Tensor, op: str = "sum") -> tuple[torch.Tensor, torch.Tensor]:
    """Runs of equal consecutive keys -> (unique keys, reduced values)."""
    starts = run_starts(keys)
    offsets = torch.cat([starts, torch.tensor([keys.numel()], dtype=torch.int64, device=starts.device)])
    return keys.reshape(-1)[starts], segment_reduce(vals, offsets, op)


def histogram_dense(sorted_: torch.Tensor, nbins: int) -> torch.Tensor:
    """Counts of values 0..nbins-1 in SORTED integer data, the Thrust idiom
    ``upper_bound(sorted, counting_iterator)`` + ``adjacent_difference``
    (``hw/hw3/programming/solve_cipher.cu:136-154``)."""
    q = torch.arange(nbins, dtype=sorted_.dtype, device=sorted_.device)
    ub = upper_bound(sorted_, q)
    return torch.diff(ub, prepend=torch.zeros(1, dtype=ub.dtype, device=ub.device))


def histogram_sparse(sorted_: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """(distinct values, counts) of sorted data: ``reduce_by_key`` with a
    constant-1 value stream (``solve_cipher_solution.cu:185-200``)."""
    ones = torch.ones(sorted_.numel(), dtype=torch.int32, device=sorted_.device)
    return reduce_by_key(sorted_, ones, "sum")


def counting_sort(keys: torch.Tensor, num_keys: int, values: torch.Tensor | None = None):
    """Stable sort of int32 keys in [0, num_keys): a radix sort restricted to
    ceil(log2(num_keys)) bits (one 8-bit counting pass when num_keys <= 256).
    CPU tensors use a stable torch sort."""
    bits = max(1, math.ceil(math.log2(max(num_keys, 2))))
    kdt = keys.dtype
    if kdt == torch.int64:  # keys < num_keys <= 2^31: sorted as int32
        keys = keys.to(torch.int32)
    if not keys.is_cuda and values is None:  # keys only: carry a dummy payload through the key-value pass
        k = _sort(keys, torch.zeros_like(keys), "radix", key_bits=bits)[0]
        return k.to(kdt)
    res = _sort(keys, values, "radix", key_bits=bits)
    if isinstance(res, tuple):
        return res[0].to(kdt), res[1]
    return res.to(kdt)


def _arg(x: torch.Tensor, is_max: bool) -> tuple[float, int]:
    if x.numel() == 0:
        raise ValueError("empty input")
    xs = x.reshape(-1).contiguous()
    if not x.is_cuda:  # first index on ties, like thrust::max_element
        val = torch.empty(1, dtype=xs.dtype)
        idx = ctypes.c_longlong(0)
        _ext.call_cpu("cme_cpu_arg_reduce", xs.data_ptr(), xs.numel(), _RED_DT_CPU[xs.dtype], int(is_max),
                      val.data_ptr(), ctypes.addressof(idx))
        return val.item(), idx.value
    ov = torch.empty(1, dtype=xs.dtype, device=xs.device)
    oi = torch.empty(1, dtype=torch.int64, device=xs.device)
    ws = _workspace(xs.device, 16 * 2048)
    _ext.call_hip("cme_arg_reduce", xs.data_ptr(), xs.numel(), _RED_DT[xs.dtype], int(is_max), ws.data_ptr(),
                  ov.data_ptr(), oi.data_ptr(), _ext.stream_ptr(xs.device))
    return ov.item(), int(oi.item())


def max_element(x: torch.Tensor) -> tuple[float, int]:
    """(max value, first index of it)."""
    return _arg(x, True)


def min_element(x: torch.Tensor) -> tuple[float, int]:
    """(min value, first index of it)."""
    return _arg(x, False)


def inner_product(a: torch.Tensor, b: torch.Tensor, op: str = "mul") -> float:
    """``op="mul"``: sum(a*b) of fp32 data with fp64 accumulation;
    ``op="eq"``: number of positions where the 32-bit words are equal (the
    ``inner_product(.., plus, equal_to)`` of the index of coincidence)."""
    if a.shape != b.shape:
        raise ValueError("shape mismatch")
    if a.element_size() != 4:
        raise TypeError("32-bit elements expected")
    if op == "mul" and a.dtype != torch.float32:
        raise TypeError("op='mul' takes float32")
    aa, bb = a.contiguous().view(-1), b.contiguous().view(-1)
    if not a.is_cuda:
        out = ctypes.c_double(0.0)
        _ext.call_cpu("cme_cpu_inner_product", aa.data_ptr(), bb.data_ptr(), aa.numel(), 0 if op == "mul" else 1,
                      ctypes.addressof(out))
        return out.value
    part = _workspace(a.device, 8 * 2048)
    out = torch.empty(1, dtype=torch.float64, device=a.device)
    _ext.call_hip("cme_inner_product", aa.data_ptr(), bb.data_ptr(), aa.numel(), 0 if op == "mul" else 1,
                  part.data_ptr(), out.data_ptr(), _ext.stream_ptr(a.device))
    return float(out.item())


# ------------------------------------------------------------------ oracles
def _ref_mask(x: torch.Tensor, flags, pred: str, value, invert: bool) -> torch.Tensor:
    x = x.reshape(-1)
    if pred == "flags":
        m = flags.reshape(-1) != 0
    elif pred == "neq":
        m = x != value
    else:
        m = torch.ones_like(x, dtype=torch.bool)
        if x.numel() > 1:
            m[1:] = x[1:] != x[:-1]
    return ~m if invert else m


def ref_copy_if(x, flags, invert=False):
    return x.reshape(-1)[_ref_mask(x, flags, "flags", 0, invert)]


def ref_remove_value(x, value):
    return x.reshape(-1)[_ref_mask(x, None, "neq", value, False)]


def ref_unique(x):
    return x.reshape(-1)[_ref_mask(x, None, "head", 0, False)]


def ref_run_starts(x):
    return torch.nonzero(_ref_mask(x, None, "head", 0, False)).view(-1)


def ref_nonzero(flags):
    return torch.nonzero(flags.reshape(-1) != 0).view(-1)


def ref_stable_partition(x, flags):
    m = _ref_mask(x, flags, "flags", 0, False)
    xs = x.reshape(-1)
    return torch.cat([xs[m], xs[~m]]), int(m.sum())


def ref_split(x, flags):
    m = _ref_mask(x, flags, "flags", 0, True)
    xs = x.reshape(-1)
    return torch.cat([xs[m], xs[~m]]), int(m.sum())


def ref_search(sorted_, q, upper):
    if sorted_.dtype == torch.uint32:  # no uint32 searchsorted in torch: widen (order-preserving)
        sorted_, q = sorted_.to(torch.int64), q.to(torch.int64)
    return torch.searchsorted(sorted_.reshape(-1), q.reshape(-1), right=upper)


def ref_segment_reduce(vals, offsets, op="sum"):
    nseg = offsets.numel() - 1
    out = torch.empty(nseg, dtype=vals.dtype)
    lens = (offsets[1:] - offsets[:-1]).tolist()
    for i, part in enumerate(torch.split(vals.reshape(-1)[int(offsets[0]):int(offsets[-1])], lens)):
        if part.numel() == 0:
            out[i] = {"sum": 0, "max": -math.inf if vals.is_floating_point() else torch.iinfo(vals.dtype).min,
                      "min": math.inf if vals.is_floating_point() else torch.iinfo(vals.dtype).max}[op]
        else:
            out[i] = {"sum": part.sum, "max": part.max, "min": part.min}[op]()
    return out


def ref_arg(x, is_max):
    xs = x.reshape(-1)
    v = xs.max() if is_max else xs.min()
    return v.item(), int(torch.nonzero(xs == v)[0])


def ref_inner_product(a, b, op="mul"):
    if op == "mul":
        return float((a.double() * b.double()).sum())
    return float((a == b).sum())
