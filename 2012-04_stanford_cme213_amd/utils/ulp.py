"""ULP-distance float comparison (vectorised).

Same criterion as the reference's ``AlmostEqual2sComplement``
(``hw/hw1/programming/mp1-util.h:44-61``): reinterpret the IEEE bits as a
two's-complement integer, map negatives onto a lexicographically ordered line,
and compare the integer distance with ``max_ulps``.

The reference's double-precision branch (``hw/hw2/programming/mp1-util.h:63-76``)
subtracts ``0x80000000`` from a 64-bit pattern, which is wrong for negative
doubles; here the 64-bit case uses ``0x8000000000000000`` (documented fix).
"""
from __future__ import annotations

import numpy as np


def _ordered_u64(a: np.ndarray) -> np.ndarray:
    """Map IEEE values onto an unsigned line where adjacent floats differ by 1
    and +0 == -0 (the reference's ``0x80000000 - aInt`` remap, then biased)."""
    if a.dtype == np.float32:
        b = a.view(np.int32).astype(np.int64)
        o = np.where(b < 0, np.int64(-(2**31)) - b, b)
        return (o + np.int64(2**31)).astype(np.uint64)
    if a.dtype == np.float64:
        b = a.view(np.int64)
        imin = np.int64(np.iinfo(np.int64).min)
        o = np.where(b < 0, imin - b, b)  # in [INT64_MIN+1, INT64_MAX]: no overflow
        return o.view(np.uint64) ^ np.uint64(1 << 63)
    raise TypeError(f"unsupported dtype {a.dtype}")


def ulp_distance(a, b) -> np.ndarray:
    """Exact element-wise ULP distance (uint64) for float32/float64 arrays."""
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    if a.dtype != b.dtype:
        raise TypeError("dtype mismatch")
    ua, ub = _ordered_u64(a), _ordered_u64(b)
    return np.where(ua > ub, ua - ub, ub - ua)


def almost_equal_ulps(a, b, max_ulps: int = 10) -> np.ndarray:
    """Boolean mask: |a - b| <= max_ulps units in the last place."""
    return ulp_distance(a, b) <= max_ulps


def almost_equal_2s_complement(a: float, b: float, max_ulps: int = 10, dtype=np.float32) -> bool:
    """Scalar form with the reference's name."""
    return bool(almost_equal_ulps(np.asarray([a], dtype), np.asarray([b], dtype), max_ulps)[0])
