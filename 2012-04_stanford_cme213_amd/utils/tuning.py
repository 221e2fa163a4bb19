"""Run-time tuning knobs of the native library (``csrc/include/cme213/
tuning.h``): arm selection, chunk heights, spin bounds, rehearsal delays.

Each knob starts from its ``CME_*`` environment variable (or the measured
default) and can be changed in-process, so tests and sweeps pick an arm
without spawning a process per setting::

    from cme213x.utils import tuning
    with tuning.override(radix_ds=1, pipe_vw=4):
        ...
    tuning.get("dist_schedule")        # -> 2
    tuning.names()                     # every knob

Names are the environment variables without ``CME_``, lower-cased.
"""
from __future__ import annotations

import contextlib
import ctypes

from .. import _ext

_ext.proto(_ext.HIP_PROTOS, "cme_tune_set", "sq")
_ext.proto(_ext.HIP_PROTOS, "cme_tune_reset", "s")
_ext.proto(_ext.HIP_PROTOS, "cme_tune_get", "spp")
_ext.proto(_ext.HIP_PROTOS, "cme_tune_name", "ipi")


def get(name: str) -> int:
    v, is_set = ctypes.c_longlong(0), ctypes.c_int(0)
    _ext.call_hip("cme_tune_get", name.encode(), ctypes.addressof(v), ctypes.addressof(is_set))
    return int(v.value)


def is_set(name: str) -> bool:
    v, s = ctypes.c_longlong(0), ctypes.c_int(0)
    _ext.call_hip("cme_tune_get", name.encode(), ctypes.addressof(v), ctypes.addressof(s))
    return bool(s.value)


def set(name: str, value: int) -> None:  # noqa: A001 - the knob API reads best as tuning.set
    _ext.call_hip("cme_tune_set", name.encode(), int(value))


def reset(name: str) -> None:
    """Back to the environment variable / default."""
    _ext.call_hip("cme_tune_reset", name.encode())


def names() -> list[str]:
    n = _ext.hip().cme_tune_count()
    out = []
    for i in range(n):
        buf = ctypes.create_string_buffer(64)
        _ext.call_hip("cme_tune_name", i, ctypes.addressof(buf), 64)
        out.append(buf.value.decode())
    return out


@contextlib.contextmanager
def override(**knobs):
    """Set knobs for the duration of a ``with`` block, then restore each to
    what it was (a value set before, or its environment default)."""
    prev = {k: (get(k), is_set(k)) for k in knobs}
    try:
        for k, v in knobs.items():
            set(k, v)
        yield
    finally:
        for k, (v, was) in prev.items():
            if was:
                set(k, v)
            else:
                reset(k)
