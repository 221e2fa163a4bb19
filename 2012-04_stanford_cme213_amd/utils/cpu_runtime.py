"""Thread policy of the OpenMP CPU backend (``csrc/cpu/runtime_cpu.cpp``):
the team size every CPU entry point uses (the reference's ``OMP_NUM_THREADS``
sweep, ``hw/hw4/programming/pa4.pbs:21-29``) and the wait policy the OpenMP
runtime was started with.

The wait policy is read once, when the runtime loads (torch loads it first);
:func:`passive_env` is the environment to start a process with so its
parallel regions sleep instead of spinning (see ``profiles/omp_floor_r6.md``).
"""
from __future__ import annotations

import ctypes
import os

from .. import _ext

_ext.proto(_ext.CPU_PROTOS, "cme_cpu_runtime_info", "ppp")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_set_threads", "i")


def info() -> dict:
    """{"threads": team size, "procs": processors seen, "wait_policy": ...}"""
    t, p = ctypes.c_int(0), ctypes.c_int(0)
    buf = ctypes.create_string_buffer(16)
    _ext.call_cpu("cme_cpu_runtime_info", ctypes.addressof(t), ctypes.addressof(p), ctypes.addressof(buf))
    return {"threads": t.value, "procs": p.value, "wait_policy": buf.value.decode()}


def set_threads(n: int) -> None:
    """Team size of every later parallel region of the CPU backend."""
    _ext.call_cpu("cme_cpu_set_threads", int(n))


def passive_env(env: dict | None = None) -> dict:
    """A copy of ``env`` (default: this process's) with OMP_WAIT_POLICY=PASSIVE
    unless the caller chose a policy: for launching a CPU-backend process."""
    e = dict(os.environ if env is None else env)
    if "OMP_WAIT_POLICY" not in e and "GOMP_SPINCOUNT" not in e:
        e["OMP_WAIT_POLICY"] = "PASSIVE"
    return e
