"""Loader for the in-tree native libraries (ctypes, C ABI).

``libcme213_hip.so`` holds every HIP kernel; ``libcme213_cpu.so`` the OpenMP
backends. Both are built in-tree by :mod:`._build` (``__graft_entry__.build``).

Policy (no silent fallbacks): when a GPU is visible the HIP library MUST load --
any op called on a ``cuda`` tensor raises if it cannot. CPU ops always use the
native OpenMP library; pure-PyTorch code is only ever used as a test oracle.

Every native entry point returns an ``int`` status (``hipError_t`` for HIP
launchers, 0/1 for CPU), checked by :func:`check` -- the replacement for the
reference's ``check_launch`` (``hw/hw1/programming/mp1-util.h:8-18``), minus the
device synchronisation and ``exit(1)``.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

import torch

_LIB_DIR = Path(__file__).resolve().parent / "lib"
_lock = threading.Lock()
_libs: dict[str, ctypes.CDLL] = {}

_CT = {
    "p": ctypes.c_void_p,
    "i": ctypes.c_int,
    "u": ctypes.c_uint,
    "q": ctypes.c_int64,
    "Q": ctypes.c_uint64,
    "f": ctypes.c_float,
    "d": ctypes.c_double,
    "s": ctypes.c_char_p,
}

# name -> argument signature (return type is always int)
HIP_PROTOS: dict[str, str] = {"cme_device_sync": ""}
CPU_PROTOS: dict[str, str] = {}
# entry points of the tuning library (libcme213_tune.so, built with CME_TUNE=1 /
# `make TUNE=1`); call_hip routes these names there
TUNE_PROTOS: dict[str, str] = {}


def proto(table: dict, name: str, sig: str) -> None:
    table[name] = sig


_bound: dict[tuple[str, str], object] = {}


def _fn(kind: str, name: str):
    """Bound native function (argtypes from the proto table, lazily)."""
    key = (kind, name)
    f = _bound.get(key)
    if f is None:
        if kind == "hip" and name in TUNE_PROTOS:
            kind = "tune"
        lib = _load(kind)
        protos = {"hip": HIP_PROTOS, "tune": TUNE_PROTOS}.get(kind, CPU_PROTOS)
        if name not in protos:
            raise KeyError(f"no prototype registered for {kind}:{name}")
        f = getattr(lib, name)
        f.restype = ctypes.c_int
        f.argtypes = [_CT[c] for c in protos[name].replace(" ", "")]
        _bound[key] = f
    return f


def _load(kind: str) -> ctypes.CDLL:
    with _lock:
        return _load_unlocked(kind)


def _load_unlocked(kind: str) -> ctypes.CDLL:
    if kind in _libs:
        return _libs[kind]
    if kind == "tune":
        # its undefined runtime symbols resolve against the HIP library
        _libs.get("hip") or _load_unlocked("hip")
    path = _LIB_DIR / f"libcme213_{kind}.so"
    alt = os.environ.get(f"CME_{kind.upper()}_LIB")  # experiments: an alternative build of the library
    if alt:
        path = Path(alt)
    if not path.exists():
        if os.environ.get("CME_AUTOBUILD", "1") != "0":
            from . import _build

            _build.build(hip=(kind in ("hip", "tune")), cpu=(kind == "cpu"), verbose=True,
                         tune=True if kind == "tune" else None)
        if not path.exists():
            raise RuntimeError(f"cme213x native library missing: {path} (run __graft_entry__.build())")
    # torch is imported first so its bundled libamdhip64.so.7 (same SONAME)
    # is the one our HIP library binds to: one HIP runtime per process.
    lib = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
    if kind == "hip":
        lib.cme_hip_error_string.restype = ctypes.c_char_p
        lib.cme_hip_error_string.argtypes = [ctypes.c_int]
        lib.cme_rccl_error_string.restype = ctypes.c_char_p
        lib.cme_rccl_error_string.argtypes = [ctypes.c_int]
    _libs[kind] = lib
    return lib


def hip() -> ctypes.CDLL:
    return _load("hip")


def cpu() -> ctypes.CDLL:
    return _load("cpu")


def hip_loaded() -> bool:
    return "hip" in _libs


def check(rc: int, what: str, kind: str = "hip") -> None:
    if rc != 0:
        if kind == "hip":
            if rc >= 10000:  # 10000 + ncclResult_t (NCCL_TRY in csrc/hip/dist_heat.hip)
                msg = hip().cme_rccl_error_string(int(rc)).decode()
                raise RuntimeError(f"{what}: RCCL error {rc - 10000} ({msg})")
            msg = hip().cme_hip_error_string(int(rc)).decode()
            raise RuntimeError(f"{what}: HIP error {rc} ({msg})")
        raise RuntimeError(f"{what}: native CPU backend returned {rc}")


def stream_ptr(device: torch.device | None = None) -> int:
    """hipStream_t of torch's current stream (so launches order with torch ops
    and are captured by torch.cuda.CUDAGraph / hipGraph)."""
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: torch.Tensor) -> int:
    return t.data_ptr()


# Debug / observability switches (read once):
#   CME_SYNC_CHECK=1  synchronise the device after every native HIP call and
#                     raise at the call that faulted (the reference's
#                     check_launch, mp1-util.h:8-18, as an opt-in; also the
#                     HIP_LAUNCH_BLOCKING-style race triage mode of SURVEY §5)
#   CME_TRACE=1       wrap every native HIP call in a roctx range named after
#                     the entry point (rocprofv3 --marker-trace shows them)
SYNC_CHECK = os.environ.get("CME_SYNC_CHECK", "0") not in ("", "0")
TRACE = os.environ.get("CME_TRACE", "0") not in ("", "0")


def call_hip(name: str, *args) -> None:
    if TRACE:
        torch.cuda.nvtx.range_push(name)
    try:
        check(_fn("hip", name)(*args), name, "hip")
        if SYNC_CHECK:
            check(_fn("hip", "cme_device_sync")(), f"{name} (asynchronous failure, CME_SYNC_CHECK)", "hip")
    finally:
        if TRACE:
            torch.cuda.nvtx.range_pop()


def call_cpu(name: str, *args) -> None:
    check(_fn("cpu", name)(*args), name, "cpu")


def gpu_available() -> bool:
    return torch.cuda.is_available()
