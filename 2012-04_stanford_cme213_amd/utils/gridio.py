"""Text and binary I/O for stencil grids.

Text: identical layout to the reference's ``operator<<(Grid)`` / ``outputGrid``
(``hw/hw2/solution/2dHeat_solution.cu:247-258, 671-688``): rows printed from the
top (y = gy-1) down, each value ``std::setw(5)`` after ``std::setprecision(3)``
(i.e. ``%.3g`` right-aligned in 5 columns) followed by one space, a newline per
row and a trailing blank line (plus one more ``std::endl`` for the
``saveStateToFile`` flavour, ``:333-342``).

Binary: lossless checkpoints (the reference has only the lossy 3-digit text
dumps -- SURVEY §5 "Checkpoint / resume"), via safetensors.
"""
from __future__ import annotations

import io

import numpy as np


def _fmt(v: float) -> str:
    s = "%.3g" % v
    return "%5s " % s


def format_grid(a: np.ndarray, extra_endl: bool = True) -> str:
    """a: (gy, gx) array in grid coordinates (row 0 = bottom)."""
    buf = io.StringIO()
    gy = a.shape[0]
    for y in range(gy - 1, -1, -1):
        buf.write("".join(_fmt(float(v)) for v in a[y]))
        buf.write("\n")
    buf.write("\n")
    if extra_endl:
        buf.write("\n")
    return buf.getvalue()


def write_grid(path: str, a: np.ndarray, extra_endl: bool = True) -> None:
    """Write a (rows, cols) grid (rows may carry a wider pitch: pass the full
    pitched array and slice columns before calling) with the native writer."""
    from .. import _ext

    a = np.ascontiguousarray(a)
    if a.dtype not in (np.float32, np.float64):
        a = a.astype(np.float64)
    name = "cme_cpu_write_grid_f32" if a.dtype == np.float32 else "cme_cpu_write_grid_f64"
    _ext.call_cpu(name, path.encode(), a.ctypes.data, a.shape[1], a.shape[0], a.shape[1], int(extra_endl))


def write_vector(path: str, v: np.ndarray) -> None:
    """``ofs << v[i] << " "`` for every element (the b.txt format)."""
    from .. import _ext

    v = np.ascontiguousarray(v)
    if v.dtype not in (np.float32, np.float64):
        v = v.astype(np.float64)
    name = "cme_cpu_write_vec_f32" if v.dtype == np.float32 else "cme_cpu_write_vec_f64"
    _ext.call_cpu(name, path.encode(), v.ctypes.data, v.size)


def _register() -> None:
    from .. import _ext

    _ext.proto(_ext.CPU_PROTOS, "cme_cpu_write_grid_f32", "spiiii")
    _ext.proto(_ext.CPU_PROTOS, "cme_cpu_write_grid_f64", "spiiii")
    _ext.proto(_ext.CPU_PROTOS, "cme_cpu_write_vec_f32", "spq")
    _ext.proto(_ext.CPU_PROTOS, "cme_cpu_write_vec_f64", "spq")


_register()


def read_grid(path: str) -> np.ndarray:
    """Parse a text dump back into (gy, gx) grid coordinates (3 sig. digits)."""
    rows = [ln.split() for ln in open(path) if ln.strip()]
    arr = np.array([[float(t) for t in r] for r in rows], dtype=np.float64)
    return arr[::-1].copy()


def save_checkpoint(path: str, tensors: dict, meta: dict) -> None:
    from safetensors.numpy import save_file

    save_file({k: np.ascontiguousarray(v) for k, v in tensors.items()}, path,
              metadata={k: str(v) for k, v in meta.items()})


def load_checkpoint(path: str) -> tuple[dict, dict]:
    from safetensors import safe_open

    out = {}
    with safe_open(path, framework="numpy") as f:
        meta = dict(f.metadata() or {})
        for k in f.keys():
            out[k] = f.get_tensor(k)
    return out, meta
