"""The native ops as PyTorch dispatcher ops: ``torch.ops.cme213x.*``.

Each op is a ``torch.library.custom_op`` over the same C ABI the eager
wrappers call (``cme_*`` in ``libcme213_hip.so`` on ``cuda`` tensors, the
OpenMP ``cme_cpu_*`` in ``libcme213_cpu.so`` on ``cpu`` tensors), plus a fake
(meta) kernel giving the output's shape/dtype without running anything. With
those, ``torch.compile`` traces through the ops without graph breaks,
``torch.library.opcheck`` can validate them, and they can be captured into
CUDA (HIP) graphs like any other op on the current stream.

Ops (schema in each docstring; "!" = mutated in place):

========================  ==============================================================
``heat_step``             curr![region] = FTCS(prev)           (hw2 kernels, any variant)
``heat_stepn``            nsteps (2-4) timesteps in one HBM pass (temporal blocking)
``scan``                  inclusive / exclusive prefix sum
``segmented_scan``        inclusive segmented sum scan (uint8 heads or int32 bitmask)
``sort`` / ``sort_by_key`` stable LSD radix sort (keys, or keys + 32-bit values)
``spmv_csr``              y = A x, A in CSR (rp, col, val)
``transpose``             2-D fp32 transpose
``sgemm`` / ``gemv``      C = A B (MFMA), y = A x
``copy_if``               stable stream compaction (data-dependent length)
========================  ==============================================================

The reference exposes none of this as a library -- every algorithm is a
``main()``; BASELINE.json's north star asks for "a thin
PyTorch-ROCm op wrapper", which this module is.
"""
from __future__ import annotations

import torch
from torch import Tensor

from . import algorithms as _alg
from . import gemm as _gemm
from . import scan as _scan
from . import sort as _sort
from . import spmv as _spmv
from . import stencil as _stencil
from . import transpose as _tr

NS = "cme213x"


def _fresh(out: Tensor, *inputs: Tensor) -> Tensor:
    """custom_op outputs may not alias inputs."""
    for t in inputs:
        if t is not None and out.untyped_storage().data_ptr() == t.untyped_storage().data_ptr():
            return out.clone()
    return out


# ------------------------------------------------------------------ stencil
@torch.library.custom_op(f"{NS}::heat_step", mutates_args=("curr",))
def heat_step(prev: Tensor, curr: Tensor, region: list[int], order: int, xcfl: float, ycfl: float,
              variant: str = "stream") -> None:
    """heat_step(Tensor prev, Tensor(a!) curr, int[] region, int order, float xcfl, float ycfl, str variant)"""
    _stencil.heat_step(prev, curr, tuple(region), order, xcfl, ycfl, variant)


@heat_step.register_fake
def _(prev, curr, region, order, xcfl, ycfl, variant="stream"):
    return None


@torch.library.custom_op(f"{NS}::heat_stepn", mutates_args=("curr",))
def heat_stepn(prev: Tensor, curr: Tensor, regions: list[int], ext: list[int], order: int, xcfl: float,
               ycfl: float, nsteps: int, fma: bool = False, kernel: str = "streamn") -> None:
    """heat_stepn(Tensor prev, Tensor(a!) curr, int[] regions (4 per region), int[] ext, int order, float xcfl,
    float ycfl, int nsteps, bool fma, str kernel)"""
    regs = [tuple(regions[i:i + 4]) for i in range(0, len(regions), 4)]
    _stencil.heat_stepn(prev, curr, regs, tuple(ext), order, xcfl, ycfl, nsteps, fma=fma, kernel=kernel)


@heat_stepn.register_fake
def _(prev, curr, regions, ext, order, xcfl, ycfl, nsteps, fma=False, kernel="streamn"):
    return None


# ------------------------------------------------------------------ scans
@torch.library.custom_op(f"{NS}::scan", mutates_args=())
def scan(x: Tensor, exclusive: bool = False) -> Tensor:
    """scan(Tensor x, bool exclusive) -> Tensor"""
    return _fresh(_scan.scan(x, exclusive=exclusive), x)


@scan.register_fake
def _(x, exclusive=False):
    return torch.empty_like(x, memory_format=torch.contiguous_format)


@torch.library.custom_op(f"{NS}::segmented_scan", mutates_args=())
def segmented_scan(x: Tensor, flags: Tensor) -> Tensor:
    """segmented_scan(Tensor x, Tensor flags) -> Tensor"""
    return _fresh(_scan.segmented_scan(x.contiguous(), flags.contiguous()), x)


@segmented_scan.register_fake
def _(x, flags):
    return torch.empty_like(x, memory_format=torch.contiguous_format)


# ------------------------------------------------------------------ sort
@torch.library.custom_op(f"{NS}::sort", mutates_args=())
def sort(keys: Tensor) -> Tensor:
    """sort(Tensor keys) -> Tensor   (stable radix sort; int32 / uint32 / float32)"""
    return _fresh(_sort.sort(keys), keys)


@sort.register_fake
def _(keys):
    return torch.empty_like(keys, memory_format=torch.contiguous_format)


@torch.library.custom_op(f"{NS}::sort_by_key", mutates_args=())
def sort_by_key(keys: Tensor, values: Tensor) -> tuple[Tensor, Tensor]:
    """sort_by_key(Tensor keys, Tensor values) -> (Tensor, Tensor)"""
    k, v = _sort.sort(keys, values)
    return _fresh(k, keys, values), _fresh(v, keys, values)


@sort_by_key.register_fake
def _(keys, values):
    return (torch.empty_like(keys, memory_format=torch.contiguous_format),
            torch.empty_like(values, memory_format=torch.contiguous_format))


# ------------------------------------------------------------------ sparse / dense linear algebra
@torch.library.custom_op(f"{NS}::spmv_csr", mutates_args=())
def spmv_csr(rp: Tensor, col: Tensor, val: Tensor, x: Tensor, ncols: int) -> Tensor:
    """spmv_csr(Tensor rp, Tensor col, Tensor val, Tensor x, int ncols) -> Tensor"""
    a = _spmv.CSR(rp.numel() - 1, ncols, rp, col, val)
    return _spmv.spmv(a, x)


@spmv_csr.register_fake
def _(rp, col, val, x, ncols):
    return x.new_empty(rp.shape[0] - 1)


@torch.library.custom_op(f"{NS}::transpose", mutates_args=())
def transpose(x: Tensor) -> Tensor:
    """transpose(Tensor x) -> Tensor   (2-D fp32)"""
    return _tr.transpose(x)


@transpose.register_fake
def _(x):
    return x.new_empty(x.shape[1], x.shape[0])


@torch.library.custom_op(f"{NS}::sgemm", mutates_args=())
def sgemm(A: Tensor, B: Tensor) -> Tensor:
    """sgemm(Tensor A, Tensor B) -> Tensor   (fp32, MFMA on the GPU)"""
    return _gemm.sgemm(A, B)


@sgemm.register_fake
def _(A, B):
    return A.new_empty(A.shape[0], B.shape[1])


@torch.library.custom_op(f"{NS}::gemv", mutates_args=())
def gemv(A: Tensor, x: Tensor) -> Tensor:
    """gemv(Tensor A, Tensor x) -> Tensor"""
    return _gemm.gemv(A, x)


@gemv.register_fake
def _(A, x):
    return A.new_empty(A.shape[0])


# ------------------------------------------------------------------ compaction
@torch.library.custom_op(f"{NS}::copy_if", mutates_args=())
def copy_if(x: Tensor, flags: Tensor) -> Tensor:
    """copy_if(Tensor x, Tensor flags) -> Tensor   (length known only after the kernel)"""
    return _fresh(_alg.copy_if(x, flags).clone(), x)


@copy_if.register_fake
def _(x, flags):
    n = torch.library.get_ctx().new_dynamic_size()
    return x.new_empty(n)


OPS = {
    "heat_step": heat_step, "heat_stepn": heat_stepn, "scan": scan, "segmented_scan": segmented_scan,
    "sort": sort, "sort_by_key": sort_by_key, "spmv_csr": spmv_csr, "transpose": transpose, "sgemm": sgemm,
    "gemv": gemv, "copy_if": copy_if,
}
