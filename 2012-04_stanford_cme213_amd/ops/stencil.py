"""2-D heat-stencil op: one FTCS sweep over a region of a pitched grid.

Tensors are 2-D ``(rows, pitch)`` views, contiguous, ``pitch % 64 == 0``;
``cuda`` tensors run the HIP kernels (``csrc/hip/heat2d.hip``), ``cpu`` tensors
the OpenMP oracle (``csrc/cpu/heat2d_cpu.cpp``). Parity target: the reference's
``gpuComputation`` / ``gpuComputationShared*`` and ``cpuComputation``
(``hw/hw2/solution/2dHeat_solution.cu:371-669``).
"""
from __future__ import annotations

import ctypes

import torch

from .. import _ext

_ext.proto(_ext.HIP_PROTOS, "cme_heat_step_f32", "ppiiiiiiiiffip")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_step_f64", "ppiiiiiiiiddip")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_run_f32", "ppiiiiiiiiffiipp")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_run_f64", "ppiiiiiiiiddiipp")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_step2_f32", "ppiipipiffiip")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_step2_f64", "ppiipipiddiip")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_stepn_f32", "ppiipipiiffiip")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_stepn_f64", "ppiipipiiddiip")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_pipe_f32", "ppiipipiiffiip")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_tile_f32", "ppiiiiiiiiffip")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_tile_f64", "ppiiiiiiiiddip")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_pipe_f64", "ppiipipiiddiip")
_ext.proto(_ext.TUNE_PROTOS, "cme_heat_streamn_tune", "ppiiiiiiffiiiip")
_ext.proto(_ext.TUNE_PROTOS, "cme_heat_pipe_tune", "ppiiiiiiffiiiiip")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_dist_run", "ippiiiddiiiiiipp")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_dist_gate_status", "p")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_pipe_gated_f32", "ppiipipiiffiipupp")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_pipe_gated_f64", "ppiipipiiddiipupp")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_dist_info", "pp")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_step_fast_f32", "ppiiiiiiiffp")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_step_fast_f64", "ppiiiiiiiddp")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_pipe_fast_f32", "ppiipipiiffiipupp")
_ext.proto(_ext.HIP_PROTOS, "cme_heat_run_fast_f32", "ppiiiiiiiiffipp")
_ext.proto(_ext.TUNE_PROTOS, "cme_heat_flow_f32", "ppiiiiiiiiiffip")
_ext.proto(_ext.TUNE_PROTOS, "cme_heat_flow_trace_f32", "ppiiiiiiiiiffippp")
_ext.proto(_ext.TUNE_PROTOS, "cme_heat_flow_status", "pi")
_ext.proto(_ext.TUNE_PROTOS, "cme_heat_flow_debug", "pi")
_ext.proto(_ext.TUNE_PROTOS, "cme_heat_tile_res_f64", "ppiiiiiiiiiddippp")
_ext.proto(_ext.TUNE_PROTOS, "cme_heat_tile_res_f32", "ppiiiiiiiiiffippp")
_ext.proto(_ext.TUNE_PROTOS, "cme_heat_tile_res_status", "pi")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_heat_step_f32", "ppiiiiiiff")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_heat_step_f64", "ppiiiiiidd")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_heat_run_f32", "ppiiiiiiffi")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_heat_run_f64", "ppiiiiiiddi")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_heat_step_fma_f32", "ppiiiiiiff")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_heat_step_fma_f64", "ppiiiiiidd")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_heat_step_fast_f32", "ppiiiiiiff")
_ext.proto(_ext.CPU_PROTOS, "cme_cpu_heat_step_fast_f64", "ppiiiiiidd")

VARIANTS = {"naive": 0, "global": 0, "lds": 1, "shared": 1, "stream": 2, "lds_nopad": 3, "stream2": 4,
            "stream2_fma": 5, "stream_fma": 6, "fma": 6, "stream3": 7, "stream3_fma": 8, "stream4": 9,
            "stream4_fma": 10, "pipe3": 11, "pipe3_fma": 12, "pipe4": 13, "pipe4_fma": 14, "pipe5": 15,
            "pipe5_fma": 16, "pipe6": 17, "pipe6_fma": 18, "tile1": 19, "tile1_fma": 20, "tile2": 21,
            "tile2_fma": 22, "tile3": 23, "tile3_fma": 24, "tile4": 25, "tile4_fma": 26}
# variants that advance more than one timestep per launch (multi-step drivers
# only); stream4 (4 steps per HBM pass) is fp32 only, stream3 takes fp32 and
# fp64 (one row per register block for doubles); pipeN = the wave-pipelined
# N-step pass (csrc/hip/heat_pipe.hip), fp32 and fp64 (pipe5 / pipe6: fp32, for
# the HBM-bound low orders)
MULTISTEP = {"stream2", "stream2_fma", "stream3", "stream3_fma", "stream4", "stream4_fma", "pipe3", "pipe3_fma",
             "pipe4", "pipe4_fma", "pipe5", "pipe5_fma", "pipe6", "pipe6_fma", "tile2", "tile2_fma", "tile3",
             "tile3_fma", "tile4", "tile4_fma"}
# tileN[_fma]: N steps per pass of the LDS-resident tile kernel (csrc/hip/heat_tile.hip) -- small grids
# (the hw5 shapes), whole-interior runs only (heat_run)
TILE_VARIANTS = {"tile1", "tile1_fma", "tile2", "tile2_fma", "tile3", "tile3_fma", "tile4", "tile4_fma"}
FP32_ONLY = {"stream4", "stream4_fma", "pipe5", "pipe5_fma", "pipe6", "pipe6_fma"}
# FMA-contracted stencil (heat_update_fma); on CPU tensors these select the
# std::fma oracle, every other variant name the exact (contraction-off) one
FMA_VARIANTS = {"stream2_fma", "stream_fma", "fma", "stream3_fma", "stream4_fma", "pipe3_fma", "pipe4_fma",
                "pipe5_fma", "pipe6_fma", "tile1_fma", "tile2_fma", "tile3_fma", "tile4_fma"}
# reassociated ("fast") arithmetic (csrc/hip/heat_fast.hip; CPU: the fast
# oracle): name -> timesteps per pass. "fast" is a single step (any order,
# fp32 / fp64); pipeN_fast are wide-lane pipelined passes, fp32 order 8
FAST_VARIANTS = {"fast": 1, "pipe2_fast": 2, "pipe3_fast": 3, "pipe4_fast": 4}


def arith_code(fma) -> int:
    """Arithmetic of a pass: False / 0 exact, True / 1 FMA-contracted,
    "fast" / 2 reassociated (the flags word of the native entry points)."""
    if fma == "fast" or (not isinstance(fma, bool) and fma == 2):
        return 2
    if fma in (True, False, 0, 1, "fma", "exact"):
        return 1 if fma in (True, 1, "fma") else 0
    raise ValueError(f"arithmetic must be exact / fma / fast, got {fma!r}")


def _check_fast(t: torch.Tensor, order: int, nsteps: int) -> None:
    if nsteps > 1 and (t.dtype != torch.float32 or order != 8):
        raise ValueError("reassociated multi-step passes: fp32, order 8")


def _check(prev: torch.Tensor, curr: torch.Tensor) -> None:
    if prev.dim() != 2 or curr.shape != prev.shape:
        raise ValueError("prev/curr must be equal-shape 2-D (rows, pitch) tensors")
    if prev.dtype != curr.dtype or prev.device != curr.device:
        raise ValueError("prev/curr dtype/device mismatch")
    if prev.dtype not in (torch.float32, torch.float64):
        raise TypeError("heat stencil supports float32/float64")
    if not (prev.is_contiguous() and curr.is_contiguous()):
        raise ValueError("prev/curr must be contiguous")
    if prev.shape[1] % 64:
        raise ValueError("pitch (row length) must be a multiple of 64 elements")


def heat_step(prev: torch.Tensor, curr: torch.Tensor, region: tuple[int, int, int, int], order: int,
              xcfl: float, ycfl: float, variant: str = "stream", chunk: int = 0) -> None:
    """curr[region] = FTCS(prev); region = (xb, xe, yb, ye) in grid coords."""
    _check(prev, curr)
    if variant in MULTISTEP or variant in TILE_VARIANTS or FAST_VARIANTS.get(variant, 1) > 1:
        raise ValueError(f"variant {variant!r} is a multi-step / whole-interior pass; use heat_run")
    xb, xe, yb, ye = map(int, region)
    rows, pitch = prev.shape
    f64 = prev.dtype == torch.float64
    if variant == "fast":
        if prev.is_cuda:
            _ext.call_hip("cme_heat_step_fast_f64" if f64 else "cme_heat_step_fast_f32", prev.data_ptr(),
                          curr.data_ptr(), pitch, rows, xb, xe, yb, ye, order, xcfl, ycfl, _ext.stream_ptr(prev.device))
        else:
            _ext.call_cpu("cme_cpu_heat_step_fast_f64" if f64 else "cme_cpu_heat_step_fast_f32", prev.data_ptr(),
                          curr.data_ptr(), pitch, xb, xe, yb, ye, order, xcfl, ycfl)
        return
    if prev.is_cuda:
        name = "cme_heat_step_f64" if f64 else "cme_heat_step_f32"
        _ext.call_hip(name, prev.data_ptr(), curr.data_ptr(), pitch, rows, xb, xe, yb, ye, order,
                      VARIANTS[variant], xcfl, ycfl, chunk, _ext.stream_ptr(prev.device))
    else:
        fma = "_fma" if variant in FMA_VARIANTS else ""
        name = f"cme_cpu_heat_step{fma}_f64" if f64 else f"cme_cpu_heat_step{fma}_f32"
        _ext.call_cpu(name, prev.data_ptr(), curr.data_ptr(), pitch, xb, xe, yb, ye, order, xcfl, ycfl)


def heat_step2(prev: torch.Tensor, curr: torch.Tensor, region: tuple[int, int, int, int],
               ext: tuple[int, int, int, int], order: int, xcfl: float, ycfl: float, chunk: int = 0,
               fma: bool = False) -> None:
    """TWO timesteps in one HBM pass (GPU only): the intermediate step covers
    ``ext`` (``region`` grown by at most B cells, e.g. into a 2B-deep halo),
    the second writes ``curr[region]``. Cells of ``ext`` outside the grid's
    update set keep their value. Equal, bit for bit, to two single steps on
    (ext, then region). On CPU it runs exactly that (through a temporary)."""
    _check(prev, curr)
    if not prev.is_cuda:
        v = "fma" if fma else "naive"
        tmp = prev.clone()
        heat_step(prev, tmp, ext, order, xcfl, ycfl, v)
        heat_step(tmp, curr, region, order, xcfl, ycfl, v)
        return
    rows, pitch = prev.shape
    r = (ctypes.c_int * 4)(*map(int, region))
    e = (ctypes.c_int * 4)(*map(int, ext))
    name = "cme_heat_step2_f64" if prev.dtype == torch.float64 else "cme_heat_step2_f32"
    _ext.call_hip(name, prev.data_ptr(), curr.data_ptr(), pitch, rows, ctypes.addressof(r), 1, ctypes.addressof(e),
                  order, xcfl, ycfl, chunk, int(fma), _ext.stream_ptr(prev.device))


def heat_stepn(prev: torch.Tensor, curr: torch.Tensor, regions, ext: tuple[int, int, int, int], order: int,
               xcfl: float, ycfl: float, nsteps: int, chunk: int = 0, fma: bool = False,
               kernel: str = "streamn") -> None:
    """``nsteps`` (2-4) timesteps in one HBM pass (temporal blocking): the
    intermediate steps cover ``ext`` (the output regions grown by at most
    (nsteps-1)*B cells, e.g. into an nsteps*B-deep halo), the last one writes
    ``curr`` on every region of ``regions`` (one tuple or a list of <= 4, one
    launch). Cells of ``ext`` outside the grid's update set keep their value.
    Bitwise equal to ``nsteps`` single steps; fp64 4-step passes need
    ``kernel="pipe"``. ``kernel="pipe"`` (3 or 4 steps) runs the wave-pipelined pass
    (csrc/hip/heat_pipe.hip) instead of streamN: same cells, same bits.
    ``fma``: False exact, True FMA-contracted, "fast" reassociated (fp32
    order 8 for nsteps > 1: the wide-lane pipelined pass of heat_fast.hip).
    On CPU it runs exactly those single steps through temporaries."""
    if kernel not in ("streamn", "pipe"):
        raise ValueError("kernel must be 'streamn' or 'pipe'")
    _check(prev, curr)
    if isinstance(regions[0], int):
        regions = [regions]
    if not 1 <= len(regions) <= 4:
        raise ValueError("1 to 4 output regions per pass")
    arith = arith_code(fma)
    single = ("naive", "fma", "fast")[arith] if not prev.is_cuda else ("stream", "fma", "fast")[arith]
    if nsteps == 1:
        for reg in regions:
            heat_step(prev, curr, reg, order, xcfl, ycfl, single)
        return
    if not 2 <= nsteps <= 4:
        raise ValueError("nsteps must be 1..4")
    if arith == 2:
        _check_fast(prev, order, nsteps)
    if not prev.is_cuda:
        v = ("naive", "fma", "fast")[arith]
        src = prev
        for _ in range(nsteps - 1):
            tmp = prev.clone()
            heat_step(src, tmp, ext, order, xcfl, ycfl, v)
            src = tmp
        for reg in regions:
            heat_step(src, curr, reg, order, xcfl, ycfl, v)
        return
    f64 = prev.dtype == torch.float64
    if f64 and nsteps > 3 and kernel != "pipe":
        raise ValueError("fp64 4-step passes need kernel='pipe'")
    rows, pitch = prev.shape
    flat = [int(v) for reg in regions for v in reg]
    r = (ctypes.c_int * len(flat))(*flat)
    e = (ctypes.c_int * 4)(*map(int, ext))
    if arith == 2:
        _ext.call_hip("cme_heat_pipe_fast_f32", prev.data_ptr(), curr.data_ptr(), pitch, rows, ctypes.addressof(r),
                      len(regions), ctypes.addressof(e), order, nsteps, xcfl, ycfl, chunk, 0, None, 0, None,
                      _ext.stream_ptr(prev.device))
        return
    name = "cme_heat_stepn_f64" if f64 else "cme_heat_stepn_f32"
    if kernel == "pipe" and nsteps >= 3:
        name = "cme_heat_pipe_f64" if f64 else "cme_heat_pipe_f32"
    _ext.call_hip(name, prev.data_ptr(), curr.data_ptr(), pitch, rows, ctypes.addressof(r), len(regions),
                  ctypes.addressof(e), order, nsteps, xcfl, ycfl, chunk, int(fma), _ext.stream_ptr(prev.device))


def heat_tile(prev: torch.Tensor, curr: torch.Tensor, region: tuple[int, int, int, int], order: int, xcfl: float,
              ycfl: float, nsteps: int, fma: bool = False) -> None:
    """ONE ``nsteps``-step (1-4) pass of the LDS-resident tile kernel
    (``csrc/hip/heat_tile.hip``): curr[region] = FTCS^nsteps(prev). Every
    cell outside ``region`` must hold the same fixed value in both buffers
    (the Dirichlet ghost layer of a whole-interior run)."""
    _check(prev, curr)
    if not prev.is_cuda:
        raise ValueError("heat_tile: GPU only")
    xb, xe, yb, ye = map(int, region)
    rows, pitch = prev.shape
    name = "cme_heat_tile_f64" if prev.dtype == torch.float64 else "cme_heat_tile_f32"
    _ext.call_hip(name, prev.data_ptr(), curr.data_ptr(), pitch, rows, xb, xe, yb, ye, order, int(nsteps), xcfl,
                  ycfl, int(fma), _ext.stream_ptr(prev.device))


def heat_run(a: torch.Tensor, b: torch.Tensor, region: tuple[int, int, int, int], order: int, xcfl: float,
             ycfl: float, iters: int, variant: str = "stream", chunk: int = 0) -> torch.Tensor:
    """``iters`` timesteps starting from ``a``; returns the buffer holding the
    final state. Single-step variants ping-pong (final = ``a`` iff iters is
    even); ``stream2`` advances two steps per HBM pass (temporal blocking), so
    the final buffer is reported by the native driver."""
    _check(a, b)
    xb, xe, yb, ye = map(int, region)
    rows, pitch = a.shape
    f64 = a.dtype == torch.float64
    if f64 and variant in FP32_ONLY:
        raise ValueError(f"variant {variant!r} is fp32 only")
    if variant in FAST_VARIANTS:
        ns = FAST_VARIANTS[variant]
        if a.is_cuda and ns > 1:
            _check_fast(a, order, ns)
            final = ctypes.c_int(0)
            _ext.call_hip("cme_heat_run_fast_f32", a.data_ptr(), b.data_ptr(), pitch, rows, xb, xe, yb, ye, order, ns,
                          xcfl, ycfl, iters, ctypes.addressof(final), _ext.stream_ptr(a.device))
            return b if final.value else a
        for i in range(iters):  # single steps (every pass length gives the same bits)
            src, dst = (a, b) if i % 2 == 0 else (b, a)
            heat_step(src, dst, region, order, xcfl, ycfl, "fast")
        return a if iters % 2 == 0 else b
    if a.is_cuda:
        name = "cme_heat_run_f64" if f64 else "cme_heat_run_f32"
        final = ctypes.c_int(0)
        _ext.call_hip(name, a.data_ptr(), b.data_ptr(), pitch, rows, xb, xe, yb, ye, order, VARIANTS[variant],
                      xcfl, ycfl, iters, chunk, ctypes.addressof(final), _ext.stream_ptr(a.device))
        return b if final.value else a
    elif variant in FMA_VARIANTS:
        for i in range(iters):
            src, dst = (a, b) if i % 2 == 0 else (b, a)
            heat_step(src, dst, region, order, xcfl, ycfl, "fma")
    else:
        name = "cme_cpu_heat_run_f64" if f64 else "cme_cpu_heat_run_f32"
        _ext.call_cpu(name, a.data_ptr(), b.data_ptr(), pitch, xb, xe, yb, ye, order, xcfl, ycfl, iters)
    return a if iters % 2 == 0 else b


def heat_flow(a: torch.Tensor, b: torch.Tensor, region: tuple[int, int, int, int], order: int, xcfl: float,
              ycfl: float, npass: int, fma="fma", ns: int = 4, trace: bool = False):
    """``npass`` four-step passes of the whole ``region`` as ONE persistent
    dataflow launch (csrc/hip_tune/heat_flow.hip, tuning library: tasks pulled from a ticket, each
    waiting for the 3 x 3 neighbourhood of the previous pass). fp32, order 8,
    GPU; ``fma``: "exact" / False, "fma" / True, or "fast". Bit for bit the
    result of ``npass`` one-pass launches (``heat_run`` with the knob
    ``heat_flow`` = 0). Returns the buffer holding the result (``b`` for odd
    ``npass``), or with ``trace=True`` ``(buffer, trace, tasks_per_pass)``:
    trace[t] = (ticket time, start, end, HW_ID | XCC_ID << 32) of ticket t, in
    100 MHz wall-clock ticks. Raises if a dependency wait gave up."""
    _check(a, b)
    if not a.is_cuda or a.dtype != torch.float32 or order != 8 or ns != 4:
        raise ValueError("heat_flow: fp32, order 8, four steps per pass, on the GPU")
    xb, xe, yb, ye = map(int, region)
    rows, pitch = a.shape
    code = arith_code(fma)
    s = _ext.stream_ptr(a.device)
    tr = None
    if trace:
        strips = -(-(xe - (xb & ~7)) // 480)
        cap = strips * (-(-(ye - yb) // 16)) * int(npass)
        tr = torch.zeros((cap, 4), dtype=torch.int64, device=a.device)
        nt = ctypes.c_int(0)
        _ext.call_hip("cme_heat_flow_trace_f32", a.data_ptr(), b.data_ptr(), pitch, rows, xb, xe, yb, ye, order, code,
                      ns, xcfl, ycfl, int(npass), tr.data_ptr(), ctypes.addressof(nt), s)
    else:
        _ext.call_hip("cme_heat_flow_f32", a.data_ptr(), b.data_ptr(), pitch, rows, xb, xe, yb, ye, order, code, ns,
                      xcfl, ycfl, int(npass), s)
    torch.cuda.synchronize(a.device)
    if flow_timed_out(reset=True):
        raise RuntimeError("heat_flow: a dependency wait gave up (CME_FLOW_SPINS)")
    out = b if npass % 2 else a
    if trace:
        return out, tr[: nt.value * int(npass)].cpu(), nt.value
    return out


def flow_timed_out(reset: bool = False) -> bool:
    """Sticky give-up flag of the dataflow launches (read after a sync)."""
    v = ctypes.c_uint(0)
    _ext.call_hip("cme_heat_flow_status", ctypes.addressof(v), int(reset))
    return bool(v.value)


HIP_COOP_TOO_LARGE = 720  # hipErrorCooperativeLaunchTooLarge


def heat_tile_res(a: torch.Tensor, b: torch.Tensor, region: tuple[int, int, int, int], order: int, xcfl: float,
                  ycfl: float, npass: int, ns: int = 2, fma: bool = False, trace: bool = False):
    """``npass`` passes of ``ns`` (2, or 4 at order 8) steps of the whole
    ``region`` with every 64 x 64 tile resident in LDS for the whole run, in
    ONE cooperative launch (csrc/hip_tune/heat_tile_res.hip, tuning library: only the NS*B-deep
    halo ring moves, behind the tile's inner cone). GPU, fp32 / fp64, orders
    2 / 4 / 8; bit for bit the result of single steps of the same arithmetic.
    Returns the buffer holding the result (``b`` for odd ``npass``), or with
    ``trace=True`` ``(buffer, trace, ntiles)``: trace[pass * ntiles + tile,
    :5] = wall-clock stamps (100 MHz) at the pass start, after the inner
    steps, with the halo in, after the outer steps (ring stores issued), and
    when the pass's ring was published (during the next pass). Raises ``RuntimeError`` if a
    neighbour wait gave up, ``ValueError`` if the tiles cannot all be
    resident (too large a grid: run tile passes)."""
    _check(a, b)
    if not a.is_cuda or order not in (2, 4, 8) or ns not in ((2, 4) if order == 8 else (2,)):
        raise ValueError("heat_tile_res: GPU, orders 2/4/8, 2 steps per exchange (or 4 at order 8)")
    xb, xe, yb, ye = map(int, region)
    rows, pitch = a.shape
    ntiles = (-(-(xe - xb) // 64)) * (-(-(ye - yb) // 64))
    tr = torch.zeros((ntiles * int(npass), 8), dtype=torch.int64, device=a.device) if trace else None
    nt = ctypes.c_int(0)
    name = "cme_heat_tile_res_f64" if a.dtype == torch.float64 else "cme_heat_tile_res_f32"
    rc = _ext._fn("hip", name)(a.data_ptr(), b.data_ptr(), pitch, rows, xb, xe, yb, ye, order, ns, int(bool(fma)),
                               xcfl, ycfl, int(npass), tr.data_ptr() if trace else None, ctypes.addressof(nt),
                               _ext.stream_ptr(a.device))
    if rc == HIP_COOP_TOO_LARGE:
        raise ValueError(f"heat_tile_res: {ntiles} tiles cannot all be resident on this device")
    _ext.check(rc, name)
    torch.cuda.synchronize(a.device)
    if tile_res_timed_out(reset=True):
        raise RuntimeError("heat_tile_res: a neighbour wait gave up (CME_FLOW_SPINS)")
    out = b if npass % 2 else a
    if trace:
        return out, tr[:, :5].cpu(), nt.value
    return out


def tile_res_timed_out(reset: bool = False) -> bool:
    """Sticky give-up flag of the resident-tile launches (read after a sync;
    ``heat_run``'s tile variants use them)."""
    v = ctypes.c_uint(0)
    _ext.call_hip("cme_heat_tile_res_status", ctypes.addressof(v), int(reset))
    return bool(v.value)


def heat_step_torch(prev: torch.Tensor, region, order: int, xcfl: float, ycfl: float) -> torch.Tensor:
    """Plain-PyTorch fp oracle of one sweep (returns a new tensor). Used only by
    tests to cross-check the native CPU oracle itself."""
    coeffs = {2: [1.0, -2.0, 1.0], 4: [-1.0, 16.0, -30.0, 16.0, -1.0],
              8: [-9.0, 128.0, -1008.0, 8064.0, -14350.0, 8064.0, -1008.0, 128.0, -9.0]}[order]
    B = len(coeffs) // 2
    xb, xe, yb, ye = region
    out = prev.clone()
    c = prev[yb:ye, xb:xe]
    dx = torch.zeros_like(c)
    dy = torch.zeros_like(c)
    for k, w in enumerate(coeffs):
        o = k - B
        dx = dx + w * prev[yb:ye, xb + o:xe + o]
        dy = dy + w * prev[yb + o:ye + o, xb:xe]
    out[yb:ye, xb:xe] = c + xcfl * dx + ycfl * dy
    return out
