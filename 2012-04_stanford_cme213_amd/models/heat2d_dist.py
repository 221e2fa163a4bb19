"""Distributed 2-D heat diffusion with halo exchange (the hw5 workload, moved
from host MPI to GPUs + RCCL over xGMI).

Parity target: ``hw/hw5/2dHeat_solution.cpp`` -- 1-D stripes / 2-D blocks,
``sync`` (compute, then exchange) and ``async`` (overlap) modes, per-rank dumps
``grid<rank>_{init,final}.txt`` and rank 0's
``"<iters> iterations on a <nx> by <ny> grid took: <s> seconds."``.

MI355X-first design:

* one process per GPU; each rank's subdomain is a :class:`HeatGrid` (both
  ping-pong states in one allocation);
* row halos are sent straight out of / received straight into the grid
  (rows are contiguous: no packing); column halos are packed into contiguous
  staging buffers;
* every exchange is ONE grouped RCCL batch (``batch_isend_irecv``) on RCCL's
  stream; in ``async`` mode the deep-interior sweep is enqueued on the compute
  stream right after posting, so halo traffic overlaps it, and the four border
  strips run after a stream-side wait (no host sync anywhere in the loop);
* several subdomains may live in one process (``LoopbackComm``): their
  exchanges become device copies -- the reference's missing single-process
  fake backend, used by the CPU tests.

Unlike the reference solution's async loop (which computes the first
iteration before any halo has been posted and relies on a uniform IC,
``:541-568``), halos of the state being read are always exchanged before they
are used, so non-uniform initial conditions are correct.
"""
from __future__ import annotations

import ctypes
import time

import numpy as np
import torch

from ..ops.stencil import arith_code, heat_run, heat_step, heat_stepn
from ..parallel.comm import Comm, LoopbackComm, P2P, Pending
from ..parallel.decomp import Block, decompose
from ..utils.params import SimParams
from .heat2d import HeatGrid


class SubDesc(ctypes.Structure):
    """Mirror of ``SubDesc`` in ``csrc/hip/dist_heat.hip`` (one subdomain of
    the native distributed loop)."""
    _fields_ = [("buf", ctypes.c_void_p * 2), ("pitch", ctypes.c_int), ("gy", ctypes.c_int),
                ("interior", ctypes.c_void_p), ("n_int", ctypes.c_int), ("border", ctypes.c_void_p),
                ("n_b", ctypes.c_int), ("ext", ctypes.c_void_p), ("rows", ctypes.c_void_p),
                ("n_rows", ctypes.c_int), ("blks", ctypes.c_void_p), ("n_blks", ctypes.c_int),
                ("stage", ctypes.c_void_p), ("rank", ctypes.c_int), ("ipc", ctypes.c_void_p)]


class IpcPeerDesc(ctypes.Structure):
    """Mirror of ``IpcPeerDesc`` (``csrc/hip/dist_heat.hip``): one
    neighbouring process's mapped memory."""
    _fields_ = [("buf", ctypes.c_void_p * 2), ("stage", ctypes.c_void_p), ("flags", ctypes.c_void_p),
                ("rank", ctypes.c_int), ("slot", ctypes.c_int)]


class IpcPlan(ctypes.Structure):
    """Mirror of ``IpcPlan``: transport 3 of the native loop."""
    _fields_ = [("flags", ctypes.c_void_p), ("timeout", ctypes.c_void_p), ("epoch", ctypes.c_void_p),
                ("row_src", ctypes.c_void_p), ("blk_src", ctypes.c_void_p), ("npeer", ctypes.c_int),
                ("peer", IpcPeerDesc * 8)]


_IPC_TIMEOUT_WORD = 16  # index of the give-up word in the flags tensor


class _Sub:
    """One subdomain: its block, grid (ghost depth ``H``) and halo views.
    Every exchange moves ``H``-deep halos: rows straight from/to the grid,
    columns (and, for ``H > B``, the diagonal corners) via staging."""

    def __init__(self, blk: Block, grid: HeatGrid, corners: bool):
        self.blk = blk
        self.grid = grid
        H, ny = grid.H, grid.ny
        self.stage = {}
        for side in ("left", "right"):
            if getattr(blk, side) >= 0:
                self.stage[side] = (torch.empty((ny, H), dtype=grid.dtype, device=grid.device),
                                    torch.empty((ny, H), dtype=grid.dtype, device=grid.device))
        self.diag = {}
        if corners:
            for dx in (-1, 1):
                for dy in (-1, 1):
                    peer = blk.neighbor(dx, dy)
                    if peer >= 0:
                        self.diag[(dx, dy)] = peer
                        self.stage[(dx, dy)] = (torch.empty((H, H), dtype=grid.dtype, device=grid.device),
                                                torch.empty((H, H), dtype=grid.dtype, device=grid.device))

    # views into state k -------------------------------------------------
    def row_send(self, k: int, side: str) -> torch.Tensor:
        g = self.grid
        H, ny = g.H, g.ny
        rows = (ny, ny + H) if side == "top" else (H, 2 * H)
        return g.buf[k, rows[0]:rows[1]]

    def row_recv(self, k: int, side: str) -> torch.Tensor:
        g = self.grid
        H, ny = g.H, g.ny
        rows = (ny + H, ny + 2 * H) if side == "top" else (0, H)
        return g.buf[k, rows[0]:rows[1]]

    def col_send_view(self, k: int, side: str) -> torch.Tensor:
        g = self.grid
        H, nx, ny = g.H, g.nx, g.ny
        cols = (nx, nx + H) if side == "right" else (H, 2 * H)
        return g.buf[k, H:H + ny, cols[0]:cols[1]]

    def col_recv_view(self, k: int, side: str) -> torch.Tensor:
        g = self.grid
        H, nx, ny = g.H, g.nx, g.ny
        cols = (nx + H, nx + 2 * H) if side == "right" else (0, H)
        return g.buf[k, H:H + ny, cols[0]:cols[1]]

    def corner_origin(self, dx: int, dy: int, send: bool) -> tuple[int, int]:
        """(x, y) of the H x H corner block toward diagonal (dx, dy)."""
        g = self.grid
        H = g.H
        if send:
            return (g.nx if dx > 0 else H), (g.ny if dy > 0 else H)
        return (g.nx + H if dx > 0 else 0), (g.ny + H if dy > 0 else 0)

    def corner_view(self, k: int, dx: int, dy: int, send: bool) -> torch.Tensor:
        x, y = self.corner_origin(dx, dy, send)
        H = self.grid.H
        return self.grid.buf[k, y:y + H, x:x + H]


_OPP = {"top": "bottom", "bottom": "top", "left": "right", "right": "left"}

# fp64 subdomains at least this large run 3-4 step passes on the pipelined
# kernel; smaller ones on streamN (measured, one MI355X, order 8, FMA:
# 1000^2 stream3 0.0058 vs pipe4 0.0074 ms/iter; 2000^2 stream3 0.0096-0.0103
# vs pipe4 0.0085 -- profiles/heat_fp64_pipe_r2.jsonl, heat_fp64_stream3_r2.jsonl,
# dist_fused_r2.md)
_F64_PIPE_MIN_POINTS = 2000 * 2000
# single-grid fp64 runs up to this size use the LDS-resident tile pass
# (csrc/hip/heat_tile.hip, four steps per pass): 1000^2 order 8, 1000 steps,
# 4.63 ms FMA / 5.35 exact vs 5.67 / 6.88 for streamN; at 2000^2 the pipelined
# pass wins (8.5 vs 15.5 ms; profiles/heat_tile_r4.md)
_F64_TILE_MAX_POINTS = 1200 * 1200
# ... and fp32 ones too (round 4, benchmarks/bench_small_variants.py, 1000 steps,
# order 8: 1000^2 tile4 3.69 / tile4_fma 3.33 ms vs pipe3 6.69 / pipe3_fma 5.34;
# 1500^2 the pipelined pass wins, 5.88 vs 7.94 FMA; profiles/heat_small_r4.md)
_TILE_MAX_POINTS = _F64_TILE_MAX_POINTS
# solo fp32 order-8 grids above the tile range and up to this size: 3-step passes (auto_tblock)
_F32_PIPE3_MAX_POINTS = 2500 * 2500


def auto_tblock(dtype, points: int, fma: bool, device: str = "cuda", solo: bool = False, order: int = 8) -> int:
    """Timesteps per HBM pass (and per halo exchange) for a subdomain of
    ``points`` cells: 4 for fp32 (pipelined pass, every N of the 16384^2
    bench) and for large fp64 subdomains; 3 (FMA) or 2 (exact) for small fp64
    ones, where streamN wins (exact fp64 1000^2: stream2 0.0073 vs stream3
    0.0087 ms/iter). A solo fp32 order-8 grid between the tile pass's range
    and 2500^2 takes 3 (exact / FMA; the 4-step pass's warm-up rows dominate
    there: 2000^2 pipe3 3.99 vs pipe4 4.97 ms per 400 steps; the reassociated
    arithmetic keeps 4, 3.97 vs 3.49; profiles/heat_small_r4.md). On the CPU
    backend: 1 (no temporal blocking)."""
    if torch.device(device).type != "cuda":
        return 1
    if dtype == torch.float32:
        if solo and order == 8 and arith_code(fma) != 2 and _TILE_MAX_POINTS < points <= _F32_PIPE3_MAX_POINTS:
            return 3
        if solo and order == 2:  # HBM-bound: 5-6 steps per pass (pipe5 / pipe6; heat_small_r4.md)
            return 6 if arith_code(fma) == 1 else 5
        return 4
    if points >= _F64_PIPE_MIN_POINTS:
        return 4
    if solo and (points <= _F64_TILE_MAX_POINTS or order < 8):
        # the tile pass (auto_kernel) / orders 2 and 4: the pipelined 4-step
        # pass (1500^2 order 2: pipe4 1.42 vs stream2 2.25 ms per 400 steps
        # exact, 1.29 vs stream3 1.64 FMA; heat_small_r4.md)
        return 4
    return 3 if fma else 2


def auto_kernel(dtype, points: int, tblock: int, solo: bool = False, fast: bool = False, order: int = 8) -> str:
    """Pass kernel for 3-4 step passes: the wave-pipelined pass for fp32 and
    for fp64 subdomains of at least 2000^2 cells (and every fp64 4-step pass:
    streamN stops at 3 for doubles), streamN below that; a small grid on one
    GPU with no neighbours (``solo``) runs the LDS-resident tile pass where it
    measured faster: order 8 (fp32 and fp64) and fp64 order 4 -- the narrower
    stencils leave the pipelined pass HBM-light enough to win (fp32 order 2
    1000^2: pipe4 2.11 vs tile4 2.63 ms FMA; profiles/heat_small_r4.md) --
    and never in the reassociated arithmetic (``fast``: pipelined only)."""
    tile_order = order == 8 or (order == 4 and dtype == torch.float64)
    if solo and not fast and tile_order and points <= _TILE_MAX_POINTS and tblock >= 2:
        return "tile"
    if tblock < 3:
        return "streamn"
    if dtype == torch.float32 or tblock > 3 or points >= _F64_PIPE_MIN_POINTS:
        return "pipe"
    return "streamn"


def _save_atomic(path: str, tensors: dict, meta: dict) -> None:
    """Write a checkpoint file under a temporary name, then rename it over
    ``path``: a crash mid-write leaves the previous checkpoint intact."""
    import os

    from ..utils.gridio import save_checkpoint

    tmp = f"{path}.tmp{os.getpid()}"
    save_checkpoint(tmp, tensors, meta)
    os.replace(tmp, path)


_ACTIVE_WRITERS: dict = {}  # realpath(directory) -> CheckpointWriter still writing


class CheckpointWriter:
    """Background writer of :meth:`DistHeat.checkpoint_async` (one thread:
    wait for the device-to-host copy, then one safetensors file per
    subdomain)."""

    def __init__(self, directory: str, items: list, event=None):
        import os
        import threading

        self.paths = [os.path.join(directory, f"heat_rank{r}.safetensors") for r, *_ in items]
        self._items, self._event, self._error = items, event, None
        # one writer per directory at a time: a new checkpoint into the same
        # files waits for the previous one (no interleaved per-rank files)
        key = os.path.realpath(directory)
        prev = _ACTIVE_WRITERS.get(key)
        if prev is not None and prev is not self:
            prev._thread.join()
        _ACTIVE_WRITERS[key] = self
        self._thread = threading.Thread(target=self._write, daemon=True)
        self._thread.start()

    def _write(self) -> None:
        try:
            if self._event is not None:
                self._event.synchronize()
            for path, (r, t, meta, _) in zip(self.paths, self._items):
                _save_atomic(path, {"interior": t.numpy()}, meta)
        except Exception as e:  # noqa: BLE001 - re-raised by wait()
            self._error = e
        finally:
            self._items = None  # release the pinned buffers and snapshots

    def done(self) -> bool:
        return not self._thread.is_alive()

    def wait(self) -> list[str]:
        self._thread.join()
        if self._error is not None:
            raise self._error
        return self.paths


class DistHeat:
    """Distributed heat solver. ``local_ranks`` lists the subdomains owned by
    this process (default: ``[comm.rank]``); ``world`` is the total number of
    subdomains (default: ``comm.size``)."""

    def __init__(self, params: SimParams, comm: Comm | None = None, dtype=torch.float32, device="cpu",
                 local_ranks: list[int] | None = None, world: int | None = None, variant: str = "stream",
                 tblock: int | str = 1, fma: bool = False, kernel: str = "streamn",
                 periodic: tuple[bool, bool] = (False, False), native: str = "off"):
        self.p = params
        self.comm = comm or LoopbackComm()
        self.world = world or self.comm.size
        self.local_ranks = local_ranks if local_ranks is not None else [self.comm.rank]
        self.periodic = (bool(periodic[0]), bool(periodic[1]))
        if self.comm.size > 1 and (len(self.local_ranks) != 1 or self.world != self.comm.size):
            raise ValueError("multi-process runs own exactly one subdomain per rank")
        if native not in ("off", "auto", "on"):
            raise ValueError("native must be 'off', 'auto' or 'on'")
        # run(): the native C++ time loop after a one-time bitwise self-test
        # ("auto": fall back to the Python loop if it fails; "on": raise)
        self.native_mode = native
        self.native_info: dict | None = None
        auto_tb = tblock == "auto"
        if tblock == "auto" or kernel == "auto":
            # by the LARGEST subdomain of the whole decomposition -- the same
            # answer on every rank (an uneven split must not give neighbours
            # different halo depths / exchange cadences)
            pts = max(b.nx * b.ny for b in (decompose(params.nx, params.ny, self.world, params.grid_method, r,
                                                      self.periodic)
                                            for r in range(self.world)))
            solo = self.world == 1 and not any(self.periodic)
            if tblock == "auto":
                tblock = auto_tblock(dtype, pts, fma, torch.device(device).type, solo, order=params.order)
            if kernel == "auto":
                kernel = auto_kernel(dtype, pts, tblock, solo and torch.device(device).type == "cuda",
                                     fast=arith_code(fma) == 2, order=params.order)
        deep = (dtype == torch.float32 and torch.device(device).type == "cuda" and self.world == 1
                and not any(self.periodic) and kernel == "pipe")
        if auto_tb and tblock > 4 and not deep:
            tblock = 4  # an explicitly chosen kernel other than the pipelined pass
        if tblock not in ((1, 2, 3, 4, 5, 6) if deep else (1, 2, 3, 4)):
            raise ValueError("tblock must be 1..4 (5-6: solo fp32 GPU grids, kernel='pipe')")
        if kernel not in ("streamn", "pipe", "tile"):
            raise ValueError("kernel must be 'streamn', 'pipe' or 'tile'")
        if kernel == "tile" and (self.world != 1 or any(self.periodic)):
            raise ValueError("kernel='tile' runs single-grid (world 1, non-periodic) passes only")
        if tblock > 3 and dtype == torch.float64 and kernel == "streamn" and torch.device(device).type == "cuda":
            raise ValueError("fp64 4-step passes need kernel='pipe' on the GPU (streamN fp64 stops at 3)")
        # arithmetic: 0 exact, 1 FMA-contracted, 2 reassociated ("fast": fma="fast";
        # fp32 order 8, the pipelined kernel for multi-step passes on the GPU)
        self.arith = arith_code(fma)
        if self.arith == 2 and tblock > 1 and (dtype != torch.float32 or params.order != 8 or kernel == "tile"
                                               or (kernel != "pipe" and torch.device(device).type == "cuda")):
            raise ValueError("fma='fast' multi-step passes: fp32, order 8, kernel='pipe'")
        if self.arith == 2 and tblock > 4:
            # the reassociated pass exists for 2-4 steps (heat_fast.hip); say so
            # here rather than fail on a missing variant in run()
            raise ValueError("fma='fast' runs 1-4 steps per pass (tblock <= 4)")
        self.fma = self.arith == 1
        # 3-4 step passes: streamN (one wave holds every step) or the
        # wave-pipelined kernel (csrc/hip/heat_pipe.hip); identical results
        self.kernel = kernel
        self.variant = {1: "fma", 2: "fast"}.get(self.arith, variant)
        self.tblock = tblock
        self.device = torch.device(device)
        self.subs: dict[int, _Sub] = {}
        for r in self.local_ranks:
            blk = decompose(params.nx, params.ny, self.world, params.grid_method, r, self.periodic)
            g = HeatGrid(params, dtype, device, nx=blk.nx, ny=blk.ny, bc_sides=blk.bc_sides,
                         halo=tblock * params.border)
            self.subs[r] = _Sub(blk, g, corners=tblock > 1)
        self.iteration = 0
        # make halos consistent with the neighbours' initial state
        self.exchange(self._cur()).wait()

    def _flags(self) -> int:
        """Kernel flags of the native loop (cme_heat_dist_run): bit 0 FMA,
        bit 1 the pipelined NS-step kernel, bit 3 reassociated arithmetic."""
        return int(self.fma) | (2 if self.kernel == "pipe" else 0) | (8 if self.arith == 2 else 0)

    def _fma_arg(self):
        """the ``fma`` argument of the stencil ops for this solver's arithmetic"""
        return "fast" if self.arith == 2 else self.fma

    def _cur(self) -> int:
        return next(iter(self.subs.values())).grid.cur

    # -- halo exchange ---------------------------------------------------
    def exchange(self, k: int) -> Pending:
        """Fill the ghost cells of state ``k`` from the neighbours' borders.

        Remote pieces are posted in the canonical halo order of the native
        plan (:meth:`_sub_plan`): sends as rows (top, bottom) then blocks
        (left, corners, right); receives in the REVERSED order of each group.
        The block order is its own mirror (piece i and piece n-1-i face
        opposite ways), so the k-th send to a peer always meets the k-th
        receive from us on the peer -- also when one peer sits on several
        sides (periodic grids with one or two blocks along an axis, where
        per-peer FIFO matching of same-side pieces would swap the halos)."""
        sends: list[P2P] = []
        recvs: list[P2P] = []
        post_unpack = []
        for r, s in self.subs.items():
            blk = s.blk
            row_recv, blk_recv = [], []
            for side in ("top", "bottom"):
                peer = getattr(blk, side)
                if peer < 0:
                    continue
                if peer in self.subs:
                    self.subs[peer].row_recv(k, _OPP[side]).copy_(s.row_send(k, side))
                else:
                    sends.append(P2P("send", s.row_send(k, side), peer))
                    row_recv.append(P2P("recv", s.row_recv(k, side), peer))
            pieces = [("left", blk.left)] + [((dx, dy), p) for (dx, dy), p in s.diag.items()] + [("right", blk.right)]
            for key, peer in pieces:
                if peer < 0:
                    continue
                if isinstance(key, str):
                    send_v, recv_v = s.col_send_view(k, key), s.col_recv_view(k, key)
                    if peer in self.subs:
                        self.subs[peer].col_recv_view(k, _OPP[key]).copy_(send_v)
                        continue
                else:
                    dx, dy = key
                    send_v, recv_v = s.corner_view(k, dx, dy, True), s.corner_view(k, dx, dy, False)
                    if peer in self.subs:
                        self.subs[peer].corner_view(k, -dx, -dy, False).copy_(send_v)
                        continue
                sbuf, rbuf = s.stage[key]
                sbuf.copy_(send_v)
                sends.append(P2P("send", sbuf, peer))
                blk_recv.append(P2P("recv", rbuf, peer))
                post_unpack.append((recv_v, rbuf))
            recvs += row_recv[::-1] + blk_recv[::-1]
        pend = self.comm.exchange(sends + recvs)
        if not post_unpack:
            return pend

        class _Unpack(Pending):
            def wait(self_inner):
                pend.wait()
                for dst, src in post_unpack:
                    dst.copy_(src)

        return _Unpack()

    # -- one timestep ----------------------------------------------------
    def step(self, sync: bool | None = None) -> None:
        sync = self.p.sync if sync is None else sync
        k = self._cur()
        if sync:
            for s in self.subs.values():
                g = s.grid
                heat_step(g.buf[k], g.buf[1 - k], g.interior, g.order, g.xcfl, g.ycfl, self.variant)
            # reference order: compute, then exchange the new state's halos
            self.exchange(1 - k).wait()
        else:
            # halos of state k are already valid (exchanged at the end of the
            # previous step / at construction); post the exchange for the state
            # being produced AFTER computing its borders, and overlap the
            # next step's deep interior with it.
            pend = getattr(self, "_pending", None)
            for s in self.subs.values():
                g = s.grid
                for reg in _interior_regions(s, g.B):
                    heat_step(g.buf[k], g.buf[1 - k], reg, g.order, g.xcfl, g.ycfl, self.variant)
            if pend is not None:
                pend.wait()
            for s in self.subs.values():
                g = s.grid
                for reg in _border_regions(s, g.B):
                    heat_step(g.buf[k], g.buf[1 - k], reg, g.order, g.xcfl, g.ycfl, self.variant)
            self._pending = self.exchange(1 - k)
        for s in self.subs.values():
            s.grid.cur = 1 - k
            s.grid.iteration += 1
        self.iteration += 1

    def step2(self, sync: bool | None = None) -> None:
        """TWO timesteps per exchange (needs ``tblock >= 2``)."""
        self.stepn(2, sync)

    def stepn(self, ns: int, sync: bool | None = None) -> None:
        """``ns`` timesteps per exchange (``2 <= ns <= tblock``): the
        ``tblock*B``-deep halos (corners included) feed one fused ``ns``-step
        pass per region; the deep interior (``tblock*B`` from any neighbour)
        overlaps the in-flight exchange in async mode, and the border strips go
        out as one launch. Same schedule as the native loop
        (``csrc/hip/dist_heat.hip``)."""
        if not 2 <= ns <= self.tblock:
            raise ValueError(f"stepn({ns}) needs 2 <= ns <= tblock={self.tblock}")
        sync = self.p.sync if sync is None else sync
        k = self._cur()

        def sweep(regions_of):
            for s in self.subs.values():
                g = s.grid
                regs = list(regions_of(s, self.tblock * g.B))
                if regs:
                    heat_stepn(g.buf[k], g.buf[1 - k], regs, _ext_region(s), g.order, g.xcfl, g.ycfl, ns,
                               fma=self._fma_arg(), kernel=self.kernel)

        if sync:
            sweep(_interior_regions)
            sweep(_border_regions)
            self.exchange(1 - k).wait()
        else:
            pend = getattr(self, "_pending", None)
            sweep(_interior_regions)
            if pend is not None:
                pend.wait()
            sweep(_border_regions)
            self._pending = self.exchange(1 - k)
        for s in self.subs.values():
            s.grid.cur = 1 - k
            s.grid.iteration += ns
        self.iteration += ns

    # -- native loop (RCCL + HIP, no per-step Python) ---------------------
    def _sub_plan(self, r: int, s: _Sub) -> dict:
        """Index plan of one subdomain for the native loop (element offsets
        and regions in its own grid coordinates)."""
        g, b = s.grid, s.blk
        H, ny, nx, pitch = g.H, g.ny, g.nx, g.pitch
        D = self.tblock * g.B
        interior = list(_interior_regions(s, D))
        border = list(_border_regions(s, D))
        rows, cols = [], []
        for side in ("top", "bottom"):
            peer = getattr(b, side)
            if peer >= 0:
                send = (ny if side == "top" else H) * pitch
                recv = (ny + H if side == "top" else 0) * pitch
                rows.append((peer, send, recv, H * pitch))
        # staged blocks: {peer, send_x, send_y, recv_x, recv_y, rows, width},
        # in the mirrored canonical order of exchange(): left, the corners
        # (-1,-1) (-1,1) (1,-1) (1,1), right -- block i and block n-1-i face
        # opposite ways, which is what lets the native transports post the
        # receives in reverse order and match repeated peers correctly
        def col(side):
            sx = nx if side == "right" else H
            rx = nx + H if side == "right" else 0
            return (getattr(b, side), sx, H, rx, H, ny, H)

        if b.left >= 0:
            cols.append(col("left"))
        for (dx, dy), peer in s.diag.items():
            sx, sy = s.corner_origin(dx, dy, True)
            rx, ry = s.corner_origin(dx, dy, False)
            cols.append((peer, sx, sy, rx, ry, H, H))
        if b.right >= 0:
            cols.append(col("right"))
        stage_elems = 2 * sum(c[5] * c[6] for c in cols)
        return {
            "interior": torch.tensor(np.array(interior, dtype=np.int32).reshape(-1, 4)),
            "border": torch.tensor(np.array(border, dtype=np.int32).reshape(-1, 4)),
            "ext": torch.tensor(np.array(_ext_region(s), dtype=np.int32)),
            "rows": torch.tensor(np.array(rows, dtype=np.int64).reshape(-1, 4)),
            "cols": torch.tensor(np.array(cols, dtype=np.int32).reshape(-1, 7)),
            "stage": torch.empty(max(stage_elems, 1), dtype=g.dtype, device=g.device),
        }

    def _native_plan(self):
        """ctypes array of SubDesc (one per local subdomain) + the tensors it
        points into (kept alive with it)."""
        if getattr(self, "_plan", None) is not None:
            return self._plan
        plans = {r: self._sub_plan(r, s) for r, s in self.subs.items()}
        arr = (SubDesc * len(plans))()
        for i, (r, s) in enumerate(self.subs.items()):
            pl, g = plans[r], s.grid
            d = arr[i]
            d.buf[0], d.buf[1] = g.buf[0].data_ptr(), g.buf[1].data_ptr()
            d.pitch, d.gy = g.pitch, g.gy
            d.interior, d.n_int = pl["interior"].data_ptr(), pl["interior"].shape[0]
            d.border, d.n_b = pl["border"].data_ptr(), pl["border"].shape[0]
            d.ext = pl["ext"].data_ptr()
            d.rows, d.n_rows = pl["rows"].data_ptr(), pl["rows"].shape[0]
            d.blks, d.n_blks = pl["cols"].data_ptr(), pl["cols"].shape[0]
            d.stage = pl["stage"].data_ptr()
            d.rank = r
            d.ipc = None
        self._plan = {"subs": arr, "plans": plans}
        return self._plan

    def _ipc_plan(self, ipc):
        """Build (once per :class:`~cme213x.parallel.ipc.NativeIpc`) the
        transport-3 plan of this process's subdomain: export its grid, staging
        and epoch words, all-gather every rank's descriptors and exchange plan,
        map the neighbours' memory and find, for each halo piece, where the
        neighbour keeps the data destined to us. Collective over ipc's group."""
        st = getattr(self, "_ipc", None)
        if st is not None and st["ipc"] is ipc:
            return st
        if len(self.subs) != 1:
            raise ValueError("IPC transport: one subdomain per process")
        (r, s), = self.subs.items()
        pl = self._native_plan()["plans"][r]
        g = s.grid
        flags = torch.zeros(32, dtype=torch.int32, device=g.device)
        rows = [list(map(int, x)) for x in pl["rows"].tolist()]
        cols = [list(map(int, x)) for x in pl["cols"].tolist()]
        neigh = sorted({x[0] for x in rows} | {c[0] for c in cols})
        if len(neigh) > 8:
            raise ValueError("IPC transport: at most 8 neighbours")
        info = {"rank": r, "buf": ipc.export(g.buf), "stage": ipc.export(pl["stage"]), "flags": ipc.export(flags),
                "state_bytes": g.buf[0].numel() * g.buf.element_size(), "rows": rows, "cols": cols, "neigh": neigh}
        torch.cuda.synchronize(g.device)  # epoch words are zero before any peer can map them
        by_rank = {i["rank"]: i for i in ipc.allgather_object(info)}
        plan = IpcPlan()
        plan.npeer = len(neigh)
        for j, p in enumerate(neigh):
            pi = by_rank[p]
            d = plan.peer[j]
            b0 = ipc.open(*pi["buf"])
            d.buf[0], d.buf[1] = b0, b0 + pi["state_bytes"]
            d.stage = ipc.open(*pi["stage"])
            d.flags = ipc.open(*pi["flags"])
            d.rank, d.slot = p, pi["neigh"].index(r)
        # piece i of ours receives what the peer sends in ITS k-th piece
        # toward us, k = i's rank among our pieces from that peer counted in
        # reverse order (the RCCL transport's matching, _recv_match)
        row_src = (ctypes.c_longlong * max(1, len(rows)))()
        for i, x in enumerate(rows):
            pr = by_rank[x[0]]["rows"]
            m = _recv_match(rows, i, pr, r)
            if m < 0 or pr[m][3] != x[3]:
                raise RuntimeError(f"rank {r}: inconsistent row halo plan with rank {x[0]}")
            row_src[i] = pr[m][1]
        blk_src = (ctypes.c_longlong * max(1, len(cols)))()
        for i, c in enumerate(cols):
            pc = by_rank[c[0]]["cols"]
            m = _recv_match(cols, i, pc, r)
            if m < 0 or list(pc[m][5:7]) != list(c[5:7]):
                raise RuntimeError(f"rank {r}: inconsistent block halo plan with rank {c[0]}")
            blk_src[i] = sum(y[5] * y[6] for y in pc[:m])
        epoch = ctypes.c_longlong(0)
        plan.flags = flags.data_ptr()
        plan.timeout = flags.data_ptr() + 4 * _IPC_TIMEOUT_WORD
        plan.epoch = ctypes.addressof(epoch)
        plan.row_src, plan.blk_src = ctypes.addressof(row_src), ctypes.addressof(blk_src)
        st = {"ipc": ipc, "plan": plan, "flags": flags, "epoch": epoch, "row_src": row_src, "blk_src": blk_src}
        ipc.keep(flags, pl["stage"], g.buf)
        self._ipc = st
        return st

    def ipc_check(self) -> None:
        """Raise if a wait of the IPC transport gave up on a peer (a peer that
        died or never signalled: the kernels stop waiting instead of hanging
        the GPU, and the state is then invalid)."""
        st = getattr(self, "_ipc", None)
        if st is None:
            return
        torch.cuda.synchronize(st["flags"].device)
        if int(st["flags"][_IPC_TIMEOUT_WORD].item()) != 0:
            raise RuntimeError("IPC halo exchange timed out waiting for a peer; state is invalid")

    def gate_check(self) -> None:
        """Raise if a border workgroup of the fused native schedule
        (CME_DIST_SCHEDULE=2) stopped waiting for a halo exchange that never
        signalled (bounded in-kernel wait; the state is then invalid)."""
        import ctypes

        from .. import _ext

        t = ctypes.c_int(0)
        _ext.call_hip("cme_heat_dist_gate_status", ctypes.addressof(t))
        if t.value:
            raise RuntimeError("fused native schedule: a border wait for the halo exchange timed out; state is invalid")

    def run_native(self, iters: int, rccl=None, sync: bool | None = None, transport: int | None = None,
                   ipc=None, fused: bool = True) -> None:
        """``iters`` timesteps in ONE native call (``cme_heat_dist_run``):
        border strips on their own stream, the halo exchange posted as soon
        as they finish, the deep interior overlapping both; with ``tblock=n``
        (2-4) each exchange of nB-deep halos feeds n timesteps done in one
        HBM pass. ``rccl``: a :class:`~cme213x.parallel.rccl.NativeRccl` (one
        subdomain per process); ``None`` = loopback transport, every
        neighbour being another local subdomain (device copies) -- the same
        stream/event schedule, testable on one GPU. ``transport=2`` skips
        the exchange (compute-schedule benchmarking only). ``fused=False``
        forbids the fused one-launch schedule for this call (schedule 0:
        streams + events); the native loop also drops it by itself under
        stream capture or when its queue-independence probe fails
        (:meth:`schedule` reports what ran). Under ``CME_SYNC_CHECK`` every
        call ends with :meth:`gate_check` / :meth:`ipc_check`, so a timed-out
        in-kernel wait raises here instead of leaving a wrong state behind."""
        import ctypes

        from .. import _ext

        if self.tblock > 4:
            raise ValueError("the native loop runs 1-4 steps per pass (tblock 5-6: solo grids, run())")
        if rccl is not None and len(self.subs) != 1:
            raise ValueError("RCCL transport: one subdomain per process")
        if rccl is not None and ipc is not None:
            raise ValueError("choose one transport: rccl or ipc")
        self.finish()
        sync = self.p.sync if sync is None else sync
        plan = self._native_plan()
        g0 = next(iter(self.subs.values())).grid
        cur_out = ctypes.c_int(0)
        if transport is None:
            transport = 0 if rccl is not None else (3 if ipc is not None else 1)
        plan["subs"][0].ipc = ctypes.addressof(self._ipc_plan(ipc)["plan"]) if transport == 3 else None
        _ext.call_hip("cme_heat_dist_run", transport, rccl.handle if rccl is not None else None,
                      ctypes.addressof(plan["subs"]), len(self.subs), 0 if g0.dtype == torch.float32 else 1,
                      g0.order, g0.xcfl, g0.ycfl, iters, g0.cur, int(sync), 0, self.tblock,
                      self._flags() | (0 if fused else 4), ctypes.addressof(cur_out), _ext.stream_ptr(g0.device))
        for s in self.subs.values():
            s.grid.cur = cur_out.value
            s.grid.iteration += iters
        self.iteration += iters
        if _ext.SYNC_CHECK:
            self.gate_check()
            if transport == 3:
                self.ipc_check()

    @staticmethod
    def schedule() -> dict:
        """What the last native run on this device used: ``schedule`` = "events"
        (0: border / comm / interior streams), "one-stream" (1), "fused" (2:
        one gated launch per pass), "sync" (3); ``probe`` = the fused
        schedule's queue-independence probe ("passed" / "failed" /
        "not run")."""
        from .. import _ext

        sch, probe = ctypes.c_int(-1), ctypes.c_int(0)
        _ext.call_hip("cme_heat_dist_info", ctypes.addressof(sch), ctypes.addressof(probe))
        names = {-1: "none", 0: "events", 1: "one-stream", 2: "fused", 3: "sync"}
        return {"schedule": names.get(sch.value, str(sch.value)),
                "probe": {1: "passed", -1: "failed"}.get(probe.value, "not run")}

    def finish(self) -> None:
        pend = getattr(self, "_pending", None)
        if pend is not None:
            pend.wait()
            self._pending = None

    def solo(self) -> bool:
        """One GPU subdomain with no neighbour on any side (world 1): nothing
        to exchange, so :meth:`run` hands the whole time loop to the native
        multi-pass driver (``cme_heat_run_*``) -- one call, no per-pass Python."""
        if self.device.type != "cuda" or len(self.subs) != 1:
            return False
        b = next(iter(self.subs.values())).blk
        return b.top < 0 and b.bottom < 0 and b.left < 0 and b.right < 0

    def run_variant(self) -> str:
        """``heat_run`` variant with this solver's pass schedule: ``tblock``
        steps per HBM pass on the chosen pass kernel, FMA or exact."""
        if self.tblock == 1:
            return self.variant
        if self.arith == 2:
            return f"pipe{self.tblock}_fast"
        suffix = "_fma" if self.fma else ""
        if self.kernel == "tile":
            return f"tile{self.tblock}" + suffix
        if self.tblock == 2:
            return "stream2" + suffix
        return ("pipe" if self.kernel == "pipe" else "stream") + str(self.tblock) + suffix

    # -- native loop selection (run) ------------------------------------
    def enable_native(self, transport: str | None = None, fused: bool = True) -> dict:
        """One-time, collective setup of the native loop that :meth:`run`
        uses on the GPU (``native="auto"`` / ``"on"``). Transports are tried
        in order until one passes (:func:`choose_native_transport`):

        * every subdomain in this process: loopback;
        * an ``nccl`` group: RCCL, then IPC-mapped peers (the neighbours'
          grids mapped with hipIpcOpenMemHandle and pulled over xGMI);
        * a ``gloo`` group on the GPU (the shared-GPU rehearsal): IPC;
        * ``transport``: one kind ("rccl", "ipc") or a comma-separated chain
          ("rccl,ipc").

        Each candidate is opened and then checked bit for bit against the
        Python loop on a small problem of the same decomposition
        (:func:`native_selftest`): with the fused one-launch schedule, then
        schedule 0. Every rank agrees on every step, so all ranks move to the
        next candidate together and none is left alone in a collective. If
        none passes, ``"auto"`` leaves :meth:`run` on the torch.distributed
        loop and ``"on"`` raises. Returns :attr:`native_info`, with the
        chain's record under ``"attempts"`` (hw/hw5/2dHeat_solution.cpp:
        630-664 is the reference's one, MPI-only, multi-process run)."""
        if self.native_info is not None:
            return self.native_info
        info = {"loop": "python", "transport": None, "fused_allowed": False, "selftest": None, "schedule": None,
                "attempts": []}
        self.native_info = info
        if self.native_mode == "off" or self.device.type != "cuda" or self.solo():
            return info
        from .. import _ext

        def agree(ok: bool) -> bool:
            t = torch.tensor([1.0 if ok else 0.0], device=self.device)
            self.comm.allreduce_(t, "min")
            return bool(t.item() == 1.0)

        # RCCL may be asked for at world 1 too (a periodic grid's halos are
        # then self-sends); IPC needs other processes to map
        if self.comm.size > 1 or transport is not None:
            backend = getattr(self.comm, "backend", None)
            kinds = (transport.split(",") if transport else (["rccl", "ipc"] if backend == "nccl" else ["ipc"]))
        else:
            kinds = ["loopback"]
        group = getattr(self.comm, "group", None)

        def open_transport(kind):
            if kind == "loopback":
                return None
            if kind == "rccl":
                from ..parallel.rccl import NativeRccl

                return NativeRccl(group)
            if kind == "ipc":
                from ..parallel.ipc import NativeIpc

                return NativeIpc(group)
            raise ValueError(f"unknown native transport {kind!r}")

        def release(kind, handle):
            if handle is None:
                return
            if kind == "rccl":
                handle.abort()  # pending native sends/recvs fail on the peers instead of hanging
            elif kind == "ipc":
                handle.close()  # collective: every rank reached the self-test with a handle

        kind, handle, fused_ok, attempts = choose_native_transport(
            kinds, agree, _ext.hip, open_transport, lambda k, h, f: native_selftest(self, k, h, f), release,
            (True, False) if fused else (False,), f"DistHeat rank {self.comm.rank}")
        info["attempts"] = attempts
        if kind is None:
            if self.native_mode == "on":
                raise RuntimeError(f"native distributed loop failed its setup or bitwise self-test ({attempts})")
            return info
        self._native = (kind, handle)
        info.update(loop="native", transport=kind, fused_allowed=fused_ok, selftest=True)
        return info

    def _run_native_selected(self, iters: int, sync: bool | None) -> None:
        kind, handle = self._native
        fused = self.native_info["fused_allowed"]
        if kind == "rccl":
            self.run_native(iters, handle, sync=sync, fused=fused)
        elif kind == "ipc":
            self.run_native(iters, ipc=handle, sync=sync, fused=fused)
        else:
            self.run_native(iters, sync=sync, fused=fused)
        self.native_info["schedule"] = self.schedule()["schedule"]

    def check_native(self) -> None:
        """After the caller's final sync: raise if the native loop's bounded
        in-kernel waits gave up (fused border gate, IPC epochs) or RCCL
        reported an asynchronous error. The sticky words live in pinned host
        memory, so this costs one device sync."""
        kind, handle = getattr(self, "_native", (None, None))
        self.gate_check()
        if kind == "ipc":
            self.ipc_check()
        elif kind == "rccl":
            handle.check()

    def close_native(self) -> None:
        """Release the native transport (collective for IPC)."""
        kind, handle = getattr(self, "_native", (None, None))
        self._native = (None, None)
        if handle is not None:
            handle.close()

    def run(self, iters: int, sync: bool | None = None) -> None:
        """``iters`` timesteps. One GPU subdomain with no neighbour: one
        native multi-pass call. Otherwise, on the GPU with ``native="auto"``
        / ``"on"``: the native C++ loop (after :meth:`enable_native`'s
        self-test), whose in-kernel waits are checked -- and raise -- at the
        end of every call; else the Python loop below (any backend)."""
        if self.solo():
            self.finish()
            s = next(iter(self.subs.values()))
            g = s.grid
            a, b = g.buf[g.cur], g.buf[1 - g.cur]
            out = heat_run(a, b, g.interior, g.order, g.xcfl, g.ycfl, iters, self.run_variant())
            g.cur = g.cur if out is a else 1 - g.cur
            g.iteration += iters
            self.iteration += iters
            return
        if self.native_mode != "off" and self.device.type == "cuda" and iters > 0:
            if self.enable_native()["loop"] == "native":
                self._run_native_selected(iters, sync)
                self.check_native()
                return
        i = 0
        while iters - i >= 2 and self.tblock >= 2:
            ns = min(self.tblock, iters - i)
            self.stepn(ns, sync)
            i += ns
        for _ in range(i, iters):
            self.step(sync)
        self.finish()

    # -- checkpoint / restart ---------------------------------------------
    def _meta(self, r: int) -> dict:
        g = self.subs[r].grid
        return {"iteration": self.iteration, "rank": r, "world": self.world, "nx": self.p.nx, "ny": self.p.ny,
                "order": self.p.order, "grid_method": self.p.grid_method, "dtype": str(g.dtype),
                "local_nx": g.nx, "local_ny": g.ny}

    def checkpoint(self, directory: str) -> list[str]:
        """Lossless per-subdomain restart files ``<dir>/heat_rank<r>.safetensors``
        (owned interior + iteration counter + decomposition). The reference
        has no restart path, only lossy text dumps."""
        import os

        self.finish()
        os.makedirs(directory, exist_ok=True)
        prev = _ACTIVE_WRITERS.get(os.path.realpath(directory))
        if prev is not None:
            prev._thread.join()  # an asynchronous checkpoint into the same files is still writing
        paths = []
        for r, s in self.subs.items():
            g = s.grid
            H = g.H
            own = g.buf[g.cur, H:H + g.ny, H:H + g.nx].cpu().numpy()
            path = os.path.join(directory, f"heat_rank{r}.safetensors")
            _save_atomic(path, {"interior": own}, self._meta(r))
            paths.append(path)
        return paths

    def checkpoint_async(self, directory: str) -> "CheckpointWriter":
        """:meth:`checkpoint` off the critical path. The owned interiors are
        snapshotted on the device (one device copy each, waited for before
        returning, so the time loop may overwrite the grids at once); the
        snapshots go to pinned host memory on a side stream and a background
        thread writes the same files as :meth:`checkpoint` once that copy has
        landed. ``.wait()`` returns the paths (and re-raises a write error)."""
        import os

        self.finish()
        os.makedirs(directory, exist_ok=True)
        snaps = []
        for r, s in self.subs.items():
            g = s.grid
            H = g.H
            snaps.append((r, g.buf[g.cur, H:H + g.ny, H:H + g.nx].clone(), self._meta(r)))
        event = None
        if self.device.type == "cuda":
            cur = torch.cuda.current_stream(self.device)
            cur.synchronize()  # snapshots complete: the grids are free again
            side = torch.cuda.Stream(self.device)
            host = []
            with torch.cuda.stream(side):
                for r, snap, meta in snaps:
                    h = torch.empty(snap.shape, dtype=snap.dtype, pin_memory=True)
                    h.copy_(snap, non_blocking=True)
                    host.append((r, h, meta, snap))  # snap kept alive until the copy is done
            event = torch.cuda.Event()
            event.record(side)
            snaps = host
        else:
            snaps = [(r, t, meta, None) for r, t, meta in snaps]
        return CheckpointWriter(directory, snaps, event)

    def restore(self, directory: str) -> None:
        """Load :meth:`checkpoint` files written by a run with the same global
        problem and decomposition, then refresh every halo."""
        import os

        from ..utils.gridio import load_checkpoint

        self.finish()
        its = set()
        for r, s in self.subs.items():
            t, meta = load_checkpoint(os.path.join(directory, f"heat_rank{r}.safetensors"))
            want = {k: str(v) for k, v in self._meta(r).items() if k != "iteration"}
            got = {k: meta.get(k) for k in want}
            if got != want:
                raise ValueError(f"checkpoint does not match this run: {got} != {want}")
            g = s.grid
            H = g.H
            own = torch.from_numpy(t["interior"]).to(g.device)
            g.buf[:, H:H + g.ny, H:H + g.nx] = own
            g.iteration = int(meta["iteration"])
            its.add(int(meta["iteration"]))
        if len(its) != 1:
            raise ValueError("subdomain checkpoints from different iterations")
        self.iteration = its.pop()
        # the native / IPC plans depend on geometry only: kept (peers' IPC
        # mappings of our grid and staging stay valid)
        self.exchange(self._cur()).wait()

    # -- io ------------------------------------------------------------------
    def save_text(self, identifier: str) -> None:
        from ..utils.gridio import write_grid

        for r, s in self.subs.items():
            write_grid(f"grid{r}_{identifier}.txt", s.grid.state(), extra_endl=True)

    def gather_global(self) -> np.ndarray:
        """Assemble the global (gy, gx) state on the host from the local subs
        (single-process use, or rank-0 after an all-gather by the caller)."""
        p = self.p
        B = p.border
        out = np.zeros((p.ny + 2 * B, p.nx + 2 * B), dtype=np.float64)
        for s in self.subs.values():
            b, st = s.blk, s.grid.state()
            out[B + b.y0:B + b.y0 + b.ny, B + b.x0:B + b.x0 + b.nx] = st[B:B + b.ny, B:B + b.nx]
        return out


def native_setup_agreement(agree, load_lib, open_transport, who: str = "", kind: str = "") -> tuple[bool, object]:
    """The collective first half of :meth:`DistHeat.enable_native`: load the
    native library, then (``open_transport`` not None) open the transport,
    each step followed by ``agree`` (an all-rank AND). Every rank makes the
    same number of ``agree`` calls and returns the same ``ok`` -- a rank whose
    library loaded falls back with a peer whose library did not, instead of
    entering the self-test's collectives alone. Returns
    ``(ok, handle)``; the handle of a transport opened on a rank whose peer
    failed is returned too, so the caller can abort it."""
    try:
        load_lib()
        ok = True
    except Exception as e:  # noqa: BLE001 - reported; every rank falls back together
        print(f"{who}: native library unavailable ({e})", flush=True)
        ok = False
    ok = agree(ok)
    handle = None
    if ok and open_transport is not None:
        try:
            handle = open_transport()
        except Exception as e:  # noqa: BLE001
            print(f"{who}: native {kind} transport unavailable ({e})", flush=True)
            ok = False
        ok = agree(ok)
    return ok, handle


def choose_native_transport(kinds, agree, load_lib, open_transport, selftest, release, schedules=(True, False),
                            who: str = "") -> tuple:
    """The transport chain of :meth:`DistHeat.enable_native` (collective).
    Loads the native library once, then for each kind in ``kinds``: opens it
    (``open_transport(kind)``) and runs ``selftest(kind, handle, fused)``
    for each schedule in ``schedules`` (fused first) until one passes --
    every step followed by ``agree`` (an all-rank AND), so every rank makes
    the same calls and moves to the next kind together. A kind whose
    self-test failed on any rank is released (``release(kind, handle)``:
    RCCL abort, IPC unmap) before the next is opened. Returns ``(kind,
    handle, fused, attempts)`` -- ``kind`` None if no candidate passed --
    with ``attempts`` = [{"transport", "result"[, "fused"]}] in the order
    tried (result "ok", "library", "setup" or "selftest")."""
    attempts = []
    ok, _ = native_setup_agreement(agree, load_lib, None, who)
    if not ok:
        return None, None, False, [{"transport": kinds[0] if kinds else None, "result": "library"}]
    for kind in kinds:
        ok, handle = native_setup_agreement(agree, lambda: None, lambda k=kind: open_transport(k), who, kind)
        if not ok:
            # a communicator this rank opened while a peer failed: RCCL's
            # abort is local; an IPC handle holds no mapping yet
            if handle is not None and kind == "rccl":
                release(kind, handle)
            attempts.append({"transport": kind, "result": "setup"})
            continue
        for f in schedules:
            try:
                good = selftest(kind, handle, f)
            except Exception as e:  # noqa: BLE001 - e.g. the gated grid refused, a timed-out wait
                print(f"{who}: native {kind} self-test raised ({e})", flush=True)
                good = False
            if agree(good):
                attempts.append({"transport": kind, "result": "ok", "fused": f})
                return kind, handle, f, attempts
        attempts.append({"transport": kind, "result": "selftest"})
        release(kind, handle)
    return None, None, False, attempts


def native_selftest(sim: "DistHeat", kind: str, handle, fused: bool, n: int = 1024) -> bool:
    """Bitwise self-test of the native loop for ``sim``'s decomposition and
    pass schedule (collective). A problem of at most ``n``^2 points with the
    same world, method, periodicity, dtype, steps per pass, kernel and FMA
    mode, and a non-uniform interior (a stale or misplaced halo changes the
    answer), runs ``2*tblock + 1`` steps (whole passes plus a tail) through
    the native loop on transport ``kind`` and through the Python loop's
    single steps; True on this rank if they agree bit for bit and no
    in-kernel wait gave up. A native run that does not finish in 60 s
    fails."""
    p0 = sim.p
    iters = 2 * sim.tblock + 1
    p = SimParams(nx=min(p0.nx, n), ny=min(p0.ny, n), iters=iters, order=p0.order, ic=5.0,
                  bc=(0.0, 10.0, 3.0, 7.0), grid_method=p0.grid_method, sync=p0.sync, flavor="hw5")
    dt = next(iter(sim.subs.values())).grid.dtype
    kw = dict(local_ranks=list(sim.local_ranks), world=sim.world, periodic=sim.periodic, fma=sim._fma_arg())
    a = DistHeat(p, sim.comm, dt, sim.device, tblock=sim.tblock, kernel=sim.kernel, **kw)
    b = DistHeat(p, sim.comm, dt, sim.device, tblock=1, **kw)
    for d in (a, b):
        for s in d.subs.values():
            g, H = s.grid, s.grid.H
            yy = torch.arange(s.blk.ny, device=sim.device, dtype=dt).view(-1, 1) + s.blk.y0
            xx = torch.arange(s.blk.nx, device=sim.device, dtype=dt).view(1, -1) + s.blk.x0
            g.buf[:, H:H + s.blk.ny, H:H + s.blk.nx] = 5.0 + torch.sin(0.05 * xx) * torch.cos(0.03 * yy)
        d.exchange(d._cur()).wait()
    if kind == "rccl":
        a.run_native(iters, handle, fused=fused)
    elif kind == "ipc":
        a.run_native(iters, ipc=handle, fused=fused)
    else:
        a.run_native(iters, fused=fused)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(sim.device))
    t_end = time.perf_counter() + 60.0
    while not ev.query():
        if time.perf_counter() > t_end:
            raise TimeoutError("native self-test run did not finish within 60 s")
        time.sleep(0.002)
    a.gate_check()
    if kind == "ipc":
        a.ipc_check()
    b.run(iters)
    torch.cuda.synchronize(sim.device)
    def own(s):
        g, H = s.grid, s.grid.H
        return g.buf[g.cur, H:H + g.ny, H:H + g.nx]

    same = all(torch.equal(own(sa), own(sb)) for sa, sb in zip(a.subs.values(), b.subs.values()))
    if kind == "ipc":
        # a's plan mapped the peers' test grids; drop those mappings before
        # the test solvers' memory is freed (collective)
        handle.close()
    return same


def _recv_match(mine: list, i: int, theirs: list, me: int) -> int:
    """Index in the peer's piece list ``theirs`` of the send that our piece
    ``i`` receives: receives are posted in reverse order, sends in forward
    order, so the k-th receive from a peer (counting our pieces i+1.. from
    it first) pairs with its k-th send to ``me``. -1 if there is none."""
    peer = mine[i][0]
    k = sum(1 for x in mine[i + 1:] if x[0] == peer)
    idx = [j for j, y in enumerate(theirs) if y[0] == me]
    return idx[k] if k < len(idx) else -1


def _inner_box(s: _Sub, depth: int):
    """Owned region shrunk by ``depth`` on every side that has a neighbour."""
    g, b = s.grid, s.blk
    H = g.H
    xb = H + depth if b.left >= 0 else H
    xe = H + g.nx - depth if b.right >= 0 else H + g.nx
    yb = H + depth if b.bottom >= 0 else H
    ye = H + g.ny - depth if b.top >= 0 else H + g.ny
    return xb, xe, yb, ye


def _interior_regions(s: _Sub, depth: int):
    """Deep interior: points whose ``depth``-wide dependency cone (B for one
    step, 2B for two) touches no ghost cell filled by a neighbour
    (physical-BC ghosts are constant and always valid)."""
    xb, xe, yb, ye = _inner_box(s, depth)
    if xe > xb and ye > yb:
        yield (xb, xe, yb, ye)


def _border_regions(s: _Sub, depth: int):
    g = s.grid
    H = g.H
    xb, xe, yb, ye = _inner_box(s, depth)
    X0, X1, Y0, Y1 = H, H + g.nx, H, H + g.ny
    if xe <= xb or ye <= yb:  # subdomain thinner than two cones: one region
        yield (X0, X1, Y0, Y1)
        return
    if yb > Y0:
        yield (X0, X1, Y0, yb)  # bottom strip, full width
    if ye < Y1:
        yield (X0, X1, ye, Y1)  # top strip, full width
    if xb > X0:
        yield (X0, xb, yb, ye)  # left strip
    if xe < X1:
        yield (xe, X1, yb, ye)  # right strip


def _ext_region(s: _Sub):
    """Region of the intermediate steps of a multi-step pass: the owned region
    grown by ``H - B`` (= (tblock-1)*B) into the halo on every neighbour side
    -- the dependency cone of the first intermediate step; later steps need
    less. Physical-BC sides stay fixed."""
    g, b = s.grid, s.blk
    H, B = g.H, g.B
    D = H - B
    return (H - D if b.left >= 0 else H, H + g.nx + D if b.right >= 0 else H + g.nx,
            H - D if b.bottom >= 0 else H, H + g.ny + D if b.top >= 0 else H + g.ny)


def run_hw5(params_path: str, comm: Comm | None = None, dtype=torch.float64, device: str | None = None,
            write_files: bool = True, tblock: int | str = "auto", fma: bool = False, kernel: str = "auto",
            native: str = "auto", local_ranks: list[int] | None = None, world: int | None = None,
            periodic: tuple[bool, bool] = (False, False), transport: str | None = None) -> dict:
    """The hw5 driver (double precision, as the reference). On the GPU the
    steps per pass and the pass kernel are chosen from the subdomain size
    (:func:`auto_tblock`, :func:`auto_kernel`); ``fma=False`` keeps the
    reference CPU's uncontracted arithmetic. With neighbours on the GPU the
    time loop is the native C++ loop (``native="auto"``: after its bitwise
    self-test, else the Python loop; rank 0 logs which); an in-kernel wait
    that gave up raises ``RuntimeError`` after the run.
    ``local_ranks``/``world``: several subdomains in this process
    (``heat2d_mpi --ranks N``)."""
    comm = comm or LoopbackComm()
    p = SimParams.from_file(params_path, flavor="hw5")
    if comm.rank == 0:
        print(p.banner())
    device = device or ("cuda" if torch.cuda.is_available() else "cpu")
    sim = DistHeat(p, comm, dtype, device, tblock=tblock, fma=fma, kernel=kernel, native=native,
                   local_ranks=local_ranks, world=world, periodic=periodic)
    if write_files:
        sim.save_text("init")
    if sim.device.type == "cuda":
        info = sim.enable_native(transport)
        if comm.rank == 0 and not sim.solo():
            print(f"time loop: {info['loop']}" + (f" ({info['transport']} transport, bitwise self-test passed, "
                                                   f"fused schedule {'allowed' if info['fused_allowed'] else 'off'})"
                                                   if info["loop"] == "native" else ""), flush=True)
        torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    sim.run(p.iters)
    if sim.device.type == "cuda":
        torch.cuda.synchronize()
    comm.barrier()
    secs = time.perf_counter() - t0
    if comm.rank == 0:
        print(f"{p.iters} iterations on a {p.nx} by {p.ny} grid took: {secs} seconds.")
        if sim.native_info and sim.native_info.get("schedule"):
            print(f"native schedule: {sim.native_info['schedule']}", flush=True)
    if write_files:
        sim.save_text("final")
    return {"seconds": secs, "sim": sim}
