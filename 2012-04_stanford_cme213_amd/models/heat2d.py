"""2-D heat diffusion on one device (the hw2 workload) -- the framework's
minimum end-to-end slice.

:class:`HeatGrid` is the MI355X-first re-design of the reference's ``Grid<T>``
(``hw/hw2/solution/2dHeat_solution.cu:213-331``): both ping-pong states live
in ONE device allocation ``(2, gy, pitch)`` with ``pitch`` rounded up to 64
elements (256-B aligned rows for 16-B vector lanes), boundary values are
written into both states once, and sweeps are enqueued back-to-back with no
host synchronisation (the reference synchronises after every launch).

``run_hw2`` reproduces the hw2 driver: params banner, ``grid_init.txt``, CPU
reference, global and shared(LDS) GPU sweeps plus the register-streaming
kernel, 10-ULP interior check, ``grid_final_gpu.txt`` / ``grid_final_cpu.txt``
and the ``"<name> took X ms"`` lines (``:713-747``).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops.stencil import heat_run, heat_step
from ..utils.gridio import load_checkpoint, save_checkpoint, write_grid
from ..utils.params import SimParams
from ..utils.timer import EventTimer
from ..utils.ulp import ulp_distance


def pitch_for(gx: int) -> int:
    return (gx + 63) // 64 * 64


class HeatGrid:
    """Ping-pong grid state for an ``nx`` x ``ny`` interior with a halo of
    ``border`` cells. ``bc_sides`` selects which sides carry the physical
    boundary condition (all four for a single device; the distributed driver
    passes only the sides with no neighbour, as ``hw/hw5/2dHeat_solution.cpp``
    does). ``halo`` (default ``border``) is the allocated ghost depth ``H``;
    the distributed driver uses ``H = 2*border`` so one exchange feeds two
    timesteps (temporal blocking). Only the inner ``border`` ghost layers are
    ever read on physical sides; :meth:`state` always returns the
    reference-layout grid with a ``border``-deep halo."""

    def __init__(self, params: SimParams, dtype=torch.float32, device="cpu", nx: int | None = None,
                 ny: int | None = None, bc_sides=(True, True, True, True), halo: int | None = None):
        self.params = params
        self.dtype = dtype
        self.device = torch.device(device)
        self.order = params.order
        self.B = params.border
        self.nx = params.nx if nx is None else nx
        self.ny = params.ny if ny is None else ny
        self.H = self.B if halo is None else int(halo)
        if self.H < self.B:
            raise ValueError("halo must be at least the stencil border")
        if self.nx <= 2 * self.H or self.ny <= 2 * self.H:
            raise ValueError("local grid too small for the stencil order")
        self.gx = self.nx + 2 * self.H
        self.gy = self.ny + 2 * self.H
        self.pitch = pitch_for(self.gx)
        self.xcfl = float(np.dtype(np.float32 if dtype == torch.float32 else np.float64).type(params.xcfl))
        self.ycfl = float(np.dtype(np.float32 if dtype == torch.float32 else np.float64).type(params.ycfl))
        self.iteration = 0
        init = torch.full((self.gy, self.pitch), params.ic, dtype=dtype, device=self.device)
        top, left, bottom, right = bc_sides
        H, ny, nx = self.H, self.ny, self.nx
        # Same write order as the reference: rows first, then columns, so the
        # corners carry the left/right values.
        if bottom:
            init[:H, :self.gx] = params.bottom_bc
        if top:
            init[H + ny:H + ny + H, :self.gx] = params.top_bc
        if left:
            init[:, :H] = params.left_bc
        if right:
            init[:, H + nx:H + nx + H] = params.right_bc
        self.buf = torch.stack([init, init.clone()])
        self.cur = 0

    # -- state --------------------------------------------------------------
    @property
    def interior(self) -> tuple[int, int, int, int]:
        return (self.H, self.H + self.nx, self.H, self.H + self.ny)

    def curr(self) -> torch.Tensor:
        return self.buf[self.cur]

    def prev(self) -> torch.Tensor:
        return self.buf[1 - self.cur]

    def view(self, k: int | None = None) -> torch.Tensor:
        """Device view of state ``k`` (default current) in the reference layout:
        ``(ny + 2B, nx + 2B)`` -- interior plus a ``border``-deep halo."""
        k = self.cur if k is None else k
        o = self.H - self.B
        return self.buf[k, o:self.gy - o, o:self.gx - o]

    def state(self) -> np.ndarray:
        """Current (ny + 2B, nx + 2B) grid as a host array."""
        return self.view().cpu().numpy()

    # -- compute ------------------------------------------------------------
    def step(self, variant: str = "stream", region=None) -> None:
        src, dst = self.buf[self.cur], self.buf[1 - self.cur]
        heat_step(src, dst, region or self.interior, self.order, self.xcfl, self.ycfl, variant)
        self.cur = 1 - self.cur
        self.iteration += 1

    def run(self, iters: int, variant: str = "stream") -> None:
        a, b = self.buf[self.cur], self.buf[1 - self.cur]
        out = heat_run(a, b, self.interior, self.order, self.xcfl, self.ycfl, iters, variant)
        self.cur = self.cur if out is a else 1 - self.cur
        self.iteration += iters

    # -- io -----------------------------------------------------------------
    def save_text(self, identifier: str, prefix: str = "grid") -> str:
        path = f"{prefix}_{identifier}.txt"
        write_grid(path, self.state(), extra_endl=True)
        return path

    def checkpoint(self, path: str) -> None:
        """Lossless restartable state (both buffers incl. halos + iteration)."""
        save_checkpoint(path, {"state": self.buf[self.cur].cpu().numpy()},
                        {"iteration": self.iteration, "nx": self.nx, "ny": self.ny, "order": self.order,
                         "dtype": str(self.dtype)})

    def restore(self, path: str) -> None:
        t, meta = load_checkpoint(path)
        st = torch.from_numpy(t["state"]).to(self.device)
        if tuple(st.shape) != (self.gy, self.pitch):
            raise ValueError("checkpoint shape mismatch")
        self.buf[0].copy_(st)
        self.buf[1].copy_(st)
        self.cur = 0
        self.iteration = int(meta["iteration"])


def bytes_per_point(order: int, dtype=torch.float32) -> int:
    """Reference-convention traffic model (24/40/72 B per point per
    iteration for fp32 orders 2/4/8: every stencil tap + the store)."""
    taps = {2: 5, 4: 9, 8: 17}[order]
    return (taps + 1) * (4 if dtype == torch.float32 else 8)


def check_errors(cpu: np.ndarray, gpu: np.ndarray, border: int, max_ulps: int = 10) -> int:
    """10-ULP interior comparison; prints the first 10 mismatches like
    ``checkErrors`` (``hw/hw2/solution/2dHeat_solution.cu:690-710``)."""
    B = border
    a, b = cpu[B:-B, B:-B], gpu[B:-B, B:-B]
    d = ulp_distance(a, b)
    bad = np.argwhere(d > max_ulps)
    for (yy, xx) in bad[:10]:
        print(f"Mis-match at pos: ({xx + B}, {yy + B}) cpu: {a[yy, xx]:f}, gpu: {b[yy, xx]:f}")
    if len(bad):
        print(f"There were {len(bad)} total locations where there was a difference between the cpu and gpu")
    return int(len(bad))


def run_hw2(params_path: str, dtype=torch.float32, device: str | None = None, outdir: str = ".",
            variants=("global", "shared", "stream"), write_files: bool = True) -> dict:
    """The hw2 driver. Returns timings (ms) and mismatch counts per variant."""
    import os

    p = SimParams.from_file(params_path, flavor="hw2")
    print(p.banner())
    print(f"({p.nx}, {p.ny}) ({p.gx}, {p.gy})")
    device = device or ("cuda" if torch.cuda.is_available() else "cpu")
    tname = "float" if dtype == torch.float32 else "double"
    cwd = os.getcwd()
    os.makedirs(outdir, exist_ok=True)
    os.chdir(outdir)
    try:
        cpu_grid = HeatGrid(p, dtype, "cpu")
        if write_files:
            cpu_grid.save_text("init")
        # warm-up of the CPU oracle, as the GPU variants get below: the first
        # call pays the OpenMP runtime's thread start-up and the library load
        # (580 ms vs 0.3 ms warm at 200^2 x 10), which would
        # inflate every GPU-over-CPU speed-up on small grids
        HeatGrid(p, dtype, "cpu").run(1, "naive")
        t = EventTimer(f"cpu computation {tname}")
        with t:
            cpu_grid.run(p.iters, "naive")
        res = {"cpu_ms": t.ms, "variants": {}}
        ref = cpu_grid.state()
        last = None
        if device != "cpu":
            labels = {"global": f"gpu computation {tname}", "shared": f"shared gpu {tname}",
                      "stream": f"stream gpu {tname}", "lds_nopad": f"shared(no pad) gpu {tname}"}
            for v in variants:
                g = HeatGrid(p, dtype, device)
                g.run(1, v)  # warm-up: first-touch + code-object load
                g = HeatGrid(p, dtype, device)
                t = EventTimer(labels.get(v, v), device=device)
                with t:
                    g.run(p.iters, v)
                out = g.state()
                errs = check_errors(ref, out, p.border)
                res["variants"][v] = {"ms": t.ms, "errors": errs,
                                      "max_ulp": int(ulp_distance(ref, out).max())}
                if write_files:
                    write_grid(f"grid_final_gpu_{v}.txt", out, extra_endl=False)
                last = out
        if write_files:
            if last is not None:
                write_grid("grid_final_gpu.txt", last, extra_endl=False)
            cpu_grid.save_text("final_cpu")
        return res
    finally:
        os.chdir(cwd)
