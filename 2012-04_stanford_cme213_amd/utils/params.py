"""Parameter files for the heat-diffusion drivers.

Same whitespace-separated format as the reference:

* hw2 (single GPU, ``hw/hw2/solution/params.in``)::

      nx ny / lx ly / alpha / iters / order / ic / bcTop bcLeft bcBottom bcRight

* hw5 (distributed, ``hw/hw5/programming/params.in``) inserts ``gridMethod``
  (1 = 1-D stripes, 2 = 2-D blocks) and ``sync`` (1/0) after ``ic``.

The CFL-limited timestep follows ``simParams::calcDtCFL``
(``hw/hw2/solution/2dHeat_solution.cu:189-211``; hw5 uses slightly different
safety margins, ``hw/hw5/2dHeat_solution.cpp`` calcDtCFL). Values are computed
in double, as in the reference, and cast to the working dtype by the caller.
"""
from __future__ import annotations

from dataclasses import dataclass, field

_BORDER = {2: 1, 4: 2, 8: 4}

# (safety margin subtracted from .5, hw2 value, hw5 value) per order
_MARGIN_HW2 = {2: 0.0001, 4: 0.0001, 8: 0.0001}
_MARGIN_HW5 = {2: 0.001, 4: 0.001, 8: 0.01}


@dataclass
class SimParams:
    nx: int = 10
    ny: int = 10
    lx: float = 1.0
    ly: float = 1.0
    alpha: float = 1.0
    iters: int = 1000
    order: int = 2
    ic: float = 5.0
    bc: tuple = (0.0, 10.0, 0.0, 10.0)  # top, left, bottom, right (counter-clockwise)
    grid_method: int = 1
    sync: bool = True
    flavor: str = "hw2"  # which CFL margins to use
    dx: float = field(init=False)
    dy: float = field(init=False)
    dt: float = field(init=False)
    xcfl: float = field(init=False)
    ycfl: float = field(init=False)

    def __post_init__(self) -> None:
        if self.order not in _BORDER:
            raise ValueError(f"Unsupported discretization order: {self.order}")
        self.dx = self.lx / (self.nx - 1)
        self.dy = self.ly / (self.ny - 1)
        self._calc_dt_cfl()

    # -- derived ------------------------------------------------------------
    @property
    def border(self) -> int:
        return _BORDER[self.order]

    @property
    def gx(self) -> int:
        return self.nx + 2 * self.border

    @property
    def gy(self) -> int:
        return self.ny + 2 * self.border

    @property
    def top_bc(self) -> float:
        return self.bc[0]

    @property
    def left_bc(self) -> float:
        return self.bc[1]

    @property
    def bottom_bc(self) -> float:
        return self.bc[2]

    @property
    def right_bc(self) -> float:
        return self.bc[3]

    def _calc_dt_cfl(self) -> None:
        dx2, dy2, a = self.dx * self.dx, self.dy * self.dy, self.alpha
        m = (_MARGIN_HW5 if self.flavor == "hw5" else _MARGIN_HW2)[self.order]
        if self.order == 2:
            self.dt = (0.5 - m) * (dx2 * dy2) / (a * (dx2 + dy2))
            self.xcfl = (a * self.dt) / dx2
            self.ycfl = (a * self.dt) / dy2
        elif self.order == 4:
            self.dt = (0.5 - m) * (12 * dx2 * dy2) / (16 * a * (dx2 + dy2))
            self.xcfl = (a * self.dt) / (12 * dx2)
            self.ycfl = (a * self.dt) / (12 * dy2)
        else:
            self.dt = (0.5 - m) * (5040 * dx2 * dy2) / (8064 * a * (dx2 + dy2))
            self.xcfl = (a * self.dt) / (5040 * dx2)
            self.ycfl = (a * self.dt) / (5040 * dy2)

    # -- io -----------------------------------------------------------------
    @classmethod
    def from_file(cls, path: str, flavor: str = "hw2") -> "SimParams":
        with open(path) as f:
            tok = f.read().split()
        vals = iter(tok)
        nx, ny = int(next(vals)), int(next(vals))
        lx, ly = float(next(vals)), float(next(vals))
        alpha = float(next(vals))
        iters = int(next(vals))
        order = int(next(vals))
        ic = float(next(vals))
        grid_method, sync = 1, True
        if flavor == "hw5":
            grid_method = int(next(vals))
            sync = bool(int(next(vals)))
        bc = tuple(float(next(vals)) for _ in range(4))
        return cls(nx=nx, ny=ny, lx=lx, ly=ly, alpha=alpha, iters=iters, order=order, ic=ic, bc=bc,
                   grid_method=grid_method, sync=sync, flavor=flavor)

    def to_file(self, path: str) -> None:
        with open(path, "w") as f:
            f.write(f"{self.nx} {self.ny}\n{self.lx} {self.ly}\n{self.alpha}\n{self.iters}\n{self.order}\n{self.ic}\n")
            if self.flavor == "hw5":
                f.write(f"{self.grid_method}\n{int(self.sync)}\n")
            f.write(" ".join(str(b) for b in self.bc) + "\n")

    def banner(self) -> str:
        """The verbose parameter dump printed by the reference's simParams."""
        s = (f"nx: {self.nx} ny: {self.ny}\ngx: {self.gx} gy: {self.gy}\nlx {self.lx:f}: ly: {self.ly:f}\n"
             f"alpha: {self.alpha:f}\niterations: {self.iters}\norder: {self.order}\nic: {self.ic:f}\n")
        if self.flavor == "hw5":
            s += f"sync: {int(self.sync)}\ndomainDecomp: {self.grid_method}\n"
        s += f"dx: {self.dx:f} dy: {self.dy:f}\ndt: {self.dt:f} xcfl: {self.xcfl:f} ycfl: {self.ycfl:f}"
        return s
