"""Domain decomposition for the distributed stencil.

Reproduces the reference's two schemes (``hw/hw5/2dHeat_solution.cpp:282-331``):

* ``method=1``: 1-D horizontal stripes; rank r owns rows ``ny/P`` (+1 for the
  first ``ny % P`` ranks), neighbours r-1 (bottom) / r+1 (top).
* ``method=2``: 2-D blocks on a Px x Py process grid, ``rank = row*Px + col``.
  The reference only accepts square P; we accept any P and pick the most
  square factorisation (Px >= Py), which the reference calls "for now, only
  squares are valid" -- a strict superset.
"""
from __future__ import annotations

from dataclasses import dataclass


def _split(n: int, parts: int, idx: int) -> tuple[int, int]:
    """(offset, count) of part ``idx`` when ``n`` is split as in the reference."""
    base, rem = divmod(n, parts)
    count = base + (1 if idx < rem else 0)
    off = idx * base + min(idx, rem)
    return off, count


def proc_grid(P: int, method: int) -> tuple[int, int]:
    if method == 1:
        return 1, P
    best = (P, 1)
    for py in range(1, int(P ** 0.5) + 1):
        if P % py == 0:
            best = (P // py, py)
    return best


@dataclass
class Block:
    rank: int
    px: int
    py: int
    col: int
    row: int
    x0: int  # global interior offset (columns)
    y0: int  # global interior offset (rows)
    nx: int
    ny: int
    left: int = -1
    right: int = -1
    top: int = -1
    bottom: int = -1
    periodic: tuple[bool, bool] = (False, False)

    def neighbor(self, dx: int, dy: int) -> int:
        """Rank of the block at (col + dx, row + dy), or -1 outside the grid
        (dy = +1 is "top"); periodic axes wrap. Diagonal peers feed the
        corner halos that temporal blocking needs."""
        c, r = self.col + dx, self.row + dy
        if self.periodic[0]:
            c %= self.px
        if self.periodic[1]:
            r %= self.py
        if 0 <= c < self.px and 0 <= r < self.py:
            return r * self.px + c
        return -1

    @property
    def bc_sides(self) -> tuple[bool, bool, bool, bool]:
        """(top, left, bottom, right): True where the physical BC applies."""
        return (self.top < 0, self.left < 0, self.bottom < 0, self.right < 0)


def decompose(nx: int, ny: int, P: int, method: int, rank: int,
              periodic: tuple[bool, bool] = (False, False)) -> Block:
    Px, Py = proc_grid(P, method)
    row, col = divmod(rank, Px)
    x0, lnx = _split(nx, Px, col)
    y0, lny = _split(ny, Py, row)
    b = Block(rank, Px, Py, col, row, x0, y0, lnx, lny, periodic=(bool(periodic[0]), bool(periodic[1])))
    b.bottom, b.top = b.neighbor(0, -1), b.neighbor(0, 1)
    b.left, b.right = b.neighbor(-1, 0), b.neighbor(1, 0)
    return b
