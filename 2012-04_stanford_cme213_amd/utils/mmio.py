"""Matrix Market reader (coordinate real/integer/pattern, general/symmetric),
the input of the final project's ``readMM.py`` (which used scipy's mmread).
Returns 0-based (rows, cols, vals, shape); symmetric files are expanded."""
from __future__ import annotations

import numpy as np


def read_matrix_market(path: str):
    with open(path) as f:
        header = f.readline().lower().split()
        if not header or header[0] != "%%matrixmarket" or header[2] != "coordinate":
            raise ValueError("only coordinate Matrix Market files are supported")
        field, sym = header[3], header[4]
        line = f.readline()
        while line.startswith("%"):
            line = f.readline()
        nr, nc, nnz = (int(v) for v in line.split())
        data = np.loadtxt(f, ndmin=2) if nnz else np.zeros((0, 3))
    r = data[:, 0].astype(np.int64) - 1
    c = data[:, 1].astype(np.int64) - 1
    v = data[:, 2].astype(np.float64) if field != "pattern" else np.ones(r.size)
    if sym in ("symmetric", "skew-symmetric", "hermitian"):
        off = r != c
        sign = -1.0 if sym == "skew-symmetric" else 1.0
        r, c, v = np.concatenate([r, c[off]]), np.concatenate([c, r[off]]), np.concatenate([v, sign * v[off]])
    return r, c, v.astype(np.float32), (nr, nc)


def write_matrix_market(path: str, rows, cols, vals, shape) -> None:
    with open(path, "w") as f:
        f.write("%%MatrixMarket matrix coordinate real general\n")
        f.write(f"{shape[0]} {shape[1]} {len(vals)}\n")
        for r, c, v in zip(rows, cols, vals):
            f.write(f"{int(r) + 1} {int(c) + 1} {float(v)!r}\n")
