#!/usr/bin/env python3
"""the hw2 driver's CPU line ("cpu computation float took X
ms", tests/data/hw2_params_test.in: 4000^2, order 4, 10 steps) against a warm
repeat of the same call in the same process. Prints one JSON line."""
import contextlib
import io
import json
import os
import re
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import tempfile

    import torch

    import cme213x  # noqa: F401
    from cme213x.models.heat2d import HeatGrid, run_hw2
    from cme213x.utils import cpu_runtime
    from cme213x.utils.params import SimParams

    params = os.path.join(REPO, "tests", "data", "hw2_params_test.in")
    buf = io.StringIO()
    with tempfile.TemporaryDirectory() as d, contextlib.redirect_stdout(buf):
        run_hw2(params, torch.float32, device="cpu", outdir=d, write_files=False)
    line = [ln for ln in buf.getvalue().splitlines() if "cpu computation" in ln][-1]
    driver_ms = float(re.search(r"took ([0-9.]+) ms", line).group(1))
    p = SimParams.from_file(params, flavor="hw2")
    warm = []
    for _ in range(3):
        g = HeatGrid(p, torch.float32, "cpu")
        t0 = time.perf_counter()
        g.run(p.iters, "naive")
        warm.append((time.perf_counter() - t0) * 1e3)
    warm_ms = sorted(warm)[1]
    print(json.dumps({"driver_line": line, "driver_ms": driver_ms, "warm_ms": round(warm_ms, 2),
                      "ratio": round(driver_ms / warm_ms, 3), "within_2x": driver_ms <= 2 * warm_ms,
                      **{f"cpu_{k}": v for k, v in cpu_runtime.info().items()}}))


if __name__ == "__main__":
    main()
