#!/usr/bin/env python3
"""hw5 1000^2 fp64 (BASELINE #17) through the driver's solver: eager native
run vs the same run captured once in a HIP graph and replayed. Does replay
shrink the per-pass kernel boundary (~3.5 us of a ~16.6 us pass,
profiles/heat_tile_r5.md)? One JSON line per mode (median of reps, ms per
1000-iteration run; the graph's output is checked bitwise against eager).

    python benchmarks/hw5_graph.py [--iters 1000] [--reps 7] [--fma]
"""
import argparse
import contextlib
import io
import json
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--fma", action="store_true")
    a = ap.parse_args()

    import torch

    import cme213x  # noqa: F401
    from cme213x.models.heat2d_dist import run_hw5

    src = open(os.path.join(REPO, "tests", "data", "hw5_params.in")).read()
    with tempfile.NamedTemporaryFile("w", suffix=".in", delete=False) as f:
        f.write(src)
        path = f.name
    with contextlib.redirect_stdout(io.StringIO()):
        res = run_hw5(path, None, torch.float64, "cuda", write_files=False, fma=a.fma)
    sim = res["sim"]
    sub = next(iter(sim.subs.values()))
    init = sub.grid.buf.clone()

    def reset():
        sub.grid.buf.copy_(init)
        sub.grid.iteration = 0
        sim.iteration = 0

    def timed(fn):
        ts = []
        for _ in range(a.reps):
            reset()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return sorted(ts)[len(ts) // 2]

    ms_eager = timed(lambda: sim.run(a.iters))
    reset()
    sim.run(a.iters)
    torch.cuda.synchronize()
    ref = sub.grid.buf.clone()
    rec = {"bench": "hw5_graph", "n": 1000, "iters": a.iters, "fma": a.fma, "tblock": sim.tblock,
           "kernel": sim.kernel, "ms_eager": round(ms_eager, 4)}
    try:
        reset()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            sim.run(a.iters)
        ms_graph = timed(g.replay)
        reset()
        g.replay()
        torch.cuda.synchronize()
        rec.update(ms_graph=round(ms_graph, 4), graph_bitwise=bool(torch.equal(sub.grid.buf, ref)))
    except Exception as e:  # noqa: BLE001 - recorded
        rec["graph_error"] = f"{type(e).__name__}: {e}"[:300]
    print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
