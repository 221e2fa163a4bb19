"""hw1 part 2: PageRank-style propagation driver.

Parity with ``hw/hw1/programming/pagerank.cu:146-249``: N = 2^21 nodes,
avg_edges 8, 20 iterations, GPU vs host reference, ULP check (10 in the
student version, 1000 in the solution), ``"Worked! CUDA and reference output
match."``. The avg_edges sweep reproduces ``analysis/bandwidth_vs_avg_edges.csv``
(GB/s under the student's byte model).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops.graph import bytes_model, iterate, make_graph
from ..utils.timer import EventTimer
from ..utils.ulp import ulp_distance


def run_hw1_pagerank(n: int = 1 << 21, avg_edges: int = 8, iters: int = 20, device: str | None = None,
                     group: int = 1, max_ulps: int = 10, seed: int = 0, blocks: int = 0) -> dict:
    """``blocks`` > 1: column-blocked sweeps (``ops.graph.block_columns``;
    fastest measured: blocks 2, group 2 -- profiles/pagerank_r3.md). The
    default (group 1, unblocked) keeps the CPU summation order bit for bit."""
    device = device or ("cuda" if torch.cuda.is_available() else "cpu")
    g = make_graph(n, avg_edges, seed)
    x0 = torch.full((n,), 1.0 / n, dtype=torch.float32)
    res = {}
    if device != "cpu":
        dev = torch.device(device)
        gd = g.to(dev)
        if blocks > 1:
            from ..ops.graph import block_columns

            gd = block_columns(gd, blocks)
        xd = x0.to(dev)
        iterate(gd, xd, 2, group)  # warm-up
        t = EventTimer("gpu graph propagate", device=dev)
        with t:
            out = iterate(gd, xd, iters, group)
        res["gpu_ms"] = t.ms
        res["GBps_model"] = bytes_model(g, iters) / t.ms / 1e6
        gpu = out.cpu().numpy()
    iterate(g, x0, 2)  # CPU warm-up (OpenMP thread start-up), like the GPU's above
    t = EventTimer("host graph propagate")
    with t:
        ref = iterate(g, x0, iters).numpy()
    res["cpu_ms"] = t.ms
    if device != "cpu":
        d = ulp_distance(gpu, ref)
        bad = np.flatnonzero(d > max_ulps)
        for i in bad[:9]:
            print(f"{i}:{gpu[i] - ref[i]:.16f}::", end="")
        if bad.size:
            print("Output of CUDA version and normal version didn't match! ")
        else:
            print("Worked! CUDA and reference output match. ")
        res["errors"] = int(bad.size)
        res["max_ulp"] = int(d.max())
    return res


def sweep_avg_edges(n: int = 1 << 21, edges=range(2, 21), iters: int = 20, device="cuda", group: int = 1):
    dev = torch.device(device)
    rows = []
    for e in edges:
        g = make_graph(n, e).to(dev)
        x = torch.full((n,), 1.0 / n, device=dev)
        iterate(g, x, 2, group)
        t = EventTimer("", device=dev, print_result=False)
        with t:
            iterate(g, x, iters, group)
        rows.append({"avg_edges": e, "ms": t.ms, "bytes": bytes_model(g, iters),
                     "GBps": bytes_model(g, iters) / t.ms / 1e6})
    return rows
