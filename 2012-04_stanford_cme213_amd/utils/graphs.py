"""hipGraph capture of launch-bound native loops.

Every native launcher enqueues on torch's *current* stream (``_ext.
stream_ptr``), so a whole sequence of native calls -- kernels, memsets, even
the native multi-step loops -- can be recorded once with torch's graph API
(hipGraph on ROCm) and replayed with a single launch. This is the MI355X
answer to per-iteration launch overhead (the reference synchronises after
every launch, e.g. ``hw/hw2/solution/2dHeat_solution.cu:549``): the final
project's small matrices spend most of their time in ~5 us launches.

Caveats (enforced by the caller): the captured work must use fixed device
pointers and sizes, and no host synchronisation may occur inside ``fn``.
"""
from __future__ import annotations

from typing import Callable

import torch


class GraphRunner:
    """Record ``fn`` (after ``warmup`` eager calls on a side stream, as torch
    recommends) and replay it with :meth:`__call__`. Recording does NOT
    execute the work; Python-side state that ``fn`` mutates (e.g. a grid's
    current-buffer index) advances once at capture time, so capture loops that
    return to their starting buffers."""

    def __init__(self, fn: Callable[[], object], warmup: int = 1):
        if not torch.cuda.is_available():
            raise RuntimeError("hipGraph capture needs a GPU")
        self.fn = fn
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                fn()
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = fn()

    def __call__(self):
        self.graph.replay()
        return self.out
