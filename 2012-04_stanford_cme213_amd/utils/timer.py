"""Timers that print the reference's ``"<name> took X ms"`` lines.

* GPU: HIP events on the current stream (``torch.cuda.Event`` wraps
  ``hipEventRecord``) -- the reference's ``event_pair`` / ``start_timer`` /
  ``stop_timer`` (``hw/hw1/programming/mp1-util.h:1-39``). Events are used
  instead of wall clocks for the reason given in ``slides/Lecture08.pdf`` 2-4:
  launches are asynchronous.
* CPU: ``time.perf_counter`` (the reference's ``omp_get_wtime`` / ``MPI_Wtime``).

``fmt="csv"`` prints ``"%.2f "`` like the analysis harness variant
(``hw/hw1/programming/analysis/mp1-util.h:36``).
"""
from __future__ import annotations

import sys
import time

import torch


class EventTimer:
    def __init__(self, name: str = "", device: torch.device | str | None = None, print_result: bool = True,
                 fmt: str = "text"):
        self.name = name
        self.gpu = device is not None and torch.device(device).type == "cuda"
        self.print_result = print_result
        self.fmt = fmt
        self.ms = 0.0
        if self.gpu:
            self._s = torch.cuda.Event(enable_timing=True)
            self._e = torch.cuda.Event(enable_timing=True)

    def start(self) -> "EventTimer":
        if self.gpu:
            self._s.record()
        else:
            self._t0 = time.perf_counter()
        return self

    def stop(self) -> float:
        if self.gpu:
            self._e.record()
            self._e.synchronize()
            self.ms = self._s.elapsed_time(self._e)
        else:
            self.ms = (time.perf_counter() - self._t0) * 1e3
        if self.print_result:
            if self.fmt == "csv":
                sys.stdout.write(f"{self.ms:.2f} ")
            else:
                print(f"{self.name} took {self.ms:.2f} ms")
        return self.ms

    def __enter__(self) -> "EventTimer":
        return self.start()

    def __exit__(self, *exc) -> None:
        self.stop()


def time_fn(fn, iters: int = 10, warmup: int = 2, device: str | torch.device = "cuda") -> float:
    """Median milliseconds per call of ``fn`` (GPU events per call)."""
    dev = torch.device(device)
    for _ in range(warmup):
        fn()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(iters):
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e))
    else:
        ts = []
        for _ in range(iters):
            t0 = time.perf_counter()
            fn()
            ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]
