#!/usr/bin/env python3
"""Per-workgroup timeline of ONE wave-pipelined pass (the fused distributed
schedule's launch: deep interior + border strips) for the subdomain one rank
of an N-GPU strong-scaled 16384^2 run owns. Needs the tuning library
(CME_TUNE=1 build: cme_heat_pipe_trace).

    python benchmarks/trace_pipe_tasks.py [--world 1 8] [--chunk 0] [--per-cu 0]

Prints one JSON line per world size: kernel span, task count, per-region
task durations (median / p90), the span between the first and last task
start (dispatch ramp) and between the first and last end (tail), and the
CU-time utilisation = sum of task spans / (CUs x workgroups-per-CU x kernel
span) -- the share of the pass the resident slots spent on tasks."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--world", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--tblock", type=int, default=4)
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--per-cu", type=int, default=0)
    ap.add_argument("--slots", type=int, default=3, help="resident workgroups per CU (occupancy)")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--dump", default="", help="path prefix: save the median rep's raw spans (npz)")
    args = ap.parse_args()
    import ctypes

    import numpy as np
    import torch

    import cme213x  # noqa: F401
    from cme213x import _ext
    from cme213x.models.heat2d_dist import DistHeat
    from cme213x.parallel.comm import Comm, Pending
    from cme213x.utils.params import SimParams

    _ext.proto(_ext.TUNE_PROTOS, "cme_heat_pipe_trace", "ppiipipiffiipp")

    class NullComm(Comm):
        def __init__(self, rank, size):
            self.rank, self.size = rank, size

        def exchange(self, ops):
            return Pending()

    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    for world in args.world:
        p = SimParams(nx=args.n, ny=args.n, order=8, ic=5.0, bc=(0.0, 10.0, 0.0, 10.0), grid_method=1, flavor="hw5")
        rank = world // 2 if world > 1 else 0  # an interior stripe (two neighbours)
        sim = DistHeat(p, NullComm(rank, world), torch.float32, "cuda", tblock=args.tblock, fma=True, kernel="pipe")
        (s,) = sim.subs.values()
        g = s.grid
        gen = torch.Generator(device="cuda").manual_seed(3)
        g.buf.copy_(torch.rand(g.buf.shape, generator=gen, device="cuda") * 10.0)
        pl = sim._native_plan()["plans"][rank]
        regs = torch.cat([pl["interior"], pl["border"]]).contiguous()
        n_int = pl["interior"].shape[0]
        ext = pl["ext"].contiguous()
        trace = torch.zeros(3 * 65536, dtype=torch.int64, device="cuda")
        st = _ext.stream_ptr()

        def launch():
            _ext.call_hip("cme_heat_pipe_trace", g.buf[0].data_ptr(), g.buf[1].data_ptr(), g.pitch, g.gy,
                          regs.data_ptr(), regs.shape[0], ext.data_ptr(), args.tblock, g.xcfl, g.ycfl, args.chunk,
                          args.per_cu, trace.data_ptr(), st)

        for _ in range(20):  # clock ramp
            launch()
        torch.cuda.synchronize()
        spans = []
        for _ in range(args.reps):
            trace.zero_()
            launch()
            torch.cuda.synchronize()
            t = trace.view(-1, 3).cpu().numpy()
            t = t[t[:, 1] > 0]
            t0 = t[:, 0].min()
            start, end = (t[:, 0] - t0) * 10.0 / 1e3, (t[:, 1] - t0) * 10.0 / 1e3  # us (100 MHz)
            region = (t[:, 2] >> 40).astype(int)
            spans.append((float(end.max()), start, end, region, (t[:, 2] & 0xFFFFFFFF), (t[:, 2] >> 32) & 0xFF))
        spans.sort(key=lambda x: x[0])
        kspan, start, end, region, hwid, xcc = spans[len(spans) // 2]
        dur = end - start
        per_region = {}
        for r in sorted(set(region.tolist())):
            d = dur[region == r]
            per_region[("interior" if r < n_int else "border") + f"{r}"] = {
                "tasks": int(d.size), "median_us": round(float(np.median(d)), 2),
                "p90_us": round(float(np.percentile(d, 90)), 2), "rows": int(regs[r, 3] - regs[r, 2])}
        util = float(dur.sum()) / (ncu * args.slots * kspan)
        if args.dump:
            os.makedirs(os.path.dirname(args.dump) or ".", exist_ok=True)
            np.savez(f"{args.dump}_w{world}.npz", start=start, end=end, region=region, hw=hwid, xcc=xcc)
        rec = {"bench": "pipe_task_trace", "world": world, "rank": rank, "tblock": args.tblock,
               "chunk": args.chunk, "per_cu": args.per_cu, "kernel_span_us": round(kspan, 2),
               "tasks": int(dur.size), "regions": per_region,
               "start_spread_us": round(float(np.percentile(start, 99)), 2),
               "last_start_us": round(float(start.max()), 2),
               "first_end_us": round(float(end.min()), 2),
               "tail_us": round(float(kspan - np.percentile(end, 50)), 2),
               "slot_utilisation": round(util, 3),
               "task_us_median": round(float(statistics.median(dur.tolist())), 2)}
        print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
