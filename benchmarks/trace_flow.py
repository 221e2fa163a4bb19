#!/usr/bin/env python3
"""Per-task timeline of the persistent dataflow heat launch (csrc/hip/
heat_flow.hip, profiling entry cme_heat_flow_trace_f32): for P four-step
passes on an n^2 fp32 order-8 grid, every ticket's fetch / start / end wall
clock (100 MHz) and HW_ID / XCC_ID. Reports task duration, dependency wait
(start - ticket), the gap each workgroup spends between tasks (release +
ticket), slot occupancy (busy task time / (workgroups x span)) and the
per-pass launch time of the same passes for comparison.

    python benchmarks/trace_flow.py [--n 16384] [--passes 6] [--arith fma] [--out x.jsonl]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--passes", type=int, default=6)
    ap.add_argument("--arith", default="fma")
    ap.add_argument("--per-cu", type=int, default=0)
    ap.add_argument("--mode", type=int, default=0, help="diagnostics knob flow_mode (4096: nt stores + release)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import numpy as np
    import torch

    import cme213x
    from cme213x.models.heat2d import HeatGrid
    from cme213x.ops.stencil import heat_flow, heat_run
    from cme213x.utils import tuning
    from cme213x.utils.params import SimParams

    p = SimParams(nx=args.n, ny=args.n, order=8, flavor="hw5")
    g = HeatGrid(p, torch.float32, "cuda")
    gen = torch.Generator(device="cuda").manual_seed(1)
    xb, xe, yb, ye = g.interior
    g.buf[0, yb:ye, xb:xe] = torch.rand((ye - yb, xe - xb), device="cuda", generator=gen) * 10
    g.buf[1].copy_(g.buf[0])
    var = {"fma": "pipe4_fma", "fast": "pipe4_fast", "exact": "pipe4"}[args.arith]
    rec = {"n": args.n, "passes": args.passes, "arith": args.arith, "per_cu": args.per_cu, "mode": args.mode}
    with tuning.override(flow_per_cu=args.per_cu, flow_mode=args.mode):
        # warm: both paths, then timed
        for _ in range(3):
            heat_run(g.buf[0], g.buf[1], g.interior, 8, g.xcfl, g.ycfl, 4 * args.passes, var)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = {}
        for flow in (1, 0):
            with tuning.override(heat_flow=flow):
                heat_run(g.buf[0], g.buf[1], g.interior, 8, g.xcfl, g.ycfl, 4 * args.passes, var)
                t = []
                for _ in range(5):
                    e0.record()
                    heat_run(g.buf[0], g.buf[1], g.interior, 8, g.xcfl, g.ycfl, 4 * args.passes, var)
                    e1.record()
                    e1.synchronize()
                    t.append(e0.elapsed_time(e1))
                ts[flow] = sorted(t)[2]
        rec["ms_per_step_flow"] = round(ts[1] / (4 * args.passes), 4)
        rec["ms_per_step_per_pass"] = round(ts[0] / (4 * args.passes), 4)
        _, tr, tpp = heat_flow(g.buf[0], g.buf[1], g.interior, 8, g.xcfl, g.ycfl, args.passes, fma=args.arith,
                               trace=True)
    tr = tr.numpy().astype(np.int64)
    t0 = tr[:, 0].min()
    tk, st, en = (tr[:, 0] - t0) / 100.0, (tr[:, 1] - t0) / 100.0, (tr[:, 2] - t0) / 100.0  # us
    hw = tr[:, 3]
    span = en.max()
    dur = en - st
    wait = st - tk
    # workgroup slots: order tickets per HW slot (HW_ID | XCC) by start time
    slots = {}
    for i in np.argsort(tk):
        slots.setdefault(int(hw[i]), []).append(i)
    gaps = []
    for ids in slots.values():
        for a, b in zip(ids[:-1], ids[1:]):
            gaps.append(tk[b] - en[a])
    rec.update({
        "tasks_per_pass": int(tpp), "tickets": int(len(tr)), "hw_slots": len(slots),
        "span_us": round(float(span), 1), "task_us_median": round(float(np.median(dur)), 1),
        "task_us_p90": round(float(np.percentile(dur, 90)), 1),
        "wait_us_median": round(float(np.median(wait)), 2), "wait_us_p90": round(float(np.percentile(wait, 90)), 2),
        "wait_us_max": round(float(wait.max()), 1),
        "gap_us_median": round(float(np.median(gaps)), 2) if gaps else None,
        "slot_busy_pct": round(100.0 * float(dur.sum()) / (len(slots) * float(span)), 1),
        "per_pass_end_us": [round(float(en[p * tpp:(p + 1) * tpp].max()), 1) for p in range(args.passes)],
        "per_pass_first_start_us": [round(float(st[p * tpp:(p + 1) * tpp].min()), 1) for p in range(args.passes)],
    })
    # per-CU concurrency: HW_ID fields (gfx9 layout: CU_ID [11:8], SH_ID [12],
    # SE_ID [15:13]) plus XCC_ID identify the CU
    cu = ((hw >> 32) << 8) | ((hw >> 8) & 0xFF)
    conc = []
    for c in np.unique(cu):
        ev = sorted([(float(a), 1) for a in st[cu == c]] + [(float(b), -1) for b in en[cu == c]],
                    key=lambda e: (e[0], e[1]))
        k = m = 0
        for _, d in ev:
            k += d
            m = max(m, k)
        conc.append(m)
    # per XCD band: busy task time and the end of its last task
    xcc = hw >> 32
    rec["per_xcd_busy_ms"] = [round(float(dur[xcc == x].sum()) / 1e3, 1) for x in range(8)]
    rec["per_xcd_last_end_us"] = [round(float(en[xcc == x].max()), 1) if (xcc == x).any() else None for x in range(8)]
    rec["per_xcd_task_us_median"] = [round(float(np.median(dur[xcc == x])), 1) if (xcc == x).any() else None
                                     for x in range(8)]
    rec["cus_seen"] = int(len(conc))
    rec["max_tasks_per_cu_hist"] = {str(v): int(c) for v, c in zip(*np.unique(conc, return_counts=True))}
    try:
        from cme213x.utils.occupancy import kernel_report
        rec["occupancy_api"] = {r["kernel"]: [r["vgprs"], r["blocks_per_cu"], r["scratch_bytes"]]
                                for r in kernel_report() if "flow" in r["kernel"] or "pipe4w" in r["kernel"]}
    except Exception as e:  # noqa: BLE001
        rec["occupancy_api"] = str(e)
    s = json.dumps(rec)
    print(s, flush=True)
    if args.out:
        with open(args.out, "a") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
