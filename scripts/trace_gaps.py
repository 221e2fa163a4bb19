#!/usr/bin/env python3
"""Kernel durations and the idle gaps between consecutive dispatches from a
rocprofv3 --kernel-trace CSV (one row per dispatch).

    python scripts/trace_gaps.py <dir with *kernel_trace.csv> [--match SUBSTR] [--skip N]

Prints, per kernel name (matching SUBSTR), the dispatch count, median / mean
duration, and the median / mean gap from the previous dispatch's end to this
one's start (all kernels, in start order), skipping the first N matching
dispatches (warm-up)."""
import argparse
import csv
import glob
import os
import re
import statistics


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name.replace("void ", ""))
    return name[:100]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    ap.add_argument("--skip", type=int, default=0)
    args = ap.parse_args()
    rows = []
    for p in glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    per = {}
    prev_end = None
    for s, e, n in rows:
        gap = (s - prev_end) if prev_end is not None else None
        prev_end = e if prev_end is None else max(prev_end, e)
        if args.match and args.match not in n:
            continue
        per.setdefault(short(n), []).append((e - s, gap))
    for n, v in per.items():
        v = v[args.skip:]
        if not v:
            continue
        d = [x[0] / 1e3 for x in v]
        g = [x[1] / 1e3 for x in v if x[1] is not None]
        print(f"{n}: n={len(v)} dur_med={statistics.median(d):.2f}us dur_mean={statistics.mean(d):.2f}us "
              f"gap_med={statistics.median(g) if g else 0:.2f}us gap_mean={statistics.mean(g) if g else 0:.2f}us")


if __name__ == "__main__":
    main()
