#!/usr/bin/env python3
"""Overlap of two kernel families in a rocprofv3 --kernel-trace output (CSV
or the default rocpd SQLite database).

    python scripts/overlap.py <dir with *kernel_trace.csv> --a heat_pipe --b nccl [--skip-a N]

For every dispatch of family A (kernel name contains --a), how many
dispatches of family B started or ran while it executed, and the fraction of
B's busy time that falls inside A dispatches. Prints a markdown table."""
import argparse
import csv
import glob
import os
import re
import statistics


def short(name: str) -> str:
    return re.sub(r"\(.*", "", name.replace("void ", ""))[:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--a", required=True)
    ap.add_argument("--b", required=True)
    ap.add_argument("--skip-a", type=int, default=0)
    args = ap.parse_args()
    rows = []
    for p in glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    for p in glob.glob(os.path.join(args.dir, "**", "*.db"), recursive=True):  # rocprofv3's default rocpd output
        import sqlite3

        rows += [(int(s), int(e), n) for s, e, n in sqlite3.connect(p).execute("select start, end, name from kernels")]
    rows.sort()
    A = [r for r in rows if args.a in r[2]][args.skip_a:]
    B = [r for r in rows if args.b.lower() in r[2].lower()]
    if not A or not B:
        print(f"no dispatches: {len(A)} of '{args.a}', {len(B)} of '{args.b}'")
        return 1
    t_lo = A[0][0]
    B = [b for b in B if b[1] >= t_lo]
    inside = 0
    b_busy = sum(e - s for s, e, _ in B)
    per_a = []
    for s, e, _ in A:
        n = 0
        for bs, be, _ in B:
            ov = min(e, be) - max(s, bs)
            if ov > 0:
                inside += ov
                n += 1
        per_a.append(n)
    names = {}
    for s, e, n in B:
        names.setdefault(short(n), []).append(e - s)
    print(f"| family | dispatches | median us | mean us |")
    print(f"|---|---|---|---|")
    print(f"| A: {args.a} | {len(A)} | {statistics.median([e - s for s, e, _ in A]) / 1e3:.1f} | "
          f"{statistics.mean([e - s for s, e, _ in A]) / 1e3:.1f} |")
    for k, v in sorted(names.items()):
        print(f"| B: {k} | {len(v)} | {statistics.median(v) / 1e3:.1f} | {statistics.mean(v) / 1e3:.1f} |")
    print()
    print(f"A dispatches overlapped by >= 1 B dispatch: {sum(1 for n in per_a if n)} / {len(per_a)}")
    print(f"B busy time inside A dispatches: {100.0 * inside / max(1, b_busy):.1f} % "
          f"({inside / 1e3:.1f} of {b_busy / 1e3:.1f} us)")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
