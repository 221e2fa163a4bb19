#!/usr/bin/env python3
"""Summarise rocprofv3 CSV outputs (kernel stats, PMC counters) into markdown
tables for profiles/. Usage: summarize_prof.py <prof_dir> <out.md> [title]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:110]


def kernel_stats(path):
    rows = list(csv.DictReader(open(path)))
    out = ["| kernel | calls | avg us | total ms | % |", "|---|---|---|---|---|"]
    for r in rows[:25]:
        out.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                   f"{float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.1f} |")
    return "\n".join(out)


def counters(path):
    agg = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    names = sorted({c for d in agg.values() for c in d})
    out = ["| kernel | dispatches | " + " | ".join(f"mean {n}" for n in names) + " |",
           "|---|---|" + "---|" * len(names)]
    for k, d in agg.items():
        nd = max(len(v) for v in d.values())
        out.append(f"| `{k}` | {nd} | " + " | ".join(f"{sum(d[n]) / len(d[n]):.4g}" if d.get(n) else "" for n in names)
                   + " |")
    return "\n".join(out)


def main():
    src, dst = sys.argv[1], sys.argv[2]
    title = sys.argv[3] if len(sys.argv) > 3 else os.path.basename(src)
    parts = [f"# {title}\n", f"Source: rocprofv3 CSV under `{src}` (MI355X, gfx950).\n"]
    for p in sorted(glob.glob(os.path.join(src, "*kernel_stats.csv"))):
        parts += [f"## Kernel stats ({os.path.basename(p)})\n", kernel_stats(p), ""]
    for p in sorted(glob.glob(os.path.join(src, "*counter_collection.csv"))):
        parts += [f"## PMC counters ({os.path.basename(p)})\n", counters(p), ""]
    open(dst, "w").write("\n".join(parts) + "\n")


if __name__ == "__main__":
    main()
