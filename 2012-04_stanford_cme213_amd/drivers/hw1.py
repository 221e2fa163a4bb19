"""hw1 drivers: ``cipher [book]`` and ``pagerank`` (+ the analysis sweeps).

    python -m cme213x cipher [mobydick.txt] [--sweep vl|bs]
    python -m cme213x pagerank [--avg-edges 8] [--group 1] [--blocks 0] [--sweep]
"""
from __future__ import annotations

import argparse
import csv
import sys

DEFAULT_BOOK = "/root/reference/hw/hw1/programming/mobydick.txt"


def cipher_main(argv=None) -> int:
    from ..models.cipher import run_hw1_cipher, sweep_block_size, sweep_vector_length

    ap = argparse.ArgumentParser(prog="cipher")
    ap.add_argument("book", nargs="?", default=DEFAULT_BOOK)
    ap.add_argument("--sweep", choices=["vl", "bs"])
    ap.add_argument("--csv", default=None)
    a = ap.parse_args(argv)
    if a.sweep:
        rows = sweep_vector_length(a.book) if a.sweep == "vl" else sweep_block_size(a.book)
        out = open(a.csv, "w", newline="") if a.csv else sys.stdout
        w = csv.DictWriter(out, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
        return 0
    res = run_hw1_cipher(a.book)
    return 0 if res.get("ok", True) else 1


def pagerank_main(argv=None) -> int:
    from ..models.pagerank import run_hw1_pagerank, sweep_avg_edges

    ap = argparse.ArgumentParser(prog="pagerank")
    ap.add_argument("--nodes", type=int, default=1 << 21)
    ap.add_argument("--avg-edges", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--group", type=int, default=1)
    ap.add_argument("--blocks", type=int, default=0, help="column-blocked sweeps (2 = fastest measured)")
    ap.add_argument("--sweep", action="store_true")
    a = ap.parse_args(argv)
    if a.sweep:
        for r in sweep_avg_edges(a.nodes, iters=a.iters, group=a.group):
            print(f"{r['avg_edges']},{r['ms']:.2f},{r['bytes']},{r['GBps']:.4f}")
        return 0
    res = run_hw1_pagerank(a.nodes, a.avg_edges, a.iters, group=a.group, blocks=a.blocks)
    return 1 if res.get("errors") else 0
