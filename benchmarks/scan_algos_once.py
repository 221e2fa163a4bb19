#!/usr/bin/env python3
"""Runs each 2^26 fp32 exclusive-scan algorithm `--reps` times (for
`rocprofv3 --kernel-trace --stats`: per-kernel time of every algorithm's
launches). Prints nothing but a done line."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 26)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--algos", nargs="*", default=["lookback", "rts", "blelloch", "hillis"])
    ap.add_argument("--sets", type=int, default=1,
                    help="operand sets visited round-robin (3: every call cold, as bench.py's config #3)")
    a = ap.parse_args()
    import torch

    from cme213x.ops.scan import scan

    xs = [torch.rand(a.n, device="cuda") for _ in range(a.sets)]
    ys = [torch.empty_like(x) for x in xs]
    for algo in a.algos:
        for i in range(a.reps):
            scan(xs[i % a.sets], True, ys[i % a.sets], algo=algo)
    torch.cuda.synchronize()
    print("done", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
