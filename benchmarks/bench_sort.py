#!/usr/bin/env python3
"""GPU sort benchmark: radix (onesweep) and merge sort vs torch.sort.

    python benchmarks/bench_sort.py [--n 16777216] [--dtype uint32|int32|float32] [--algo radix merge]
                                     [--values] [--reps 20]

Times back-to-back calls with hipEvents (median over reps), one JSON line per
(algo, n): ms, Gkeys/s, and the "equivalent bandwidth" of a 4-pass LSD sort
(read + write of the keys per pass; BASELINE #15-16 compare against the
hw4 OpenMP sorts, hw/hw4/programming/radixsort.cpp / mergesort.cpp)."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[16 * 1024 * 1024])
    ap.add_argument("--dtype", default="uint32", choices=["uint32", "int32", "float32"])
    ap.add_argument("--algo", nargs="+", default=["radix", "merge", "torch"])
    ap.add_argument("--values", action="store_true", help="sort (key, 32-bit value) pairs")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--kind", default="random", choices=["random", "small", "sorted"],
                    help="random: uniform 32-bit keys; small: keys < 2^16 (the high digits all zero); sorted")
    ap.add_argument("--tune", nargs="*", default=[],
                    help="tuning knobs name=value (cme213x.utils.tuning), e.g. radix_ds=10")
    a = ap.parse_args()

    import torch

    import cme213x  # noqa: F401
    from cme213x.ops.sort import sort
    from cme213x.utils import tuning

    knobs = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in a.tune}
    for k, val in knobs.items():
        tuning.set(k, val)

    dt = getattr(torch, a.dtype)
    for n in a.n:
        g = torch.Generator(device="cuda").manual_seed(1)
        if dt == torch.float32:
            x = torch.randn(n, device="cuda", generator=g)
        else:
            x = torch.randint(0, 2**31 - 1, (n,), device="cuda", dtype=torch.int64, generator=g)
            x = (x * 2 + (x & 1)).to(torch.int64) if dt == torch.uint32 else x - 2**30
            if a.kind == "small":
                x = x % 65536
            x = x.to(torch.int32).view(dt) if dt == torch.uint32 else x.to(dt)
        if a.kind == "sorted":
            x = torch.sort(x.to(torch.int64) if dt == torch.uint32 else x).values.to(x.dtype)
            x = x.view(dt) if dt == torch.uint32 else x
        v = torch.arange(n, device="cuda", dtype=torch.int32) if a.values else None
        ref = torch.sort(x.to(torch.int64) if dt == torch.uint32 else x).values
        for algo in a.algo:
            if algo == "torch":
                if dt == torch.uint32:
                    continue  # torch.sort has no uint32 kernel on ROCm
                fn = (lambda: torch.sort(x)) if v is None else (lambda: torch.sort(x))
            else:
                fn = (lambda al=algo: sort(x, v, algo=al)) if v is not None else (lambda al=algo: sort(x, algo=al))
            out = fn()
            keys = out[0] if isinstance(out, tuple) else out
            ok = torch.equal(keys.to(torch.int64) if dt == torch.uint32 else keys, ref)
            for _ in range(3):
                fn()
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            ts.sort()
            ms = ts[len(ts) // 2]
            rec = {"bench": "sort", "algo": algo, "n": n, "dtype": a.dtype, "values": a.values, "kind": a.kind,
                   "tune": knobs, "ms": round(ms, 4),
                   "Gkeys_per_s": round(n / ms / 1e6, 2),
                   "eq_TBps_4pass": round(n * 4 * (2 if a.values else 1) * 2 * 4 / ms / 1e9, 2), "ok": ok}
            print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
