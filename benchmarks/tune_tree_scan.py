#!/usr/bin/env python3
"""Cold A/B of the Blelloch tile-parallel reduce-then-scan arms
(csrc/hip_tune/scan_tune.hip cme_scan_tree_tune; BASELINE config #3).

    python benchmarks/tune_tree_scan.py [--arms 0 1 2 ...] [--n 67108864]

Same protocol as bench.py's cold primitives: 3 operand sets of 2^26 fp32
uniform(0, 1) visited round-robin (every call's input comes from HBM), the
median over 7 event-timed batches. Each arm is first checked against a float64
reference (max relative error of the exclusive prefix), one JSON line per arm.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", type=int, nargs="+", default=[0, 1, 2, 3, 4, 5, 6, 7])
    ap.add_argument("--n", type=int, default=1 << 26)
    ap.add_argument("--rounds", type=int, default=2, help="passes over the 3 operand sets per timed batch")
    a = ap.parse_args()

    import torch

    import cme213x
    from cme213x import _ext

    sys.path.insert(0, REPO)
    from bench import _cold_ms

    _ext.proto(_ext.TUNE_PROTOS, "cme_scan_tree_tune", "ppqipp")
    dev = torch.device("cuda", 0)
    n = a.n
    g = torch.Generator(device=dev).manual_seed(7)
    sets = [(torch.rand(n, device=dev, generator=g), torch.empty(n, device=dev)) for _ in range(3)]
    tiles = (n + 4095) // 4096
    ws = torch.zeros((tiles * 4 + 255) // 256 * 256 + 256, dtype=torch.uint8, device=dev)
    x0 = sets[0][0].double()
    ref = torch.cumsum(x0, 0) - x0
    scale = ref.abs().clamp_min(1.0)
    for arm in a.arms:
        def fn(s, arm=arm):
            _ext.call_hip("cme_scan_tree_tune", s[0].data_ptr(), s[1].data_ptr(), n, arm, ws.data_ptr(),
                          _ext.stream_ptr(dev))
        fn(sets[0])
        torch.cuda.synchronize(dev)
        err = float(((sets[0][1].double() - ref).abs() / scale).max())
        ms = _cold_ms(dev, sets, fn, rounds=a.rounds)
        print(json.dumps({"bench": "tree_scan_tune", "arm": arm, "n": n, "ms_cold": round(ms, 4),
                          "GBps_12B": round(12 * n / ms / 1e6, 1), "max_rel_err": err, "ok": err < 1e-5}),
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
