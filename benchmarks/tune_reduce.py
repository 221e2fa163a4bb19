#!/usr/bin/env python3
"""Cold A/B of the f32 sum-reduction arms (csrc/hip_tune/scan_tune.hip
cme_reduce_tune; BASELINE config #3), bench.py's cold protocol: 3 operand sets
of 2^26 uniform(0, 1) floats visited round-robin, median of 7 event-timed
batches; each arm checked against a float64 sum first. One JSON line per arm.

    python benchmarks/tune_reduce.py [--arms 0 1 2 3]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", type=int, nargs="+", default=[0, 1, 2, 3])
    ap.add_argument("--n", type=int, default=1 << 26)
    a = ap.parse_args()

    import torch

    import cme213x  # noqa: F401
    from cme213x import _ext
    from bench import _cold_ms

    _ext.proto(_ext.TUNE_PROTOS, "cme_reduce_tune", "pqippp")
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(11)
    sets = [torch.rand(a.n, device=dev, generator=g) for _ in range(3)]
    part = torch.zeros(2048 + 64, dtype=torch.float32, device=dev)
    out = torch.zeros((), dtype=torch.float32, device=dev)
    ref = float(sets[0].double().sum())
    for arm in a.arms:
        def fn(x, arm=arm):
            _ext.call_hip("cme_reduce_tune", x.data_ptr(), a.n, arm, part.data_ptr(), out.data_ptr(),
                          _ext.stream_ptr(dev))
        fn(sets[0])
        torch.cuda.synchronize(dev)
        err = abs(float(out) - ref) / ref
        ms = _cold_ms(dev, sets, fn)
        print(json.dumps({"bench": "reduce_tune", "arm": arm, "n": a.n, "ms_cold": round(ms, 4),
                          "GBps": round(4 * a.n / ms / 1e6, 1), "rel_err": err, "ok": err < 1e-5}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
