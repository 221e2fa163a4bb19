#!/usr/bin/env python3
"""SGEMM MFMA tuning arms (``cme_sgemm_tune``) at M = N = K = --n against
torch.mm (hipBLASLt). Each arm is checked against torch.mm, then timed as
the median of --reps runs of --calls back-to-back launches.

    python benchmarks/tune_sgemm.py [--n 8192] [--arms 0 8 ...]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="*", default=[8192])
    ap.add_argument("--arms", type=int, nargs="*", default=None)
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from cme213x import _ext
    from cme213x.ops.gemm import sgemm

    _ext.proto(_ext.HIP_PROTOS, "cme_sgemm_tune", "iiipppip")
    arms = args.arms if args.arms is not None else [int(a) for a in os.environ.get("CME_SGEMM_ARMS", "0 8").split()]

    def t_ms(fn):
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.calls):
                fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / args.calls)
        return sorted(ts)[len(ts) // 2]

    for n in args.n:
        g = torch.Generator(device="cuda").manual_seed(0)
        A = torch.rand(n, n, device="cuda", generator=g) * 2 - 1
        B = torch.rand(n, n, device="cuda", generator=g) * 2 - 1
        C = torch.empty(n, n, device="cuda")
        ref = A @ B
        fl = 2.0 * n ** 3
        torch.mm(A, B, out=C)
        ms = t_ms(lambda: torch.mm(A, B, out=C))
        print(json.dumps({"n": n, "arm": "torch.mm", "ms": round(ms, 4), "TFLOPs": round(fl / ms / 1e9, 1)}), flush=True)
        sgemm(A, B, C)
        ms = t_ms(lambda: sgemm(A, B, C))
        err = float((C - ref).abs().max())
        print(json.dumps({"n": n, "arm": "production", "ms": round(ms, 4), "TFLOPs": round(fl / ms / 1e9, 1),
                          "max_abs_err": err}), flush=True)
        s = _ext.stream_ptr(A.device)
        for arm in arms:
            def run():
                _ext.call_hip("cme_sgemm_tune", n, n, n, A.data_ptr(), B.data_ptr(), C.data_ptr(), arm, s)

            C.zero_()
            run()
            torch.cuda.synchronize()
            err = float((C - ref).abs().max())
            ms = t_ms(run)
            print(json.dumps({"n": n, "arm": arm, "ms": round(ms, 4), "TFLOPs": round(fl / ms / 1e9, 1),
                              "max_abs_err": err}), flush=True)


if __name__ == "__main__":
    main()
