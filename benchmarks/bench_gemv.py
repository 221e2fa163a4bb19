#!/usr/bin/env python3
"""GEMV y = A x (framework ``cme_gemv``) against torch.mv (rocBLAS) on the
shapes of the Lecture20 dense matvecs: square, column block (n x n/P) and
2-D block (n/q x n/q). HBM-bound: reported as GB/s of A + x + y and as % of
the measured 16-B copy bandwidth. Each timing rotates R copies of A whose
total exceeds the 256 MB MALL, so no call finds A in cache.

    python benchmarks/bench_gemv.py [--out profiles/gemv_r2.jsonl]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FOOTPRINT = 768 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--calls", type=int, default=32)
    args = ap.parse_args()
    import torch

    import cme213x  # noqa: F401
    from cme213x.ops import elementwise
    from cme213x.ops.gemm import gemv

    out = open(args.out, "a") if args.out else None

    def emit(**kw):
        s = json.dumps(kw)
        print(s, flush=True)
        if out:
            out.write(s + "\n")
            out.flush()

    def t_ms(fn, reps=5):
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return sorted(ts)[reps // 2]

    a = torch.empty(1 << 28, dtype=torch.float32, device="cuda")
    b = torch.empty_like(a)
    elementwise.copy_(b, a)
    copy_GBps = 2 * a.numel() * 4 / t_ms(lambda: elementwise.copy_(b, a)) / 1e6
    del a, b
    emit(bench="copy", GBps=round(copy_GBps, 1))

    shapes = [(8192, 8192), (16384, 16384), (16384, 2048), (2048, 16384), (8192, 1024), (65536, 256), (4096, 4096)]
    for dt in (torch.float32, torch.float64):
        for M, K in shapes:
            nbytes = (M * K + M + K) * (4 if dt == torch.float32 else 8)
            R = max(1, min(16, -(-FOOTPRINT // nbytes)))
            As = [torch.randn(M, K, dtype=dt, device="cuda") for _ in range(R)]
            x = torch.randn(K, dtype=dt, device="cuda")
            y = torch.empty(M, dtype=dt, device="cuda")
            err = float((gemv(As[0], x, y) - As[0] @ x).abs().max())
            res = {}
            for name, fn in (("cme_gemv", lambda A: gemv(A, x, y)), ("torch.mv", lambda A: torch.mv(A, x, out=y))):
                def loop(fn=fn):
                    for i in range(args.calls):
                        fn(As[i % R])

                loop()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    loop()
                g.replay()
                torch.cuda.synchronize()
                ms = t_ms(g.replay) / args.calls
                res[name] = ms
                del g
            emit(bench="gemv", dtype=str(dt).split(".")[-1], M=M, K=K, sets=R, max_abs_err=err,
                 **{f"ms_{k}": round(v, 5) for k, v in res.items()},
                 GBps=round(nbytes / res["cme_gemv"] / 1e6, 1),
                 pct_copy=round(100 * nbytes / res["cme_gemv"] / 1e6 / copy_GBps, 1),
                 speedup_vs_torch=round(res["torch.mv"] / res["cme_gemv"], 3))
            del As
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
