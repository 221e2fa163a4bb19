#!/usr/bin/env python3
"""Sweep the vector-tile transpose (tile rows x cols, block remap) at 8192^2
and 4096^2; interleaved rounds, median of 5; effective GB/s = 2 * bytes / t."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import cme213x
    from cme213x import _ext

    _ext.proto(_ext.HIP_PROTOS, "cme_transpose_tune", "ppiiiiip")
    s = _ext.stream_ptr()
    sizes = [int(v) for v in os.environ.get("CME_TR_SIZES", "8192,4096,16384").split(",")]
    remaps = [int(v) for v in os.environ.get("CME_TR_REMAPS", "0,1,2").split(",")]
    tiles = [tuple(map(int, v.split("x"))) for v in os.environ.get("CME_TR_TILES", "64x64,64x128,128x64,128x128,256x64,256x128").split(",")]
    for n in sizes:
        x = torch.rand(n, n, device="cuda")
        y = torch.empty_like(x)
        cfgs = [(tr, tc, rm) for tr, tc in tiles for rm in remaps]
        times = {c: [] for c in cfgs}
        for _ in range(5):
            for c in cfgs:
                f = lambda: _ext.call_hip("cme_transpose_tune", x.data_ptr(), y.data_ptr(), n, n, *c, s)  # noqa
                f()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    f()
                e1.record()
                e1.synchronize()
                times[c].append(e0.elapsed_time(e1) / 5)
        for c in cfgs:  # every arm must transpose correctly
            y.zero_()
            _ext.call_hip("cme_transpose_tune", x.data_ptr(), y.data_ptr(), n, n, *c, s)
            assert torch.equal(y, x.t()), c
        for c in cfgs:
            ms = sorted(times[c])[2]
            print(json.dumps({"n": n, "tr": c[0], "tc": c[1], "remap": c[2], "ms": round(ms, 4),
                              "GBps": round(2 * n * n * 4 / ms / 1e6)}), flush=True)
        del x, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
