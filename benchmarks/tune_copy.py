#!/usr/bin/env python3
"""Calibrate the achievable HBM copy rate (the ceiling for every streaming
kernel): unroll x non-temporal x grid size, plus a block-contiguous variant
and torch's own copy. 1 GiB source, median of 5 interleaved rounds."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import cme213x
    from cme213x import _ext

    _ext.proto(_ext.HIP_PROTOS, "cme_copy_tune", "ppqiiiip")
    nbytes = int(os.environ.get("COPY_BYTES", str(1 << 30)))
    a = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda").uniform_()
    b = torch.empty_like(a)
    s = _ext.stream_ptr()
    cfgs = [(0, u, nt, bpc) for u in (1, 2, 4, 8) for nt in (0, 1) for bpc in (2, 4, 8, 16, 32)]
    cfgs += [(1, 4, 0, bpc) for bpc in (1, 2, 4, 8)]
    cfgs += [(2, u, 1, 0) for u in (1, 2, 4, 8)]  # one-shot tiles
    times = {c: [] for c in cfgs}
    times["torch"] = []
    for _ in range(5):
        for c in cfgs + ["torch"]:
            if c == "torch":
                fn = lambda: b.copy_(a)  # noqa: E731
            else:
                fn = lambda c=c: _ext.call_hip("cme_copy_tune", a.data_ptr(), b.data_ptr(), nbytes, *c, s)  # noqa
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                fn()
            e1.record()
            e1.synchronize()
            times[c].append(e0.elapsed_time(e1) / 5)
    for c, t in sorted(times.items(), key=lambda kv: sorted(kv[1])[2]):
        ms = sorted(t)[2]
        print(json.dumps({"cfg": c, "ms": round(ms, 4), "GBps": round(2 * nbytes / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
