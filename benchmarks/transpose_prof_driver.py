#!/usr/bin/env python3
"""Tiny driver for rocprofv3 counter runs of the transpose ladder at 8192^2:
each variant runs 3 times (kernel names identify the variant)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import cme213x  # noqa: F401
    from cme213x.ops.transpose import transpose

    n = int(os.environ.get("N", "8192"))
    x = torch.rand(n, n, device="cuda")
    y = torch.empty_like(x)
    for v in ("lds", "lds_pad", "lds_swizzle", "diagonal", "vec"):
        for _ in range(3):
            transpose(x, v, out=y)
        torch.cuda.synchronize()
        assert torch.equal(y, x.t()), v
    print("ok", flush=True)


if __name__ == "__main__":
    main()
