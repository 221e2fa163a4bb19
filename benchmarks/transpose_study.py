#!/usr/bin/env python3
"""8192^2 LDS-tiled transpose bank-conflict padding study (BASELINE.json
config #2): runs every variant 5x so rocprofv3 --pmc can attribute
SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE per kernel."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import cme213x  # noqa: E402,F401
from cme213x.ops.transpose import VARIANTS, transpose  # noqa: E402

n = int(os.environ.get("N", "8192"))
x = torch.rand(n, n, device="cuda")
out = torch.empty_like(x)
for v in VARIANTS:
    for _ in range(5):
        transpose(x, v, out)
torch.cuda.synchronize()
print("done")
