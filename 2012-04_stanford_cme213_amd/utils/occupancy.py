"""Kernel resource / occupancy report and Little's-law sizing.

The reference ships the CUDA Occupancy Calculator spreadsheet and teaches
``ptxas -v`` + Little's law (``refs/CUDA_Occupancy_Calculator.xls``;
``slides/Lecture08.pdf`` 7-9, ``slides/Lecture09.pdf`` 2-3). Here the native
library registers its main kernels (``CME_REGISTER_KERNEL``) and
``cme_kernel_query`` reports, from the HIP runtime of the running device,
VGPRs, static LDS, scratch (spills), and resident blocks per CU from the
occupancy API; :func:`littles_law` gives the bytes that must be in flight to
saturate HBM.

    python -m cme213x occupancy
"""
from __future__ import annotations

import ctypes

from .. import _ext

_ext.proto(_ext.HIP_PROTOS, "cme_kernel_count", "")
_ext.proto(_ext.HIP_PROTOS, "cme_kernel_query", "ipip")

FIELDS = ("block", "vgprs", "lds_bytes", "scratch_bytes", "max_threads", "blocks_per_cu", "waves_per_simd",
          "max_dyn_lds")

# MI355X (gfx950): 256 CUs x 4 SIMDs, <= 8 waves per SIMD (wave64),
# 512 VGPRs per lane per SIMD budget, 160 KB LDS per CU.
MAX_WAVES_PER_SIMD = 8
LDS_PER_CU = 160 * 1024


def kernel_report() -> list[dict]:
    """One dict per registered kernel (needs a GPU: the runtime answers)."""
    n = _ext._fn("hip", "cme_kernel_count")()
    rows = []
    for i in range(n):
        name = ctypes.create_string_buffer(128)
        out = (ctypes.c_int * 8)()
        _ext.call_hip("cme_kernel_query", i, ctypes.addressof(name), 128, ctypes.addressof(out))
        r = {"kernel": name.value.decode()}
        r.update(dict(zip(FIELDS, list(out))))
        r["occupancy"] = round(r["waves_per_simd"] / MAX_WAVES_PER_SIMD, 3)
        rows.append(r)
    return rows


def littles_law(bandwidth_Bps: float = 8.0e12, latency_s: float = 1.0e-6, cus: int = 256) -> dict:
    """Bytes in flight needed to sustain ``bandwidth`` at ``latency``
    (concurrency = throughput x latency), total and per CU, and the 16-B
    loads per lane that implies at full occupancy."""
    total = bandwidth_Bps * latency_s
    per_cu = total / cus
    lanes = 4 * MAX_WAVES_PER_SIMD * 64
    return {"bytes_in_flight": total, "bytes_per_cu": per_cu, "loads16_per_lane_at_full_occupancy": per_cu / lanes / 16}


def format_report(rows: list[dict]) -> str:
    cols = ("kernel",) + FIELDS[:6] + ("occupancy",)
    w = {c: max(len(c), *(len(str(r[c])) for r in rows)) for c in cols}
    lines = ["  ".join(c.ljust(w[c]) for c in cols)]
    for r in rows:
        lines.append("  ".join(str(r[c]).ljust(w[c]) for c in cols))
    return "\n".join(lines)


def main(argv=None) -> int:
    rows = kernel_report()
    print(format_report(rows))
    ll = littles_law()
    print(f"\nLittle's law @ 8 TB/s, 1 us: {ll['bytes_in_flight'] / 2**20:.1f} MiB in flight, "
          f"{ll['bytes_per_cu'] / 1024:.1f} KiB per CU, {ll['loads16_per_lane_at_full_occupancy']:.2f} "
          f"16-B loads per lane at full occupancy")
    return 0
