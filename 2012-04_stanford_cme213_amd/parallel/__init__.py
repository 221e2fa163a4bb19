from . import comm, decomp, collectives, rccl, dist_scan  # noqa: F401
