from . import comm, decomp, collectives, rccl  # noqa: F401
