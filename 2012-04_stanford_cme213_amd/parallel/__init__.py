from . import comm, decomp, collectives  # noqa: F401
