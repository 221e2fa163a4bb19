from . import comm, decomp  # noqa: F401
