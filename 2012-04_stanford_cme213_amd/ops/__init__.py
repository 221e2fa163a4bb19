from . import stencil, elementwise, graph, scan, transpose, spmv  # noqa: F401
