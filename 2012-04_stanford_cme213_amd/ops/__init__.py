from . import stencil, elementwise, graph, scan, transpose, spmv, sort, text  # noqa: F401
