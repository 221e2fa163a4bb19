from . import stencil, elementwise, graph, scan, transpose, spmv, sort, text, gemm, atomics  # noqa: F401
