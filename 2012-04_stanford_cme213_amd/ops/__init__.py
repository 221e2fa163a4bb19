from . import stencil, elementwise, graph, scan, transpose, spmv, sort, text, gemm, atomics, algorithms, studies  # noqa: F401
