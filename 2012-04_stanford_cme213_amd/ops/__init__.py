from . import stencil, elementwise, graph, scan, transpose, spmv, sort, text, gemm, atomics, algorithms, studies  # noqa: F401
from . import library  # noqa: F401  (registers torch.ops.cme213x.*)
