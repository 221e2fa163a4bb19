from . import stencil, elementwise, graph, scan  # noqa: F401
