from . import stencil, elementwise, graph  # noqa: F401
