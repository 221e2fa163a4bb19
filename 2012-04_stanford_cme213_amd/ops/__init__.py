from . import stencil  # noqa: F401
