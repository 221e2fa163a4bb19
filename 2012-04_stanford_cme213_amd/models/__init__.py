from . import heat2d, heat2d_dist  # noqa: F401
