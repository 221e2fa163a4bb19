from . import heat2d, heat2d_dist, cipher, pagerank  # noqa: F401
