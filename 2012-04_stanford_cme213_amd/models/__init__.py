from . import heat2d, heat2d_dist, cipher, pagerank, spmv_scan  # noqa: F401
