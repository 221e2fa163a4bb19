from . import heat2d, heat2d_dist, cipher, pagerank, spmv_scan, vigenere  # noqa: F401
