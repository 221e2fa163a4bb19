from . import heat2d, heat2d_dist, cipher, pagerank, spmv_scan, vigenere, dist_spmv  # noqa: F401
