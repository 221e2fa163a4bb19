"""cme213x -- MI355X-native parallel primitives and numerical kernels with the
capabilities of the Stanford CME213 (2012) coursework.

Layout:
    ops/       thin PyTorch-ROCm wrappers over the hand-written HIP kernels
               (csrc/hip) and OpenMP CPU backends (csrc/cpu)
    models/    the course workloads as reusable solvers/drivers (heat2d,
               distributed heat2d, pagerank, cipher, vigenere, sorts, SpMV,
               segmented SpMV-scan)
    parallel/  communicators (RCCL/gloo/loopback), decomposition, halo exchange
    utils/     timers, ULP compare, params files, reference-format I/O
    drivers/   command-line programs keeping the reference's argv / output files

The on-disk package name is ``2012-04_stanford_cme213_amd``; ``import cme213x``
is the importable alias (see ``cme213x/__init__.py``).
"""
from __future__ import annotations

import torch  # noqa: F401  (load torch's HIP runtime before our native libs)

from . import _ext  # noqa: F401
from . import utils, ops, parallel, models  # noqa: F401

__version__ = "0.1.0"
