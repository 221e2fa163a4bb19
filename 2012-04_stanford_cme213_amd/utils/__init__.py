from . import params, ulp, timer, gridio, mmio, occupancy  # noqa: F401
