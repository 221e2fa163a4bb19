from . import params, ulp, timer, gridio, mmio, occupancy, graphs  # noqa: F401
