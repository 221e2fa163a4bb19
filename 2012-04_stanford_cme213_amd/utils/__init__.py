from . import params, ulp, timer, gridio, mmio  # noqa: F401
