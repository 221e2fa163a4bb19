from . import params, ulp, timer, gridio  # noqa: F401
