"""Parallel performance models from ``slides/Lecture20.pdf`` (last slides):
speed-up and efficiency, Amdahl's and Gustafson's laws, the Karp-Flatt
serial fraction, and the iso-efficiency of the tree dot product -- plus the
two MI355X cost models the framework's own scaling is reasoned with: a
strong-scaled halo-exchange stencil and a ring collective over xGMI links.

These are pure functions (no GPU); ``benchmarks/`` and the docs use them to
put measured scaling curves next to the model.
"""
from __future__ import annotations

import math

# MI355X constants (MI355X_MICROARCH.md): achievable HBM copy rate and one
# xGMI link's rate; 7 links per GPU in an 8-GPU node.
HBM_BPS = 6.3e12
XGMI_LINK_BPS = 153e9
XGMI_LINKS = 7


def speedup(t1: float, tp: float) -> float:
    """S(p) = T(1) / T(p)."""
    return t1 / tp


def efficiency(t1: float, tp: float, p: int) -> float:
    """E(p) = S(p) / p."""
    return t1 / (tp * p)


def amdahl(serial_fraction: float, p: float) -> float:
    """Amdahl: fixed problem, S(p) = 1 / (f + (1 - f) / p)."""
    if not 0.0 <= serial_fraction <= 1.0:
        raise ValueError("serial fraction must be in [0, 1]")
    return 1.0 / (serial_fraction + (1.0 - serial_fraction) / p)


def amdahl_limit(serial_fraction: float) -> float:
    """lim_{p->inf} of Amdahl's speed-up: 1 / f."""
    return math.inf if serial_fraction == 0 else 1.0 / serial_fraction


def gustafson(serial_fraction: float, p: float) -> float:
    """Gustafson: problem grows with p (fixed time), scaled speed-up
    S(p) = p - f (p - 1), f = serial fraction of the PARALLEL run."""
    if not 0.0 <= serial_fraction <= 1.0:
        raise ValueError("serial fraction must be in [0, 1]")
    return p - serial_fraction * (p - 1)


def karp_flatt(measured_speedup: float, p: int) -> float:
    """Experimentally determined serial fraction e = (1/S - 1/p) / (1 - 1/p);
    a value that grows with p points at overhead (communication), a constant
    one at a true serial part."""
    if p <= 1:
        raise ValueError("p must be > 1")
    return (1.0 / measured_speedup - 1.0 / p) / (1.0 - 1.0 / p)


def tree_dot_time(n: int, p: int, t_flop: float = 1.0, t_comm: float = 1.0) -> float:
    """Parallel dot product of length n on p ranks: n/p local multiply-adds
    then a log2(p)-deep reduction tree, each level one add + one message."""
    return 2.0 * n / p * t_flop + math.ceil(math.log2(p)) * (t_flop + t_comm) if p > 1 else 2.0 * n * t_flop


def tree_dot_efficiency(n: int, p: int, t_flop: float = 1.0, t_comm: float = 1.0) -> float:
    return tree_dot_time(n, 1, t_flop, t_comm) / (p * tree_dot_time(n, p, t_flop, t_comm))


def isoefficiency_n(p: int, target_efficiency: float, t_flop: float = 1.0, t_comm: float = 1.0) -> float:
    """Problem size n that keeps the tree dot product at ``target_efficiency``
    on p ranks. E = 2n / (2n + p log p (t_flop + t_comm)/t_flop) gives
    n = E/(1-E) * p log2 p (t_flop + t_comm) / (2 t_flop): the iso-efficiency
    function is Theta(p log p)."""
    if not 0.0 < target_efficiency < 1.0:
        raise ValueError("target efficiency must be in (0, 1)")
    if p <= 1:
        return 0.0
    e = target_efficiency
    return e / (1.0 - e) * p * math.ceil(math.log2(p)) * (t_flop + t_comm) / (2.0 * t_flop)


def stencil_strong_scaling(n: int, p: int, bytes_per_point: float, halo_rows: int, elem_bytes: int = 4,
                           t_step_fixed: float = 0.0, hbm_bps: float = HBM_BPS,
                           link_bps: float = XGMI_LINK_BPS, latency_s: float = 10e-6,
                           overlap: bool = True, steps_per_exchange: int = 1) -> dict:
    """Per-step time of an n x n stencil strong-scaled over p GPUs in 1-D
    stripes: compute = n*n/p points x bytes_per_point / HBM rate; exchange =
    two messages of halo_rows x n elements, each on its own xGMI link, plus
    a latency, once per ``steps_per_exchange`` steps (temporal blocking:
    halo_rows = steps x B); overlapped (async mode) the step costs the larger
    of the two, otherwise their sum. ``t_step_fixed`` adds launch/border
    overheads."""
    compute = n * n / p * bytes_per_point / hbm_bps
    exchange = 0.0 if p == 1 else (latency_s + halo_rows * n * elem_bytes / link_bps) / steps_per_exchange
    step = (max(compute, exchange) if overlap else compute + exchange) + t_step_fixed
    t1 = n * n * bytes_per_point / hbm_bps + t_step_fixed
    return {"compute_s": compute, "exchange_s": exchange, "step_s": step, "speedup": t1 / step,
            "efficiency": t1 / (p * step)}


def ring_allreduce_time(nbytes: float, p: int, link_bps: float = XGMI_LINK_BPS, latency_s: float = 5e-6) -> float:
    """Ring all-reduce: 2(p-1) steps, each moving nbytes/p over one link --
    per-link bound on point-to-point xGMI (what bucket sizes must amortise)."""
    if p <= 1:
        return 0.0
    return 2 * (p - 1) * (latency_s + nbytes / p / link_bps)
