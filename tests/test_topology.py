"""Cartesian topologies, blocking point-to-point, vector datatypes (gloo
ranks, CPU) and the performance-model helpers (SURVEY §2.3 lecture MPI
features; slides/Lecture18.pdf, Lecture20.pdf)."""
import math

import pytest
import torch

from dist_util import run_ranks


def test_dims_create_matches_mpi():
    from cme213x.parallel.topology import dims_create

    assert dims_create(8, 2) == [4, 2]
    assert dims_create(16, 2) == [4, 4]
    assert dims_create(12, 3) == [3, 2, 2]
    assert dims_create(7, 2) == [7, 1]
    assert dims_create(8, 2, [0, 4]) == [2, 4]
    assert dims_create(1, 3) == [1, 1, 1]
    with pytest.raises(ValueError):
        dims_create(9, 2, [2, 0])


def test_cart_coords_rank_shift_single_process():
    from cme213x.parallel.comm import Comm
    from cme213x.parallel.topology import CartComm, all_coords

    class Fake(Comm):
        def __init__(self, rank, size):
            self.rank, self.size = rank, size

    dims = [2, 3]
    for r in range(6):
        c = CartComm(Fake(r, 6), dims, [False, True])
        assert c.coords(r) == all_coords(dims)[r]
        assert c.rank_of(c.coords(r)) == r
    c = CartComm(Fake(0, 6), dims, [False, True])  # coords (0, 0)
    assert c.shift(0, 1) == (-1, 3)  # non-periodic rows: nothing above row 0
    assert c.shift(1, 1) == (2, 1)  # periodic columns wrap
    assert c.neighbours() == {(0, -1): -1, (0, 1): 3, (1, -1): 2, (1, 1): 1}
    with pytest.raises(ValueError):
        CartComm(Fake(0, 6), [4, 2])


def _cart_rank(rank, world):
    from cme213x.parallel.comm import TorchComm
    from cme213x.parallel.topology import cart_create, sendrecv

    comm = TorchComm()
    cart = cart_create(comm, [0, 0], [False, False])  # 2 x 2
    r, c = cart.my_coords
    # row / column sub-communicators: sums of the global rank along each
    rows = cart.sub([False, True])
    cols = cart.sub([True, False])
    t = torch.tensor([float(rank)])
    rows.comm.allreduce_(t)
    u = torch.tensor([float(rank)])
    cols.comm.allreduce_(u)
    # face halo exchange: send my rank to every neighbour
    sends = {k: torch.tensor([float(rank)]) for k in [(0, -1), (0, 1), (1, -1), (1, 1)]}
    recvs = {k: torch.full((1,), -1.0) for k in sends}
    cart.halo_exchange(sends, recvs).wait()
    got = {k: int(v.item()) for k, v in recvs.items()}
    # periodic ring of all ranks: sendrecv shift by one
    ring = cart_create(comm, [world], [True])
    src, dst = ring.shift(0, 1)
    out = sendrecv(comm, torch.tensor([10.0 * rank]), dst, torch.empty(1), src)
    return (r, c, rows.size, cols.size, t.item(), u.item(), got, out.item(), cart.neighbours())


def test_cart_sub_halo_and_sendrecv_gloo():
    out = run_ranks(_cart_rank, 4)
    for rank, (r, c, nrow, ncol, rsum, csum, got, ring, nb) in enumerate(out):
        assert (r, c) == divmod(rank, 2)
        assert nrow == 2 and ncol == 2
        assert rsum == sum(q for q in range(4) if q // 2 == r)
        assert csum == sum(q for q in range(4) if q % 2 == c)
        for k, v in got.items():
            assert v == (nb[k] if nb[k] >= 0 else -1)
        assert ring == 10.0 * ((rank - 1) % 4)


def test_vector_type_pack_unpack():
    from cme213x.parallel.topology import VectorType

    g = torch.arange(6 * 8, dtype=torch.float32).reshape(6, 8)
    col = VectorType(count=6, blocklength=2, stride=8)  # a 2-wide column halo
    packed = col.pack(g, offset=5)
    assert torch.equal(packed, g[:, 5:7].reshape(-1))
    h = torch.zeros_like(g)
    col.unpack(packed, h, offset=1)
    assert torch.equal(h[:, 1:3], g[:, 5:7])
    assert h.sum() == g[:, 5:7].sum()
    with pytest.raises(ValueError):
        col.view(g, offset=7)  # runs past the end


def test_perf_models():
    from cme213x.utils import perfmodel as pm

    assert pm.amdahl(0.0, 8) == 8
    assert pm.amdahl(0.1, 8) == pytest.approx(1 / (0.1 + 0.9 / 8))
    assert pm.amdahl_limit(0.05) == pytest.approx(20)
    assert pm.gustafson(0.1, 8) == pytest.approx(8 - 0.7)
    # Karp-Flatt recovers Amdahl's serial fraction
    assert pm.karp_flatt(pm.amdahl(0.2, 16), 16) == pytest.approx(0.2)
    assert pm.efficiency(10.0, 2.5, 4) == pytest.approx(1.0)
    # iso-efficiency: n(p) keeps the tree dot product at the target efficiency
    for p in (2, 8, 64):
        n = pm.isoefficiency_n(p, 0.8)
        assert pm.tree_dot_efficiency(n, p) == pytest.approx(0.8)
    assert pm.isoefficiency_n(64, 0.8) / pm.isoefficiency_n(8, 0.8) == pytest.approx(64 * 6 / (8 * 3))
    # stencil model: overlap hides the exchange while compute dominates
    m1 = pm.stencil_strong_scaling(16384, 8, 8 / 3, halo_rows=12, steps_per_exchange=3)
    assert m1["exchange_s"] < m1["compute_s"] and m1["efficiency"] == pytest.approx(1.0)
    m2 = pm.stencil_strong_scaling(1024, 8, 8 / 3, halo_rows=12)
    assert m2["efficiency"] < 0.5  # latency-bound small grid
    assert pm.ring_allreduce_time(1 << 30, 8) > pm.ring_allreduce_time(1 << 20, 8) > 0
    assert math.isinf(pm.amdahl_limit(0))
