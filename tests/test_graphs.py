"""hipGraph capture of native loops (utils/graphs.py): replay must equal eager
execution bit for bit."""
import numpy as np
import pytest
import torch


@pytest.mark.gpu
def test_graph_replay_spmv_scan(gpu):
    from cme213x.models.spmv_scan import SpmvScanSolver, generate
    from cme213x.utils.graphs import GraphRunner

    prob = generate(37035, 3128, 1000, 6, seed=4)
    eager = SpmvScanSolver(prob, gpu)
    ref = eager.run().clone()
    sol = SpmvScanSolver(prob, gpu)
    g = GraphRunner(lambda: sol.run(), warmup=0)  # capture records, does not execute
    g()
    torch.cuda.synchronize()
    # look-back reassociation may differ in the last bits run to run
    np.testing.assert_allclose(sol.a.cpu().numpy(), ref.cpu().numpy(), rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_graph_replay_heat(gpu):
    from cme213x.models.heat2d import HeatGrid
    from cme213x.utils.graphs import GraphRunner
    from cme213x.utils.params import SimParams

    p = SimParams(nx=700, ny=500, order=8)
    a = HeatGrid(p, torch.float32, gpu)
    b = HeatGrid(p, torch.float32, gpu)
    a.run(16, "stream2_fma")
    # capture 8 steps = 4 two-step passes (the state returns to buffer 0, so
    # the recorded pointers stay valid for the next replay); capture records
    # without executing
    g = GraphRunner(lambda: b.run(8, "stream2_fma"), warmup=0)
    b.cur = 0
    g()
    g()
    torch.cuda.synchronize()
    assert torch.equal(a.buf[0], b.buf[0])
