import math

import pytest
import torch

from cme213x.ops.atomics import global_max, monte_carlo_pi, segment_sums_workqueue


def test_mc_pi_cpu():
    pi, hits = monte_carlo_pi(1 << 20, seed=7, device="cpu")
    assert abs(pi - math.pi) < 0.01


@pytest.mark.gpu
def test_mc_pi_gpu_matches_cpu_stream(gpu):
    n = 3_000_017
    assert monte_carlo_pi(n, 11, gpu)[1] == monte_carlo_pi(n, 11, "cpu")[1]


@pytest.mark.gpu
def test_global_max_gpu(gpu):
    for x in (torch.randn(1_000_003), -torch.rand(5000) - 1.0, torch.tensor([3.5]), torch.randn(1 << 24)):
        assert global_max(x.to(gpu)) == float(x.max())
    # unaligned start (scalar path) and a maximum in the scalar tail
    x = torch.randn(100_001)
    x[-1] = 50.0
    assert global_max(x.to(gpu)[1:]) == 50.0


@pytest.mark.gpu
def test_workqueue_gpu(gpu):
    lens = torch.randint(0, 3000, (5000,))
    lens[::97] = 100000  # ragged
    offs = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(lens, 0)]).to(torch.int32)
    v = torch.randint(-3, 4, (int(offs[-1]),)).float()
    ref = segment_sums_workqueue(offs, v)
    out = segment_sums_workqueue(offs.to(gpu), v.to(gpu)).cpu()
    assert torch.equal(out, ref)
