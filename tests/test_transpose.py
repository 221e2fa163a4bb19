import pytest
import torch

from cme213x.ops.transpose import VARIANTS, transpose


@pytest.mark.parametrize("shape", [(1024, 1024), (37, 91), (64, 128)])
@pytest.mark.parametrize("variant", ["naive", "lds_pad"])
def test_transpose_cpu(shape, variant):
    x = torch.randn(shape)
    assert torch.equal(transpose(x, variant), x.t())


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(1024, 1024), (8192, 64), (37, 91), (100, 260), (516, 1028)])
@pytest.mark.parametrize("variant", [v for v in VARIANTS if v != "copy"])
def test_transpose_gpu(gpu, shape, variant):
    x = torch.randn(shape, device=gpu)
    assert torch.equal(transpose(x, variant), x.t())


@pytest.mark.gpu
def test_copy_variant_gpu(gpu):
    x = torch.randn(300, 200, device=gpu)
    assert torch.equal(transpose(x, "copy"), x)
