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


@pytest.mark.gpu
def test_transpose_diagnostics_and_reps(gpu):
    from cme213x.ops.transpose import diagnostic, transpose_reps

    n = 256
    x = torch.randn(n, n, device=gpu)
    T = 64
    xt = x.view(n // T, T, n // T, T)  # [tile_r, r, tile_c, c]
    # coarse: tile (I, J) lands at tile (J, I) with its elements untransposed
    coarse = xt.permute(2, 1, 0, 3).reshape(n, n)
    assert torch.equal(diagnostic(x, "coarse"), coarse)
    # fine: tile (I, J) stays, its elements are transposed
    fine = xt.permute(0, 3, 2, 1).reshape(n, n)
    assert torch.equal(diagnostic(x, "fine"), fine)
    assert torch.equal(transpose_reps(x, 5), x.t())
