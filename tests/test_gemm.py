import pytest
import torch

from cme213x.ops.gemm import sgemm


def test_sgemm_cpu():
    A, B, C = torch.randn(70, 50), torch.randn(50, 90), torch.randn(70, 90)
    out = sgemm(A, B, C.clone(), 1.5, 0.5)
    torch.testing.assert_close(out, 1.5 * A.double().mm(B.double()).float() + 0.5 * C, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(256, 384, 512), (128, 128, 32), (100, 70, 33), (512, 256, 1024)])
@pytest.mark.parametrize("variant", ["naive", "lds", "mfma"])
def test_sgemm_gpu(gpu, shape, variant):
    M, N, K = shape
    A, B, C = torch.randn(M, K), torch.randn(K, N), torch.randn(M, N)
    ref = (2.0 * A.double().mm(B.double()) + 0.25 * C.double()).float()
    out = sgemm(A.to(gpu), B.to(gpu), C.to(gpu), 2.0, 0.25, variant=variant).cpu()
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
def test_sgemm_mfma_asymmetric_identity(gpu):
    # A = I with an asymmetric B catches a transposed C/D register map
    n = 128
    A = torch.eye(n)
    B = torch.arange(n * n, dtype=torch.float32).view(n, n) / 1000.0
    out = sgemm(A.to(gpu), B.to(gpu), variant="mfma").cpu()
    assert torch.equal(out, B)
