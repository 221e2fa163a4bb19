import pytest
import torch

from cme213x.ops.gemm import gemv, sgemm


def test_sgemm_cpu():
    A, B, C = torch.randn(70, 50), torch.randn(50, 90), torch.randn(70, 90)
    out = sgemm(A, B, C.clone(), 1.5, 0.5)
    torch.testing.assert_close(out, 1.5 * A.double().mm(B.double()).float() + 0.5 * C, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(256, 384, 512), (128, 128, 32), (100, 70, 33), (512, 256, 1024), (256, 256, 32),
                                   (768, 512, 96), (1024, 1024, 2048), (4096, 4096, 64)])
@pytest.mark.parametrize("variant", ["naive", "lds", "mfma"])
def test_sgemm_gpu(gpu, shape, variant):
    M, N, K = shape
    A, B, C = torch.randn(M, K), torch.randn(K, N), torch.randn(M, N)
    ref = (2.0 * A.double().mm(B.double()) + 0.25 * C.double()).float()
    out = sgemm(A.to(gpu), B.to(gpu), C.to(gpu), 2.0, 0.25, variant=variant).cpu()
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [128, 512, 4096])
def test_sgemm_mfma_asymmetric_identity(gpu, n):
    # A = I with an asymmetric B catches a transposed C/D register map
    # (n <= 512: the 128x128 kernel; 4096 fills the CUs with 256x256 blocks)
    A = torch.eye(n)
    B = torch.arange(n * n, dtype=torch.float32).view(n, n) / 1000.0
    out = sgemm(A.to(gpu), B.to(gpu), variant="mfma").cpu()
    assert torch.equal(out, B)
    out = sgemm(B.to(gpu), A.to(gpu), variant="mfma").cpu()
    assert torch.equal(out, B)


GEMV_SHAPES = [(1, 1), (7, 3), (64, 64), (300, 1001), (1000, 4096), (33, 20000), (4099, 130)]


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_gemv_cpu(dtype):
    for M, K in GEMV_SHAPES[:5]:
        A, x, y = torch.randn(M, K, dtype=dtype), torch.randn(K, dtype=dtype), torch.randn(M, dtype=dtype)
        ref = 1.5 * (A.double() @ x.double()) - 0.5 * y.double()
        out = gemv(A, x, y.clone(), 1.5, -0.5)
        tol = 1e-4 if dtype == torch.float32 else 1e-10
        torch.testing.assert_close(out.double(), ref, rtol=tol, atol=tol * max(1.0, K ** 0.5))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("shape", GEMV_SHAPES)
def test_gemv_gpu(gpu, dtype, shape):
    M, K = shape
    A, x, y = torch.randn(M, K, dtype=dtype), torch.randn(K, dtype=dtype), torch.randn(M, dtype=dtype)
    ref = 2.0 * (A.double() @ x.double()) + 0.25 * y.double()
    out = gemv(A.to(gpu), x.to(gpu), y.to(gpu), 2.0, 0.25).cpu()
    tol = 1e-4 if dtype == torch.float32 else 1e-10
    torch.testing.assert_close(out.double(), ref, rtol=tol, atol=tol * max(1.0, K ** 0.5))
    # unaligned operands take the scalar-load kernel
    buf = torch.randn(M * K + 1, dtype=dtype, device=gpu)
    Au = buf[1:].view(M, K)
    out2 = gemv(Au, x.to(gpu)).cpu()
    torch.testing.assert_close(out2.double(), Au.cpu().double() @ x.double(), rtol=tol, atol=tol * max(1.0, K ** 0.5))


@pytest.mark.gpu
def test_sgemm_mfma_misaligned_c_view(gpu):
    """the MFMA epilogue stores 16-B vectors of C; an offset view of
    C (4-B aligned only) must take the fallback, not misaligned vector stores."""
    M = N = 256
    K = 64
    A, B = torch.randn(M, K), torch.randn(K, N)
    big = torch.randn(M * N + 1)
    Cv = big[1:].view(M, N)
    ref = (A.double().mm(B.double()) + 0.5 * Cv.double()).float()
    Cg = big.to(gpu)[1:].view(M, N)
    out = sgemm(A.to(gpu), B.to(gpu), Cg, 1.0, 0.5, variant="mfma").cpu()
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-3)
