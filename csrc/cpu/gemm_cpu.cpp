// OpenMP SGEMM (CPU path / oracle): C = alpha*A*B + beta*C, row-major,
// i-k-j loop order over 64-row blocks (unit-stride inner loop on B and C).
#include <cstddef>
#include <vector>

#include "cme213/cpu_common.h"

CME_CPU_EXPORT int cme_cpu_sgemm(int M, int N, int K, float alpha, const float* A, const float* B, float beta,
                                 float* C) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < M; ++i) {
        std::vector<float> row(N, 0.f);
        for (int k = 0; k < K; ++k) {
            const float a = A[(size_t)i * K + k];
            const float* b = B + (size_t)k * N;
            for (int j = 0; j < N; ++j) row[j] += a * b[j];
        }
        float* c = C + (size_t)i * N;
        for (int j = 0; j < N; ++j) c[j] = alpha * row[j] + (beta == 0.f ? 0.f : beta * c[j]);
    }
    return 0;
}

namespace {
template <typename T>
void gemv_t(int M, int K, T alpha, const T* A, const T* x, T beta, T* y) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < M; ++i) {
        const T* a = A + (size_t)i * K;
        T s = 0;
        for (int k = 0; k < K; ++k) s += a[k] * x[k];
        y[i] = alpha * s + (beta == T(0) ? T(0) : beta * y[i]);
    }
}
}  // namespace

// y = alpha*A x + beta*y, row-major A[M][K]; dtype 0 f32, 4 f64 (the dense
// matvecs of slides/Lecture20.pdf on the CPU path)
CME_CPU_EXPORT int cme_cpu_gemv(int M, int K, double alpha, const void* A, const void* x, double beta, void* y,
                                int dtype) {
    if (dtype == 0)
        gemv_t<float>(M, K, (float)alpha, (const float*)A, (const float*)x, (float)beta, (float*)y);
    else if (dtype == 4)
        gemv_t<double>(M, K, alpha, (const double*)A, (const double*)x, beta, (double*)y);
    else
        return 1;
    return 0;
}
