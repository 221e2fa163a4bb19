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
