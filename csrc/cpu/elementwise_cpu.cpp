// OpenMP CPU oracles for the streaming kernels (hw1 host_shift_cypher,
// hw/hw1/programming/cipher.cu:53-60) and the PageRank host propagate
// (hw/hw1/programming/pagerank.cu:45-67).
#include <cstddef>
#include <cstdint>

#include "cme213/cpu_common.h"

CME_CPU_EXPORT int cme_cpu_shift_cipher(const uint8_t* in, uint8_t* out, long long n, int shift) {
    const uint8_t s = (uint8_t)shift;
#pragma omp parallel for schedule(static)
    for (long long i = 0; i < n; ++i) out[i] = (uint8_t)(in[i] + s);
    return 0;
}

CME_CPU_EXPORT int cme_cpu_mul_f32(float* a, const float* b, long long n) {
#pragma omp parallel for schedule(static)
    for (long long i = 0; i < n; ++i) a[i] *= b[i];
    return 0;
}

// One propagate sweep with the reference's arithmetic (two loads per edge,
// sequential sum per row).
CME_CPU_EXPORT int cme_cpu_pr_propagate(const uint32_t* idx, const uint32_t* edges, const float* in, float* out,
                                        const float* inv, int n) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        float sum = 0.f;
        for (uint32_t j = idx[i]; j < idx[i + 1]; ++j) sum += in[edges[j]] * inv[edges[j]];
        out[i] = 0.5f / (float)n + 0.5f * sum;
    }
    return 0;
}
