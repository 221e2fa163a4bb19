// OpenMP CPU transpose (BASELINE.json config #1: 1024x1024 fp32 without a
// GPU). Cache-blocked 64x64 tiles, parallel over tile rows; `naive` is the
// one-loop reference (my-refs/cuda_many_cores.pdf p.17 semantics).
#include <cstddef>

#include "cme213/cpu_common.h"

CME_CPU_EXPORT int cme_cpu_transpose_f32(const float* in, float* out, int rows, int cols, int blocked) {
    if (!blocked) {
#pragma omp parallel for schedule(static)
        for (int r = 0; r < rows; ++r)
            for (int c = 0; c < cols; ++c) out[(size_t)c * rows + r] = in[(size_t)r * cols + c];
        return 0;
    }
    constexpr int B = 64;
#pragma omp parallel for collapse(2) schedule(static)
    for (int rb = 0; rb < rows; rb += B)
        for (int cb = 0; cb < cols; cb += B) {
            const int re = rb + B < rows ? rb + B : rows;
            const int ce = cb + B < cols ? cb + B : cols;
            for (int c = cb; c < ce; ++c)
                for (int r = rb; r < re; ++r) out[(size_t)c * rows + r] = in[(size_t)r * cols + c];
        }
    return 0;
}
