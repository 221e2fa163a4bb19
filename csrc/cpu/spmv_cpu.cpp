// OpenMP CSR SpMV (oracle and CPU path): y = A x + beta*y, rows in parallel.
#include "cme213/cpu_common.h"

CME_CPU_EXPORT int cme_cpu_spmv_csr(int nrows, const int* rp, const int* col, const float* val, const float* x,
                                    float* y, float beta) {
#pragma omp parallel for schedule(static)
    for (int r = 0; r < nrows; ++r) {
        float s = 0.f;
        for (int j = rp[r]; j < rp[r + 1]; ++j) s += val[j] * x[col[j]];
        y[r] = beta == 0.f ? s : beta * y[r] + s;
    }
    return 0;
}

// out[i] = x[idx[i]]: the send-side pack of the distributed SpMV halo
CME_CPU_EXPORT int cme_cpu_gather_f32(int n, const float* x, const int* idx, float* out) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) out[i] = x[idx[i]];
    return 0;
}

// y[rows[b]] += sum_j val[j] * h[col[j]] over the compact boundary rows
// (rows distinct): the off-rank columns of a row-partitioned SpMV
CME_CPU_EXPORT int cme_cpu_spmv_halo(int nb, const int* rows, const int* rp, const int* col, const float* val,
                                     const float* h, float* y) {
#pragma omp parallel for schedule(static)
    for (int b = 0; b < nb; ++b) {
        float s = 0.f;
        for (int j = rp[b]; j < rp[b + 1]; ++j) s += val[j] * h[col[j]];
        y[rows[b]] += s;
    }
    return 0;
}
