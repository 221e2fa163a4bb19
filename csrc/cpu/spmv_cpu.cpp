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
