// OpenMP CPU backend for the 2-D heat stencil: the correctness oracle for the
// HIP kernels and the GPU-less execution path.
//
// Mirrors the reference's cpuComputation (hw/hw2/solution/2dHeat_solution.cu:
// 371-411) and the hw5 per-rank compute loops, over an arbitrary region of a
// pitched grid, parallelised over rows with OpenMP.
#include <cstddef>

#include "cme213/cpu_common.h"
#include "cme213/heat_stencil.h"

using namespace cme;

namespace {

// FMA: 0 exact (contraction off), 1 FMA-contracted, 2 reassociated ("fast")
template <typename T, int ORDER, int FMA>
void heat_region(const T* prev, T* curr, int pitch, int xb, int xe, int yb, int ye, T xcfl, T ycfl) {
    constexpr int B = HeatOrder<ORDER>::B;
    const HeatFast<ORDER, T> fc = heat_fast_coefs<ORDER>(xcfl, ycfl);
#pragma omp parallel for schedule(static)
    for (int y = yb; y < ye; ++y) {
        const T* row = prev + (size_t)y * pitch;
        T* out = curr + (size_t)y * pitch;
        for (int x = xb; x < xe; ++x) {
            T xm[B], xp[B], ym[B], yp[B];
            for (int k = 0; k < B; ++k) {
                xm[k] = row[x - (k + 1)];
                xp[k] = row[x + (k + 1)];
                ym[k] = row[x - (ptrdiff_t)(k + 1) * pitch];
                yp[k] = row[x + (ptrdiff_t)(k + 1) * pitch];
            }
            if constexpr (FMA == 2)
                out[x] = heat_update_fast<ORDER>(row[x], xm, xp, ym, yp, fc);
            else
                out[x] = heat_update_sel<ORDER, FMA == 1>(row[x], xm, xp, ym, yp, xcfl, ycfl);
        }
    }
}

template <typename T, int FMA = 0>
int heat_dispatch(const T* prev, T* curr, int pitch, int xb, int xe, int yb, int ye, int order, T xcfl, T ycfl) {
    switch (order) {
        case 2: heat_region<T, 2, FMA>(prev, curr, pitch, xb, xe, yb, ye, xcfl, ycfl); return 0;
        case 4: heat_region<T, 4, FMA>(prev, curr, pitch, xb, xe, yb, ye, xcfl, ycfl); return 0;
        case 8: heat_region<T, 8, FMA>(prev, curr, pitch, xb, xe, yb, ye, xcfl, ycfl); return 0;
        default: return 1;
    }
}

}  // namespace

CME_CPU_EXPORT int cme_cpu_heat_step_f32(const float* prev, float* curr, int pitch, int xb, int xe, int yb, int ye,
                                         int order, float xcfl, float ycfl) {
    return heat_dispatch<float>(prev, curr, pitch, xb, xe, yb, ye, order, xcfl, ycfl);
}

CME_CPU_EXPORT int cme_cpu_heat_step_f64(const double* prev, double* curr, int pitch, int xb, int xe, int yb, int ye,
                                         int order, double xcfl, double ycfl) {
    return heat_dispatch<double>(prev, curr, pitch, xb, xe, yb, ye, order, xcfl, ycfl);
}

CME_CPU_EXPORT int cme_cpu_heat_run_f32(float* a, float* b, int pitch, int xb, int xe, int yb, int ye, int order,
                                        float xcfl, float ycfl, int iters) {
    for (int i = 0; i < iters; ++i) {
        int rc = heat_dispatch<float>((i & 1) ? b : a, (i & 1) ? a : b, pitch, xb, xe, yb, ye, order, xcfl, ycfl);
        if (rc) return rc;
    }
    return 0;
}

CME_CPU_EXPORT int cme_cpu_heat_run_f64(double* a, double* b, int pitch, int xb, int xe, int yb, int ye, int order,
                                        double xcfl, double ycfl, int iters) {
    for (int i = 0; i < iters; ++i) {
        int rc = heat_dispatch<double>((i & 1) ? b : a, (i & 1) ? a : b, pitch, xb, xe, yb, ye, order, xcfl, ycfl);
        if (rc) return rc;
    }
    return 0;
}

// FMA-contracted oracle (heat_update_fma): bitwise reference for the GPU's
// FMA stencil variants (std::fma is correctly rounded).
CME_CPU_EXPORT int cme_cpu_heat_step_fma_f32(const float* prev, float* curr, int pitch, int xb, int xe, int yb, int ye,
                                             int order, float xcfl, float ycfl) {
    return heat_dispatch<float, 1>(prev, curr, pitch, xb, xe, yb, ye, order, xcfl, ycfl);
}

CME_CPU_EXPORT int cme_cpu_heat_step_fma_f64(const double* prev, double* curr, int pitch, int xb, int xe, int yb,
                                             int ye, int order, double xcfl, double ycfl) {
    return heat_dispatch<double, 1>(prev, curr, pitch, xb, xe, yb, ye, order, xcfl, ycfl);
}

// Reassociated oracle (heat_update_fast): bitwise reference for the GPU's
// "fast" stencil variants.
CME_CPU_EXPORT int cme_cpu_heat_step_fast_f32(const float* prev, float* curr, int pitch, int xb, int xe, int yb,
                                              int ye, int order, float xcfl, float ycfl) {
    return heat_dispatch<float, 2>(prev, curr, pitch, xb, xe, yb, ye, order, xcfl, ycfl);
}

CME_CPU_EXPORT int cme_cpu_heat_step_fast_f64(const double* prev, double* curr, int pitch, int xb, int xe, int yb,
                                              int ye, int order, double xcfl, double ycfl) {
    return heat_dispatch<double, 2>(prev, curr, pitch, xb, xe, yb, ye, order, xcfl, ycfl);
}
