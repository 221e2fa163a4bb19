// Floating-point summation accuracy study (slides/Lecture11 "Reductions and
// Floating Point": serial O(n eps) vs pairwise O(log n eps) error growth),
// in fp32 on the host: serial left-to-right, pairwise (recursive halving,
// serial below 8 elements), and Kahan compensated summation.
// Built with -ffp-contract=off so no FMA changes the rounding being studied.
#include <cstddef>

#include "cme213/cpu_common.h"

namespace {

float pairwise(const float* x, long long n) {
    if (n <= 8) {
        float s = 0.f;
        for (long long i = 0; i < n; ++i) s += x[i];
        return s;
    }
    const long long h = n / 2;
    return pairwise(x, h) + pairwise(x + h, n - h);
}

}  // namespace

// algo: 0 serial, 1 pairwise, 2 Kahan. Result in *out (fp32 rounding).
CME_CPU_EXPORT int cme_cpu_sum_f32(const float* x, long long n, int algo, float* out) {
    if (algo == 0) {
        float s = 0.f;
        for (long long i = 0; i < n; ++i) s += x[i];
        *out = s;
    } else if (algo == 1) {
        *out = pairwise(x, n);
    } else if (algo == 2) {
        float s = 0.f, c = 0.f;
        for (long long i = 0; i < n; ++i) {
            const volatile float y = x[i] - c;  // volatile: keep the compensation
            const volatile float t = s + y;
            c = (t - s) - y;
            s = t;
        }
        *out = s;
    } else {
        return 1;
    }
    return 0;
}
