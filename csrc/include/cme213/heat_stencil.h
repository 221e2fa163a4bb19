// FTCS heat-equation point update, orders 2/4/8, shared by the HIP kernels and
// the OpenMP CPU oracle so both evaluate the SAME expression tree.
//
// Coefficients and evaluation order follow the reference's stencil2/4/8
// (hw/hw2/solution/2dHeat_solution.cu:344-369, hw/hw5/2dHeat_solution.cpp
// stencil2/4/8): c + xcfl*(Dxx) + ycfl*(Dyy), left-to-right sums. FMA
// contraction is disabled here (and the CPU build uses -ffp-contract=off) so the
// GPU result is bitwise identical to the CPU oracle rather than merely within
// the reference's 10-ULP tolerance.
#pragma once

#include <cmath>

#if defined(__HIPCC__)
#define CME_HD __host__ __device__ __forceinline__
#else
#define CME_HD inline
#endif

namespace cme {

template <int ORDER> struct HeatOrder;
template <> struct HeatOrder<2> { static constexpr int B = 1; };
template <> struct HeatOrder<4> { static constexpr int B = 2; };
template <> struct HeatOrder<8> { static constexpr int B = 4; };

// m[k] = u(i-(k+1)), p[k] = u(i+(k+1)) along one axis.
template <int ORDER, typename T>
CME_HD T heat_d2(T c, const T* m, const T* p) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    if constexpr (ORDER == 2) {
        return p[0] + m[0] - 2 * c;
    } else if constexpr (ORDER == 4) {
        return -p[1] + 16 * p[0] - 30 * c + 16 * m[0] - m[1];
    } else {
        return -9 * p[3] + 128 * p[2] - 1008 * p[1] + 8064 * p[0] - 14350 * c + 8064 * m[0] - 1008 * m[1] +
               128 * m[2] - 9 * m[3];
    }
}

template <int ORDER, typename T>
CME_HD T heat_update(T c, const T* xm, const T* xp, const T* ym, const T* yp, T xcfl, T ycfl) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    T dx = heat_d2<ORDER>(c, xm, xp);
    T dy = heat_d2<ORDER>(c, ym, yp);
    return c + xcfl * dx + ycfl * dy;
}

// ---- FMA-contracted form ------------------------------------------------
// The same left-to-right sums with every multiply-add fused -- what nvcc
// generates for the reference's GPU kernels by default (-fmad=true), and why
// the reference checks GPU vs CPU within 10 ULP. Explicit fma() calls are
// correctly rounded on both sides, so the GPU result is bitwise equal to the
// CPU oracle's FMA mode. 20 flops-instructions per point at order 8 instead
// of 38.
template <typename T>
CME_HD T fmaT(T a, T b, T c) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (sizeof(T) == 4)
        return __builtin_fmaf(a, b, c);
    else
        return __builtin_fma(a, b, c);
#else
    return std::fma(a, b, c);
#endif
}

template <int ORDER, typename T>
CME_HD T heat_d2_fma(T c, const T* m, const T* p) {
    if constexpr (ORDER == 2) {
        return fmaT<T>(T(-2), c, p[0] + m[0]);
    } else if constexpr (ORDER == 4) {
        T t = -p[1];
        t = fmaT<T>(T(16), p[0], t);
        t = fmaT<T>(T(-30), c, t);
        t = fmaT<T>(T(16), m[0], t);
        return t - m[1];
    } else {
        T t = T(-9) * p[3];
        t = fmaT<T>(T(128), p[2], t);
        t = fmaT<T>(T(-1008), p[1], t);
        t = fmaT<T>(T(8064), p[0], t);
        t = fmaT<T>(T(-14350), c, t);
        t = fmaT<T>(T(8064), m[0], t);
        t = fmaT<T>(T(-1008), m[1], t);
        t = fmaT<T>(T(128), m[2], t);
        return fmaT<T>(T(-9), m[3], t);
    }
}

// heat_d2_fma over N points at once, term-major: every FMA of the chain is
// issued for all N points before the next, so the N independent chains
// interleave (a chain-major order leaves each packed FMA waiting on the one
// before it). Per point the same operations in the same order: bitwise equal
// to heat_d2_fma. m[k][j] / p[k][j] = u(x_j -/+ (k+1)).
template <int ORDER, int N, typename T>
CME_HD void heat_d2_fma_n(T* out, const T* c, const T (*m)[N], const T (*p)[N]) {
    if constexpr (ORDER == 2) {
        for (int j = 0; j < N; ++j) out[j] = fmaT<T>(T(-2), c[j], p[0][j] + m[0][j]);
    } else if constexpr (ORDER == 4) {
        for (int j = 0; j < N; ++j) out[j] = -p[1][j];
        for (int j = 0; j < N; ++j) out[j] = fmaT<T>(T(16), p[0][j], out[j]);
        for (int j = 0; j < N; ++j) out[j] = fmaT<T>(T(-30), c[j], out[j]);
        for (int j = 0; j < N; ++j) out[j] = fmaT<T>(T(16), m[0][j], out[j]);
        for (int j = 0; j < N; ++j) out[j] = out[j] - m[1][j];
    } else {
        const T w[4] = {T(8064), T(-1008), T(128), T(-9)};
        for (int j = 0; j < N; ++j) out[j] = T(-9) * p[3][j];
        for (int k = 2; k >= 0; --k)
            for (int j = 0; j < N; ++j) out[j] = fmaT<T>(w[k], p[k][j], out[j]);
        for (int j = 0; j < N; ++j) out[j] = fmaT<T>(T(-14350), c[j], out[j]);
        for (int k = 0; k < 4; ++k)
            for (int j = 0; j < N; ++j) out[j] = fmaT<T>(w[k], m[k][j], out[j]);
    }
}

template <int ORDER, typename T>
CME_HD T heat_update_fma(T c, const T* xm, const T* xp, const T* ym, const T* yp, T xcfl, T ycfl) {
    const T dx = heat_d2_fma<ORDER>(c, xm, xp);
    const T dy = heat_d2_fma<ORDER>(c, ym, yp);
    return fmaT<T>(ycfl, dy, fmaT<T>(xcfl, dx, c));
}

// ---- reassociated ("fast") form --------------------------------------------
// The same FTCS stencil with the CFL numbers folded into the weights once per
// launch and each symmetric pair summed first:
//   u' = c0*c + sum_k ax_k (xp_k + xm_k) + sum_k ay_k (yp_k + ym_k),
//   c0 = 1 + w_c (xcfl + ycfl), ax_k = w_k xcfl, ay_k = w_k ycfl,
// 1 multiply + 4B adds + 4B FMAs per point (17 at order 8 instead of 20). A
// different rounding order from the reference's expression tree (within its
// 10-ULP criterion of the other modes); bitwise equal between the GPU kernels
// and the CPU oracle, which share this code.
template <int ORDER, typename T>
struct HeatFast {
    static constexpr int B = HeatOrder<ORDER>::B;
    T c0;
    T ax[B], ay[B];
};

// The rounded fp32 weights no longer sum to one: c0 + 2 sum(ax + ay) = 1 + e
// with |e| ~ 1e-8, so every step scales a smooth field by (1 + e) and the
// reassociated form drifted 16-40 ULP from the exact stencil over whole runs
// (profiles/heat_arith_ulp_r5.md). Here c0 is recomputed from the rounded
// pair weights, and the remaining residual -- exact in double: the nine fp32
// terms span < 40 bits -- is folded into the smallest pair weights until the
// weights sum to exactly one (a constant field is then a fixed point, as in
// the exact and FMA forms). Measured drift from exact: 2048^2 x 200 random
// 39 -> 7 ULP, 4000^2 x 10 random 15 -> 9. Host and device evaluate the same
// IEEE double sequence, so the GPU kernels and the CPU oracle stay bitwise
// equal.
template <int ORDER, typename T>
CME_HD void heat_fast_make_consistent(HeatFast<ORDER, T>& f) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    constexpr int B = HeatOrder<ORDER>::B;
    double s = 0.0;
    for (int k = 0; k < B; ++k) s += 2.0 * (double)f.ax[k] + 2.0 * (double)f.ay[k];
    f.c0 = (T)(1.0 - s);
    for (int it = 0; it < 4 * B; ++it) {
        double tot = (double)f.c0;
        for (int k = 0; k < B; ++k) tot += 2.0 * (double)f.ax[k] + 2.0 * (double)f.ay[k];
        const double r = 1.0 - tot;
        if (r == 0.0) break;
        const int k = B - 1 - (it / 2) % B;  // the smallest weights first, y then x
        T& wk = (it % 2 == 0) ? f.ay[k] : f.ax[k];
        wk = (T)((double)wk + 0.5 * r);
    }
}

template <int ORDER, typename T>
CME_HD HeatFast<ORDER, T> heat_fast_coefs(T xcfl, T ycfl) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    HeatFast<ORDER, T> f;
    if constexpr (ORDER == 2) {
        f.c0 = T(1) + T(-2) * (xcfl + ycfl);
        f.ax[0] = xcfl;
        f.ay[0] = ycfl;
    } else if constexpr (ORDER == 4) {
        f.c0 = T(1) + T(-30) * (xcfl + ycfl);
        f.ax[0] = T(16) * xcfl, f.ax[1] = T(-1) * xcfl;
        f.ay[0] = T(16) * ycfl, f.ay[1] = T(-1) * ycfl;
    } else {
        const T w[4] = {T(8064), T(-1008), T(128), T(-9)};
        f.c0 = T(1) + T(-14350) * (xcfl + ycfl);
        for (int k = 0; k < 4; ++k) {
            f.ax[k] = w[k] * xcfl;
            f.ay[k] = w[k] * ycfl;
        }
    }
    if constexpr (sizeof(T) == 4) heat_fast_make_consistent<ORDER>(f);
    return f;
}

template <int ORDER, typename T>
CME_HD T heat_update_fast(T c, const T* xm, const T* xp, const T* ym, const T* yp, const HeatFast<ORDER, T>& f) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    constexpr int B = HeatOrder<ORDER>::B;
    T u = f.c0 * c;
    for (int k = B - 1; k >= 0; --k) u = fmaT<T>(f.ax[k], xp[k] + xm[k], u);
    for (int k = B - 1; k >= 0; --k) u = fmaT<T>(f.ay[k], yp[k] + ym[k], u);
    return u;
}

template <int ORDER, bool FMA, typename T>
CME_HD T heat_update_sel(T c, const T* xm, const T* xp, const T* ym, const T* yp, T xcfl, T ycfl) {
    if constexpr (FMA)
        return heat_update_fma<ORDER>(c, xm, xp, ym, yp, xcfl, ycfl);
    else
        return heat_update<ORDER>(c, xm, xp, ym, yp, xcfl, ycfl);
}

}  // namespace cme
