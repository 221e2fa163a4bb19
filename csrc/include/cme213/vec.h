// 4-wide element vectors used by the streaming kernels: one lane moves 16 B
// (fp32) or 32 B (fp64) per access, the width the CDNA memory pipe wants
// (cdna_hip_programming.md Guideline 13).
#pragma once
#include "common.h"
#include "wave.h"

namespace cme {

template <typename T>
struct alignas(16) V4 {
    T v[4];
    __device__ __forceinline__ T& operator[](int i) { return v[i]; }
    __device__ __forceinline__ const T& operator[](int i) const { return v[i]; }
};

template <typename T>
__device__ __forceinline__ V4<T> load4(const T* p) {
    if constexpr (sizeof(T) == 4) {
        float4 f = *reinterpret_cast<const float4*>(p);
        V4<T> r;
        r.v[0] = __builtin_bit_cast(T, f.x);
        r.v[1] = __builtin_bit_cast(T, f.y);
        r.v[2] = __builtin_bit_cast(T, f.z);
        r.v[3] = __builtin_bit_cast(T, f.w);
        return r;
    } else {
        double2 a = reinterpret_cast<const double2*>(p)[0];
        double2 b = reinterpret_cast<const double2*>(p)[1];
        V4<T> r;
        r.v[0] = __builtin_bit_cast(T, a.x);
        r.v[1] = __builtin_bit_cast(T, a.y);
        r.v[2] = __builtin_bit_cast(T, b.x);
        r.v[3] = __builtin_bit_cast(T, b.y);
        return r;
    }
}

template <typename T>
__device__ __forceinline__ void store4(T* p, const V4<T>& r) {
    if constexpr (sizeof(T) == 4) {
        float4 f;
        f.x = __builtin_bit_cast(float, r.v[0]);
        f.y = __builtin_bit_cast(float, r.v[1]);
        f.z = __builtin_bit_cast(float, r.v[2]);
        f.w = __builtin_bit_cast(float, r.v[3]);
        *reinterpret_cast<float4*>(p) = f;
    } else {
        double2 a, b;
        a.x = __builtin_bit_cast(double, r.v[0]);
        a.y = __builtin_bit_cast(double, r.v[1]);
        b.x = __builtin_bit_cast(double, r.v[2]);
        b.y = __builtin_bit_cast(double, r.v[3]);
        reinterpret_cast<double2*>(p)[0] = a;
        reinterpret_cast<double2*>(p)[1] = b;
    }
}

// N (a multiple of 4) consecutive elements per lane, moved as N/4 16-B (fp32)
// pieces: the wide-lane pipelined heat pass keeps 8 columns per lane.
template <typename T, int N>
struct alignas(16) VecN {
    static_assert(N % 4 == 0, "VecN: multiple of 4 elements");
    T v[N];
    __device__ __forceinline__ T& operator[](int i) { return v[i]; }
    __device__ __forceinline__ const T& operator[](int i) const { return v[i]; }
};

template <int N, typename T>
__device__ __forceinline__ VecN<T, N> load_n(const T* p) {
    VecN<T, N> r;
#pragma unroll
    for (int h = 0; h < N / 4; ++h) {
        const V4<T> q = load4(p + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) r.v[4 * h + j] = q.v[j];
    }
    return r;
}

template <int N, typename T>
__device__ __forceinline__ V4<T> piece4(const VecN<T, N>& x, int h) {
    V4<T> q;
#pragma unroll
    for (int j = 0; j < 4; ++j) q.v[j] = x.v[4 * h + j];
    return q;
}

// Whole-vector lane shifts: lane i receives lane i-1 (shr) / i+1 (shl); the
// edge lane (0 for shr, 63 for shl) receives 0.
template <typename T>
__device__ __forceinline__ V4<T> wave_shr1(const V4<T>& x) {
    V4<T> r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r.v[j] = dpp_shift<kDppWaveShr1>(x.v[j]);
    return r;
}
template <typename T>
__device__ __forceinline__ V4<T> wave_shl1(const V4<T>& x) {
    V4<T> r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r.v[j] = dpp_shift<kDppWaveShl1>(x.v[j]);
    return r;
}

}  // namespace cme
