// Tuning arms of the 2-D heat streaming kernels (libcme213_tune.so only,
// `make TUNE=1`): rows per block, waves per block / per EU, prefetch depth,
// non-temporal stores. Production dispatch is in csrc/hip/heat2d.hip.
#include "../hip/heat2d_kernels.h"

// Tuning entry point for the streaming kernel (order 8, fp32): explores rows
// per register block (rb 4/8/12), waves per block (4/8/16) and non-temporal
// stores. Used by benchmarks/tune_heat.py; the production path is variant 2.
namespace {
template <int RB, int WPB, bool NT>
int tune_launch(const float* prev, float* curr, int pitch, int gy, Region g, float xcfl, float ycfl, int chunk,
                hipStream_t s) {
    const int H = g.ye - g.yb;
    const int x_lo = g.xb & ~3;
    const int strips = (int)cdiv(g.xe - x_lo, kStripOut);
    if (chunk <= 0) {
        long rows = ((long)strips * H + 4095) / 4096;
        chunk = (int)(rows < RB ? RB : (rows > 512 ? 512 : rows));
    }
    chunk = ((chunk + RB - 1) / RB) * RB;
    const int total_waves = strips * (int)cdiv(H, chunk);
    hipLaunchKernelGGL((heat_stream_kernel<float, 8, RB, WPB, NT>), dim3(cdiv(total_waves, WPB)), dim3(WPB * 64), 0,
                       s, prev, curr, pitch, gy, g.xb, g.xe, g.yb, g.ye, strips, chunk, total_waves, xcfl, ycfl);
    CME_LAUNCH_STATUS();
}
template <int RB, int WPB>
int tune_nt(int nt, const float* prev, float* curr, int pitch, int gy, Region g, float xcfl, float ycfl, int chunk,
            hipStream_t s) {
    return nt ? tune_launch<RB, WPB, true>(prev, curr, pitch, gy, g, xcfl, ycfl, chunk, s)
              : tune_launch<RB, WPB, false>(prev, curr, pitch, gy, g, xcfl, ycfl, chunk, s);
}
template <int RB>
int tune_wpb(int wpb, int nt, const float* prev, float* curr, int pitch, int gy, Region g, float xcfl, float ycfl,
             int chunk, hipStream_t s) {
    switch (wpb) {
        case 4: return tune_nt<RB, 4>(nt, prev, curr, pitch, gy, g, xcfl, ycfl, chunk, s);
        case 8: return tune_nt<RB, 8>(nt, prev, curr, pitch, gy, g, xcfl, ycfl, chunk, s);
        case 16: return tune_nt<RB, 16>(nt, prev, curr, pitch, gy, g, xcfl, ycfl, chunk, s);
        default: return (int)hipErrorInvalidValue;
    }
}
}  // namespace

CME_EXPORT int cme_heat_stream_tune_f32(const float* prev, float* curr, int pitch, int gy, int xb, int xe, int yb,
                                        int ye, float xcfl, float ycfl, int rb, int wpb, int nt, int chunk,
                                        void* stream) {
    Region g{xb, xe, yb, ye};
    hipStream_t s = as_stream(stream);
    switch (rb) {
        case 4: return tune_wpb<4>(wpb, nt, prev, curr, pitch, gy, g, xcfl, ycfl, chunk, s);
        case 8: return tune_wpb<8>(wpb, nt, prev, curr, pitch, gy, g, xcfl, ycfl, chunk, s);
        case 12: return tune_wpb<12>(wpb, nt, prev, curr, pitch, gy, g, xcfl, ycfl, chunk, s);
        default: return (int)hipErrorInvalidValue;
    }
}

// Tuning entry for the two-step kernel (order 8): rows per block rb 2/4/8 and
// a waves-per-EU register cap wpe 1 (none)/2/3/4, exact or FMA, f32 or f64.
// Used by benchmarks/tune_heat.py --stream2; production uses the defaults.
namespace {
template <typename T, bool FMA, int RB>
int tune2_wpe(const T* prev, T* curr, int pitch, int gy, Region g, T xcfl, T ycfl, int chunk, int wpe, hipStream_t s) {
    switch (wpe) {
        case 1: return launch_stream2<T, 8, FMA, RB, 1>(prev, curr, pitch, gy, g, g, xcfl, ycfl, chunk, s);
        case 2: return launch_stream2<T, 8, FMA, RB, 2>(prev, curr, pitch, gy, g, g, xcfl, ycfl, chunk, s);
        case 3: return launch_stream2<T, 8, FMA, RB, 3>(prev, curr, pitch, gy, g, g, xcfl, ycfl, chunk, s);
        case 4: return launch_stream2<T, 8, FMA, RB, 4>(prev, curr, pitch, gy, g, g, xcfl, ycfl, chunk, s);
        default: return (int)hipErrorInvalidValue;
    }
}
template <typename T, bool FMA>
int tune2_rb(const T* prev, T* curr, int pitch, int gy, Region g, T xcfl, T ycfl, int chunk, int rb, int wpe,
             hipStream_t s) {
    switch (rb) {
        case 2: return tune2_wpe<T, FMA, 2>(prev, curr, pitch, gy, g, xcfl, ycfl, chunk, wpe, s);
        case 4: return tune2_wpe<T, FMA, 4>(prev, curr, pitch, gy, g, xcfl, ycfl, chunk, wpe, s);
        case 8: return tune2_wpe<T, FMA, 8>(prev, curr, pitch, gy, g, xcfl, ycfl, chunk, wpe, s);
        default: return (int)hipErrorInvalidValue;
    }
}
}  // namespace

CME_EXPORT int cme_heat_stream2_tune(const void* prev, void* curr, int dtype, int pitch, int gy, int xb, int xe,
                                     int yb, int ye, double xcfl, double ycfl, int chunk, int rb, int wpe, int fma,
                                     void* stream) {
    hipStream_t s = as_stream(stream);
    const Region g{xb, xe, yb, ye};
    if (dtype == 0) {
        const float* p = (const float*)prev;
        float* c = (float*)curr;
        return fma ? tune2_rb<float, true>(p, c, pitch, gy, g, (float)xcfl, (float)ycfl, chunk, rb, wpe, s)
                   : tune2_rb<float, false>(p, c, pitch, gy, g, (float)xcfl, (float)ycfl, chunk, rb, wpe, s);
    }
    const double* p = (const double*)prev;
    double* c = (double*)curr;
    return fma ? tune2_rb<double, true>(p, c, pitch, gy, g, xcfl, ycfl, chunk, rb, wpe, s)
               : tune2_rb<double, false>(p, c, pitch, gy, g, xcfl, ycfl, chunk, rb, wpe, s);
}

// Tuning entry for the NS-step kernels (order 8, fp32, FMA): ns 3/4, rows per
// block rb 1/2/4, prefetch depth pd 1/2 (phases of input rows in flight; 13 =
// depth 1 under a 3-waves/SIMD register cap), explicit chunk (0 = default).
namespace {
template <int NS, int RB>
int tunen_pd(const float* p, float* c, int pitch, int gy, Region g, float xcfl, float ycfl, int chunk, int pd,
             hipStream_t s) {
    switch (pd) {
        case 1: return launch_streamn_multi<float, 8, NS, true, RB, 1, 1>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl, chunk, s);
        case 2: return launch_streamn_multi<float, 8, NS, true, RB, 1, 2>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl, chunk, s);
        // pd 13: prefetch depth 1 with a 3-waves-per-SIMD register cap (<= 168 VGPRs)
        case 13: return launch_streamn_multi<float, 8, NS, true, RB, 3, 1>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl, chunk, s);
        // pd 21: depth 1, non-temporal output stores
        case 21: return launch_streamn_multi<float, 8, NS, true, RB, 1, 1, true>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                                chunk, s);
        default: return (int)hipErrorInvalidValue;
    }
}
template <int NS>
int tunen_rb(const float* p, float* c, int pitch, int gy, Region g, float xcfl, float ycfl, int chunk, int rb,
             int pd, hipStream_t s) {
    switch (rb) {
        case 1: return tunen_pd<NS, 1>(p, c, pitch, gy, g, xcfl, ycfl, chunk, pd, s);
        case 2: return tunen_pd<NS, 2>(p, c, pitch, gy, g, xcfl, ycfl, chunk, pd, s);
        case 4: return tunen_pd<NS, 4>(p, c, pitch, gy, g, xcfl, ycfl, chunk, pd, s);
        default: return (int)hipErrorInvalidValue;
    }
}
}  // namespace

CME_EXPORT int cme_heat_streamn_tune(const float* prev, float* curr, int pitch, int gy, int xb, int xe, int yb,
                                     int ye, float xcfl, float ycfl, int chunk, int rb, int ns, int pd,
                                     void* stream) {
    hipStream_t s = as_stream(stream);
    const Region g{xb, xe, yb, ye};
    if (ns == 3) return tunen_rb<3>(prev, curr, pitch, gy, g, xcfl, ycfl, chunk, rb, pd, s);
    if (ns == 4) return tunen_rb<4>(prev, curr, pitch, gy, g, xcfl, ycfl, chunk, rb, pd, s);
    return (int)hipErrorInvalidValue;
}

