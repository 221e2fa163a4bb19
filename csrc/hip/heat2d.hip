// 2-D heat diffusion: C entry points (kernels and launchers in
// heat2d_kernels.h). Reference: hw/hw2/solution/2dHeat_solution.cu:413-669,
// hw/hw5/2dHeat_solution.cpp:501-628.
#include "heat2d_kernels.h"

// heat_pipe.hip: the wave-pipelined NS-step pass (variants 11-14)
extern "C" int cme_heat_pipe_f64(const double* prev, double* curr, int pitch, int gy, const int* out, int nout,
                                 const int* ext, int order, int nsteps, double xcfl, double ycfl, int chunk, int fma,
                                 void* stream);
extern "C" int cme_heat_pipe_f32(const float* prev, float* curr, int pitch, int gy, const int* out, int nout,
                                 const int* ext, int order, int nsteps, float xcfl, float ycfl, int chunk, int fma,
                                 void* stream);

namespace {

template <typename T, int ORDER>
int launch_heat(int variant, const T* prev, T* curr, int pitch, int gy, Region g, T xcfl, T ycfl, int chunk_hint,
                hipStream_t s) {
    const int W = g.xe - g.xb, H = g.ye - g.yb;
    if (W <= 0 || H <= 0) return 0;
    if ((pitch & 63) != 0) return (int)hipErrorInvalidValue;
    if (variant == 0) {
        dim3 grid(cdiv(W, 64), cdiv(H, 4));
        hipLaunchKernelGGL((heat_naive_kernel<T, ORDER>), grid, dim3(256), 0, s, prev, curr, pitch, g.xb, g.xe, g.yb,
                           g.ye, xcfl, ycfl);
    } else if (variant == 1) {
        constexpr int TY = 32;
        dim3 grid(cdiv(W, 64), cdiv(H, TY));
        hipLaunchKernelGGL((heat_lds_kernel<T, ORDER, TY, 1>), grid, dim3(256), 0, s, prev, curr, pitch, gy, g.xb,
                           g.xe, g.yb, g.ye, xcfl, ycfl);
    } else if (variant == 4 || variant == 5) {
        // TWO timesteps per launch (temporal blocking), step-1 region = output
        return variant == 4 ? launch_stream2<T, ORDER, false>(prev, curr, pitch, gy, g, g, xcfl, ycfl, chunk_hint, s)
                            : launch_stream2<T, ORDER, true>(prev, curr, pitch, gy, g, g, xcfl, ycfl, chunk_hint, s);
    } else if (variant >= 7 && variant <= 10) {
        // NS = 3 (variants 7, 8) or 4 (9, 10) timesteps per launch; fp64:
        // NS = 3 only, one row per register block
        if constexpr (sizeof(T) == 8) {
            if (variant == 7)
                return launch_streamn_multi<T, ORDER, 3, false, 1>(prev, curr, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                   chunk_hint, s);
            if (variant == 8)
                return launch_streamn_multi<T, ORDER, 3, true, 1>(prev, curr, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                  chunk_hint, s);
        }
        if constexpr (sizeof(T) == 4) {
            switch (variant) {
                case 7: return launch_streamn_multi<T, ORDER, 3, false>(prev, curr, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                        chunk_hint, s);
                case 8: return launch_streamn_multi<T, ORDER, 3, true>(prev, curr, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                       chunk_hint, s);
                case 9: return launch_streamn_multi<T, ORDER, 4, false>(prev, curr, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                        chunk_hint, s);
                default: return launch_streamn_multi<T, ORDER, 4, true>(prev, curr, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                        chunk_hint, s);
            }
        } else {
            return (int)hipErrorInvalidValue;
        }
    } else if (variant >= 11 && variant <= 18) {
        // wave-pipelined NS = 3 (11 exact, 12 FMA) / 4 (13, 14) / 5 (15, 16) /
        // 6 (17, 18, fp32) steps per pass
        const int r[4] = {g.xb, g.xe, g.yb, g.ye};
        const int ns = (variant - 11) / 2 + 3;
        if constexpr (sizeof(T) == 4)
            return cme_heat_pipe_f32(prev, curr, pitch, gy, r, 1, r, ORDER, ns, xcfl, ycfl, chunk_hint,
                                     (variant & 1) ? 0 : 1, s);
        else
            return ns > 4 ? (int)hipErrorInvalidValue
                          : cme_heat_pipe_f64(prev, curr, pitch, gy, r, 1, r, ORDER, ns, xcfl, ycfl, chunk_hint,
                                              (variant & 1) ? 0 : 1, s);
    } else if (variant == 3) {
        // LDS tile without the +1 pad (bank-conflict study arm).
        constexpr int TY = 32;
        dim3 grid(cdiv(W, 64), cdiv(H, TY));
        hipLaunchKernelGGL((heat_lds_kernel<T, ORDER, TY, 0>), grid, dim3(256), 0, s, prev, curr, pitch, gy, g.xb,
                           g.xe, g.yb, g.ye, xcfl, ycfl);
    } else {
        constexpr int RB = sizeof(T) == 4 ? 8 : 4;
        const int x_lo = g.xb & ~3;
        const int strips = (int)cdiv(g.xe - x_lo, kStripOut);
        // Enough waves to fill 256 CUs x 16 waves, chunk a multiple of RB.
        int chunk = chunk_hint;
        if (chunk <= 0) {
            const long target_waves = 256L * 16;
            long rows = ((long)strips * H + target_waves - 1) / target_waves;
            rows = rows < RB ? RB : rows;
            rows = rows > 512 ? 512 : rows;
            chunk = (int)rows;
        }
        chunk = ((chunk + RB - 1) / RB) * RB;
        const int chunks = (int)cdiv(H, chunk);
        const int total_waves = strips * chunks;
        if (variant == 6)
            hipLaunchKernelGGL((heat_stream_kernel<T, ORDER, RB, 4, false, true>), dim3(cdiv(total_waves, 4)),
                               dim3(256), 0, s, prev, curr, pitch, gy, g.xb, g.xe, g.yb, g.ye, strips, chunk,
                               total_waves, xcfl, ycfl);
        else
            hipLaunchKernelGGL((heat_stream_kernel<T, ORDER, RB>), dim3(cdiv(total_waves, 4)), dim3(256), 0, s, prev,
                               curr, pitch, gy, g.xb, g.xe, g.yb, g.ye, strips, chunk, total_waves, xcfl, ycfl);
    }
    CME_LAUNCH_STATUS();
}

template <typename T>
int dispatch_heat(int order, int variant, const T* prev, T* curr, int pitch, int gy, Region g, T xcfl, T ycfl,
                  int chunk, hipStream_t s) {
    switch (order) {
        case 2: return launch_heat<T, 2>(variant, prev, curr, pitch, gy, g, xcfl, ycfl, chunk, s);
        case 4: return launch_heat<T, 4>(variant, prev, curr, pitch, gy, g, xcfl, ycfl, chunk, s);
        case 8: return launch_heat<T, 8>(variant, prev, curr, pitch, gy, g, xcfl, ycfl, chunk, s);
        default: return (int)hipErrorInvalidValue;
    }
}

template <typename T, bool FMA>
int dispatch_stream2_t(int order, const T* prev, T* curr, int pitch, int gy, const Region* gs, int n, Region g1,
                       T xcfl, T ycfl, int chunk, hipStream_t s) {
    switch (order) {
        case 2: return launch_stream2_multi<T, 2, FMA>(prev, curr, pitch, gy, gs, n, g1, xcfl, ycfl, chunk, s);
        case 4: return launch_stream2_multi<T, 4, FMA>(prev, curr, pitch, gy, gs, n, g1, xcfl, ycfl, chunk, s);
        case 8: return launch_stream2_multi<T, 8, FMA>(prev, curr, pitch, gy, gs, n, g1, xcfl, ycfl, chunk, s);
        default: return (int)hipErrorInvalidValue;
    }
}

template <typename T>
int dispatch_stream2(int order, const T* prev, T* curr, int pitch, int gy, const Region* gs, int n, Region g1,
                     T xcfl, T ycfl, int chunk, int fma, hipStream_t s) {
    return fma ? dispatch_stream2_t<T, true>(order, prev, curr, pitch, gy, gs, n, g1, xcfl, ycfl, chunk, s)
               : dispatch_stream2_t<T, false>(order, prev, curr, pitch, gy, gs, n, g1, xcfl, ycfl, chunk, s);
}

}  // namespace

// TWO timesteps in one pass: curr[out] = FTCS^2(prev) where the intermediate
// step is applied on region `ext` (out grown by <= B cells into a halo).
// fma: 0 exact (contraction off), 1 FMA-contracted stencil. `out` holds
// nout (<= 4) regions {xb, xe, yb, ye}, done in ONE launch.
CME_EXPORT int cme_heat_step2_f32(const float* prev, float* curr, int pitch, int gy, const int* out, int nout,
                                  const int* ext, int order, float xcfl, float ycfl, int chunk, int fma,
                                  void* stream) {
    Region gs[kMaxS2Regions];
    if (nout < 1 || nout > kMaxS2Regions) return (int)hipErrorInvalidValue;
    for (int i = 0; i < nout; ++i) gs[i] = Region{out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]};
    return dispatch_stream2<float>(order, prev, curr, pitch, gy, gs, nout, Region{ext[0], ext[1], ext[2], ext[3]},
                                   xcfl, ycfl, chunk, fma, as_stream(stream));
}

CME_EXPORT int cme_heat_step2_f64(const double* prev, double* curr, int pitch, int gy, const int* out, int nout,
                                  const int* ext, int order, double xcfl, double ycfl, int chunk, int fma,
                                  void* stream) {
    Region gs[kMaxS2Regions];
    if (nout < 1 || nout > kMaxS2Regions) return (int)hipErrorInvalidValue;
    for (int i = 0; i < nout; ++i) gs[i] = Region{out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]};
    return dispatch_stream2<double>(order, prev, curr, pitch, gy, gs, nout, Region{ext[0], ext[1], ext[2], ext[3]},
                                    xcfl, ycfl, chunk, fma, as_stream(stream));
}

// NS timesteps in one pass (NS = 2, 3, 4; 3 and 4 fp32 only): intermediate
// steps over `ext` (out grown by <= (NS-1)B cells into an NS*B-deep halo),
// the last one writes `out` (nout <= 4 regions, one launch).
namespace {
template <int ORDER, bool FMA>
int stepn_f32(const float* prev, float* curr, int pitch, int gy, const Region* gs, int n, Region e, int ns,
              float xcfl, float ycfl, int chunk, hipStream_t s) {
    switch (ns) {
        case 2: return launch_stream2_multi<float, ORDER, FMA>(prev, curr, pitch, gy, gs, n, e, xcfl, ycfl, chunk, s);
        case 3: return launch_streamn_multi<float, ORDER, 3, FMA>(prev, curr, pitch, gy, gs, n, e, xcfl, ycfl, chunk,
                                                                  s);
        case 4: return launch_streamn_multi<float, ORDER, 4, FMA>(prev, curr, pitch, gy, gs, n, e, xcfl, ycfl, chunk,
                                                                  s);
        default: return (int)hipErrorInvalidValue;
    }
}
template <bool FMA>
int stepn_f32_o(int order, const float* prev, float* curr, int pitch, int gy, const Region* gs, int n, Region e,
                int ns, float xcfl, float ycfl, int chunk, hipStream_t s) {
    switch (order) {
        case 2: return stepn_f32<2, FMA>(prev, curr, pitch, gy, gs, n, e, ns, xcfl, ycfl, chunk, s);
        case 4: return stepn_f32<4, FMA>(prev, curr, pitch, gy, gs, n, e, ns, xcfl, ycfl, chunk, s);
        case 8: return stepn_f32<8, FMA>(prev, curr, pitch, gy, gs, n, e, ns, xcfl, ycfl, chunk, s);
        default: return (int)hipErrorInvalidValue;
    }
}
}  // namespace

CME_EXPORT int cme_heat_stepn_f32(const float* prev, float* curr, int pitch, int gy, const int* out, int nout,
                                  const int* ext, int order, int nsteps, float xcfl, float ycfl, int chunk, int fma,
                                  void* stream) {
    Region gs[kMaxS2Regions];
    if (nout < 1 || nout > kMaxS2Regions) return (int)hipErrorInvalidValue;
    for (int i = 0; i < nout; ++i) gs[i] = Region{out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]};
    const Region e{ext[0], ext[1], ext[2], ext[3]};
    return fma ? stepn_f32_o<true>(order, prev, curr, pitch, gy, gs, nout, e, nsteps, xcfl, ycfl, chunk,
                                   as_stream(stream))
               : stepn_f32_o<false>(order, prev, curr, pitch, gy, gs, nout, e, nsteps, xcfl, ycfl, chunk,
                                    as_stream(stream));
}

namespace {
// fp64 NS = 3: the streamN design with one row per register block (RB = 1):
// three 9-row windows of 4 doubles per lane stay within two waves per SIMD.
template <int ORDER, bool FMA>
int stepn3_f64(const double* prev, double* curr, int pitch, int gy, const Region* gs, int n, Region e, double xcfl,
               double ycfl, int chunk, hipStream_t s) {
    return launch_streamn_multi<double, ORDER, 3, FMA, 1>(prev, curr, pitch, gy, gs, n, e, xcfl, ycfl, chunk, s);
}
template <bool FMA>
int stepn3_f64_o(int order, const double* prev, double* curr, int pitch, int gy, const Region* gs, int n, Region e,
                 double xcfl, double ycfl, int chunk, hipStream_t s) {
    switch (order) {
        case 2: return stepn3_f64<2, FMA>(prev, curr, pitch, gy, gs, n, e, xcfl, ycfl, chunk, s);
        case 4: return stepn3_f64<4, FMA>(prev, curr, pitch, gy, gs, n, e, xcfl, ycfl, chunk, s);
        case 8: return stepn3_f64<8, FMA>(prev, curr, pitch, gy, gs, n, e, xcfl, ycfl, chunk, s);
        default: return (int)hipErrorInvalidValue;
    }
}
}  // namespace

CME_EXPORT int cme_heat_stepn_f64(const double* prev, double* curr, int pitch, int gy, const int* out, int nout,
                                  const int* ext, int order, int nsteps, double xcfl, double ycfl, int chunk, int fma,
                                  void* stream) {
    if (nsteps == 2)
        return cme_heat_step2_f64(prev, curr, pitch, gy, out, nout, ext, order, xcfl, ycfl, chunk, fma, stream);
    if (nsteps != 3) return (int)hipErrorInvalidValue;  // 4-step passes: fp32 only
    Region gs[kMaxS2Regions];
    if (nout < 1 || nout > kMaxS2Regions) return (int)hipErrorInvalidValue;
    for (int i = 0; i < nout; ++i) gs[i] = Region{out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]};
    const Region e{ext[0], ext[1], ext[2], ext[3]};
    return fma ? stepn3_f64_o<true>(order, prev, curr, pitch, gy, gs, nout, e, xcfl, ycfl, chunk, as_stream(stream))
               : stepn3_f64_o<false>(order, prev, curr, pitch, gy, gs, nout, e, xcfl, ycfl, chunk, as_stream(stream));
}

// variant: 0 naive, 1 lds(+1 pad), 2 stream, 3 lds(no pad), 4 stream2 (TWO
// steps), 5 stream2 FMA (TWO steps), 6 stream FMA, 7 / 8 stream3 exact / FMA
// (THREE steps, fp32), 9 / 10 stream4 exact / FMA (FOUR steps, fp32),
// 11 / 12 pipe3 exact / FMA, 13 / 14 pipe4 exact / FMA (wave-pipelined, fp32
// and fp64), 15 / 16 pipe5, 17 / 18 pipe6 (fp32: HBM-bound low orders)
CME_EXPORT int cme_heat_step_f32(const float* prev, float* curr, int pitch, int gy, int xb, int xe, int yb, int ye,
                                 int order, int variant, float xcfl, float ycfl, int chunk, void* stream) {
    return dispatch_heat<float>(order, variant, prev, curr, pitch, gy, Region{xb, xe, yb, ye}, xcfl, ycfl, chunk,
                                as_stream(stream));
}

CME_EXPORT int cme_heat_step_f64(const double* prev, double* curr, int pitch, int gy, int xb, int xe, int yb, int ye,
                                 int order, int variant, double xcfl, double ycfl, int chunk, void* stream) {
    return dispatch_heat<double>(order, variant, prev, curr, pitch, gy, Region{xb, xe, yb, ye}, xcfl, ycfl, chunk,
                                 as_stream(stream));
}

extern "C" int cme_heat_tile_f32(const float* prev, float* curr, int pitch, int gy, int xb, int xe, int yb, int ye,
                                 int order, int nsteps, float xcfl, float ycfl, int fma, void* stream);
extern "C" int cme_heat_tile_f64(const double* prev, double* curr, int pitch, int gy, int xb, int xe, int yb,
                                 int ye, int order, int nsteps, double xcfl, double ycfl, int fma, void* stream);
namespace {
int tile_pass_t(const float* p, float* c, int pitch, int gy, Region g, int order, int ns, int fma, float xc,
                float yc, hipStream_t s) {
    return cme_heat_tile_f32(p, c, pitch, gy, g.xb, g.xe, g.yb, g.ye, order, ns, xc, yc, fma, (void*)s);
}
int tile_pass_t(const double* p, double* c, int pitch, int gy, Region g, int order, int ns, int fma, double xc,
                double yc, hipStream_t s) {
    return cme_heat_tile_f64(p, c, pitch, gy, g.xb, g.xe, g.yb, g.ye, order, ns, xc, yc, fma, (void*)s);
}
}  // namespace

// Multi-step driver: `iters` sweeps of the full region in one call (buffers
// a/b, first sweep reads a). Avoids per-iteration host round trips (the
// reference synchronises after every launch: 2dHeat_solution.cu:549).
// variants 4/5 advance TWO steps per launch (+ one single step, variant 2/6,
// for odd iters). Variants 19..26: tileN exact / FMA, N = 1..4 steps per
// pass of the LDS-resident tile kernel (heat_tile.hip, small grids), the
// remainder as one shorter tile pass. (The persistent schedules measured
// slower than these per-pass launches -- the cross-pass dataflow launch and
// the LDS-resident tiles, profiles/heat_flow_r5.md, heat_tile_res_r5.md --
// and live in the tuning library, csrc/hip_tune/.)
// *final_idx = 0 if the result is in a, 1 if in b.
template <typename T>
int heat_run_impl(T* a, T* b, int pitch, int gy, Region g, int order, int variant, T xcfl, T ycfl, int iters,
                  int chunk, int* final_idx, hipStream_t s) {
    int cur = 0;
    T* bufs[2] = {a, b};
    int i = 0;
    if (variant >= 19 && variant <= 26) {
        const int ns = (variant - 19) / 2 + 1, fma = (variant - 19) & 1;
        while (i < iters) {
            const int k = iters - i < ns ? iters - i : ns;
            int rc = tile_pass_t(bufs[cur], bufs[cur ^ 1], pitch, gy, g, order, k, fma, xcfl, ycfl, s);
            if (rc) return rc;
            cur ^= 1;
            i += k;
        }
        *final_idx = cur;
        return 0;
    }
    if (variant >= 7 && variant <= 18) {
        if (sizeof(T) != 4 && (variant == 9 || variant == 10 || variant >= 15)) return (int)hipErrorInvalidValue;
        const int ns = variant >= 11 ? (variant - 11) / 2 + 3 : (variant <= 8 ? 3 : 4);
        for (; i + ns <= iters; i += ns) {
            int rc = dispatch_heat<T>(order, variant, bufs[cur], bufs[cur ^ 1], pitch, gy, g, xcfl, ycfl, chunk, s);
            if (rc) return rc;
            cur ^= 1;
        }
        // remainder: two-step passes, then one single step
        variant = (variant & 1) ? 4 : 5;
    }
    if (variant == 4 || variant == 5) {
        for (; i + 1 < iters; i += 2) {
            int rc = dispatch_heat<T>(order, variant, bufs[cur], bufs[cur ^ 1], pitch, gy, g, xcfl, ycfl, chunk, s);
            if (rc) return rc;
            cur ^= 1;
        }
        variant = variant == 4 ? 2 : 6;
    }
    for (; i < iters; ++i) {
        int rc = dispatch_heat<T>(order, variant, bufs[cur], bufs[cur ^ 1], pitch, gy, g, xcfl, ycfl, chunk, s);
        if (rc) return rc;
        cur ^= 1;
    }
    *final_idx = cur;
    return 0;
}

CME_EXPORT int cme_heat_run_f32(float* a, float* b, int pitch, int gy, int xb, int xe, int yb, int ye, int order,
                                int variant, float xcfl, float ycfl, int iters, int chunk, int* final_idx,
                                void* stream) {
    return heat_run_impl<float>(a, b, pitch, gy, Region{xb, xe, yb, ye}, order, variant, xcfl, ycfl, iters, chunk,
                                final_idx, as_stream(stream));
}

CME_EXPORT int cme_heat_run_f64(double* a, double* b, int pitch, int gy, int xb, int xe, int yb, int ye, int order,
                                int variant, double xcfl, double ycfl, int iters, int chunk, int* final_idx,
                                void* stream) {
    return heat_run_impl<double>(a, b, pitch, gy, Region{xb, xe, yb, ye}, order, variant, xcfl, ycfl, iters, chunk,
                                 final_idx, as_stream(stream));
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(heat_naive_f32_o8, 256, heat_naive_kernel<float, 8>);
CME_REGISTER_KERNEL(heat_lds_f32_o8, 256, heat_lds_kernel<float, 8, 32, 1>);
CME_REGISTER_KERNEL(heat_stream_f32_o8, 256, heat_stream_kernel<float, 8, 4>);
CME_REGISTER_KERNEL(heat_stream2_f32_o8, 256, heat_stream2_kernel<float, 8, 4, false>);
CME_REGISTER_KERNEL(heat_stream2_fma_f32_o8, 256, heat_stream2_kernel<float, 8, 4, true>);
CME_REGISTER_KERNEL(heat_stream2_f64_o8, 256, heat_stream2_kernel<double, 8, 2, false>);
CME_REGISTER_KERNEL(heat_stream3_fma_f32_o8, 256, heat_streamn_kernel<float, 8, 4, 3, true>);
CME_REGISTER_KERNEL(heat_stream4_fma_f32_o8, 256, heat_streamn_kernel<float, 8, 2, 4, true>);
