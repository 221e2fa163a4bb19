// Reassociated ("fast") arithmetic for the 2-D heat stencil on the GPU.
//
// The same FTCS update as the reference's stencil (hw/hw2/solution/
// 2dHeat_solution.cu:344-369) with the CFL numbers folded into the weights
// and each symmetric pair summed first (heat_stencil.h heat_update_fast):
// 17 flop-instructions per point at order 8 instead of 20 (FMA-contracted) or
// 38 (exact). A different rounding order from the reference's expression
// tree, within its 10-ULP criterion of the exact result (tests/
// test_heat_pipe.py test_fast_oracle_close_to_exact); bitwise equal to the
// CPU fast oracle (csrc/cpu heat2d_cpu.cpp cme_cpu_heat_step_fast_*), which
// shares the expression.
//
// Why it exists: the flagship pass is VALU-issue and power bound. On the
// wide-lane pipelined pass the reassociated form with its terms interleaved
// across a lane's 8 points (heat_pipe.h FMA arm 5) runs 6.5 % faster than the
// FMA-contracted pass on random data at 16384^2 and 8 % faster on one N = 8
// rank's 2048-row share (profiles/heat_fast_r4.md).
//
// Entry points:
//   cme_heat_step_fast_f32/f64 : one step over a region (a plain one-thread-
//                                per-point kernel: remainders, self-tests)
//   cme_heat_pipe_fast_f32     : 2-4 steps in one wide-lane pipelined pass
//                                over <= 4 output regions (optionally gated:
//                                the fused distributed schedule), order 8
//   cme_heat_run_fast_f32      : a whole-interior multi-pass run (heat_run)
#include "heat_pipe.h"

using namespace cme;

namespace {

template <typename T, int ORDER>
__global__ __launch_bounds__(256) void heat_step_fast_kernel(const T* __restrict__ prev, T* __restrict__ curr,
                                                             int pitch, Region g, HeatFast<ORDER, T> f) {
    constexpr int B = HeatOrder<ORDER>::B;
    const int x = g.xb + (int)(blockIdx.x * 64 + threadIdx.x);
    const int y = g.yb + (int)(blockIdx.y * 4 + threadIdx.y);
    if (x >= g.xe || y >= g.ye) return;
    const T* r = prev + (size_t)y * pitch + x;
    T xm[B], xp[B], ym[B], yp[B];
#pragma unroll
    for (int k = 0; k < B; ++k) {
        xm[k] = r[-(k + 1)];
        xp[k] = r[k + 1];
        ym[k] = r[-(ptrdiff_t)(k + 1) * pitch];
        yp[k] = r[(ptrdiff_t)(k + 1) * pitch];
    }
    curr[(size_t)y * pitch + x] = heat_update_fast<ORDER>(r[0], xm, xp, ym, yp, f);
}

template <typename T, int ORDER>
int step_fast_o(const T* p, T* c, int pitch, Region g, T xcfl, T ycfl, hipStream_t s) {
    const int w = g.xe - g.xb, h = g.ye - g.yb;
    if (w <= 0 || h <= 0) return 0;
    const HeatFast<ORDER, T> f = heat_fast_coefs<ORDER>(xcfl, ycfl);
    hipLaunchKernelGGL((heat_step_fast_kernel<T, ORDER>), dim3(cdiv(w, 64), cdiv(h, 4)), dim3(64, 4), 0, s, p, c,
                       pitch, g, f);
    return (int)hipGetLastError();
}

template <typename T>
int step_fast(const T* p, T* c, int pitch, Region g, int order, T xcfl, T ycfl, hipStream_t s) {
    switch (order) {
        case 2: return step_fast_o<T, 2>(p, c, pitch, g, xcfl, ycfl, s);
        case 4: return step_fast_o<T, 4>(p, c, pitch, g, xcfl, ycfl, s);
        case 8: return step_fast_o<T, 8>(p, c, pitch, g, xcfl, ycfl, s);
        default: return (int)hipErrorInvalidValue;
    }
}

}  // namespace

CME_EXPORT int cme_heat_step_fast_f32(const float* prev, float* curr, int pitch, int gy, int xb, int xe, int yb,
                                      int ye, int order, float xcfl, float ycfl, void* stream) {
    (void)gy;
    return step_fast<float>(prev, curr, pitch, Region{xb, xe, yb, ye}, order, xcfl, ycfl, as_stream(stream));
}

CME_EXPORT int cme_heat_step_fast_f64(const double* prev, double* curr, int pitch, int gy, int xb, int xe, int yb,
                                      int ye, int order, double xcfl, double ycfl, void* stream) {
    (void)gy;
    return step_fast<double>(prev, curr, pitch, Region{xb, xe, yb, ye}, order, xcfl, ycfl, as_stream(stream));
}

// nsteps (2-4) reassociated timesteps in one pass of the wide-lane pipelined
// kernel (fp32, order 8: FMA arm 5 = terms interleaved across the lane's 8
// points, registers capped for 3 waves per SIMD), like cme_heat_pipe_f32:
// intermediate steps over `ext`, the last writes the nout (<= 4) regions of
// `out`. flag != nullptr: regions [wait_from, nout) wait for *flag >= value
// first (the fused distributed schedule; timeout: the sticky give-up word).
CME_EXPORT int cme_heat_pipe_fast_f32(const float* prev, float* curr, int pitch, int gy, const int* out, int nout,
                                      const int* ext, int order, int nsteps, float xcfl, float ycfl, int chunk,
                                      int wait_from, const unsigned* flag, unsigned value, unsigned* timeout,
                                      void* stream) {
    Region gs[kMaxS2Regions];
    if (order != 8 || nout < 1 || nout > kMaxS2Regions || (flag && !timeout)) return (int)hipErrorInvalidValue;
    for (int i = 0; i < nout; ++i) gs[i] = Region{out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]};
    const Region e{ext[0], ext[1], ext[2], ext[3]};
    PipeGate gate;
    if (flag) {
        gate.flag = flag;
        gate.val = value;
        gate.from = wait_from;
        gate.timeout = timeout;
        const long v = cme::tune_get(cme::kTuneDistGateSpins);
        gate.spins = v > 0 ? (unsigned)v : (1u << 24);
    }
    hipStream_t s = as_stream(stream);
    // four steps (the production pass): registers capped for 3 waves per SIMD
    // (168 VGPRs, 32 B/lane of scratch) -- 0.1537 vs 0.1653 ms/step uncapped
    // (2 waves per SIMD) on random data; two / three steps (remainders only)
    // uncapped: the same cap spills hundreds of bytes per lane there
    switch (nsteps) {
        case 2: return launch_pipe_multi<float, 8, 2, 5, 2, 1, true, 1, 8>(prev, curr, pitch, gy, gs, nout, e, xcfl, ycfl, chunk, 0, s, gate);
        case 3: return launch_pipe_multi<float, 8, 3, 5, 2, 1, true, 1, 8>(prev, curr, pitch, gy, gs, nout, e, xcfl, ycfl, chunk, 0, s, gate);
        case 4: return launch_pipe_multi<float, 8, 4, 5, 2, 1, true, 1, 8, 3>(prev, curr, pitch, gy, gs, nout, e, xcfl, ycfl, chunk, 0, s, gate);
        default: return (int)hipErrorInvalidValue;
    }
}

// iters reassociated timesteps of the whole region [xb, xe) x [yb, ye) from
// `a` (every cell outside it holds the same fixed value in a and b): passes
// of ns (1-4) steps, the remainder as one shorter pass (a single step on the
// plain kernel). *final_idx = 0 if the result is in a, 1 if in b.
CME_EXPORT int cme_heat_run_fast_f32(float* a, float* b, int pitch, int gy, int xb, int xe, int yb, int ye, int order,
                                     int ns, float xcfl, float ycfl, int iters, int* final_idx, void* stream) {
    if (ns < 1 || ns > 4 || (ns > 1 && order != 8) || iters < 0) return (int)hipErrorInvalidValue;
    const int r[4] = {xb, xe, yb, ye};
    float* bufs[2] = {a, b};
    int cur = 0;
    int i = 0;
    while (i < iters) {
        const int k = iters - i < ns ? iters - i : ns;
        const int rc = k >= 2 ? cme_heat_pipe_fast_f32(bufs[cur], bufs[cur ^ 1], pitch, gy, r, 1, r, order, k, xcfl,
                                                       ycfl, 0, 0, nullptr, 0u, nullptr, stream)
                              : cme_heat_step_fast_f32(bufs[cur], bufs[cur ^ 1], pitch, gy, xb, xe, yb, ye, order,
                                                       xcfl, ycfl, stream);
        if (rc) return rc;
        cur ^= 1;
        i += k;
    }
    *final_idx = cur;
    return 0;
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(heat_pipe4w_fast_f32_o8, 256, heat_pipe_kernel<float, 8, 2, 4, 5, 1, true, 1, 8, 3>);
CME_REGISTER_KERNEL(heat_step_fast_f32_o8, 256, heat_step_fast_kernel<float, 8>);
