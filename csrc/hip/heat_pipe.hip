// C entry points of the wave-pipelined heat pass (kernel: heat_pipe.h).
#include "heat_pipe.h"

// Production entry: NS (3, 4) timesteps in one pass, like cme_heat_stepn_f32
// (intermediate steps over `ext`, the last writes `out`, nout <= 4 regions).
// fp32 order 8: wide lanes (8 columns per lane), RB = 2 rows per phase (156
// VGPRs, 3 waves per SIMD), the FMA chains of a lane's 8 points interleaved,
// one phase of input loads in flight, non-temporal output stores: 0.1308 vs
// 0.1417 ms/step for the round-2 4-column pass (RB 4) on the bench's 16384^2
// field (benchmarks/tune_heat_pipe.py, profiles/heat_pipe_wide_r3.md).
// Orders 2 / 4 keep 4 columns per lane (faster on the 4000^2 rows there).
// CME_PIPE_VW=4 / 8 forces one width at every order.
namespace {
// CME_PIPE_VW: unset = the measured default (8 columns per lane at order 8,
// 4 at orders 2 / 4), 4 / 8 = that width at every order
int pipe_vw_env() {
    const long x = cme::tune_get(cme::kTunePipeVW);
    return (x == 4 || x == 8) ? (int)x : 0;
}

template <int ORDER, bool FMA>
int pipe_ns(const float* p, float* c, int pitch, int gy, const Region* gs, int n, Region e, int ns, float xcfl,
            float ycfl, int chunk, hipStream_t s, PipeGate gate) {
    constexpr int FW = FMA ? 4 : 0;  // wide lanes: term-major FMA chains (bitwise = FMA)
    const int env = pipe_vw_env();
    if (env == 8 || (env == 0 && ORDER == 8)) {
        switch (ns) {
            case 3: return launch_pipe_multi<float, ORDER, 3, FW, 2, 1, true, 1, 8>(p, c, pitch, gy, gs, n, e, xcfl, ycfl, chunk, 0, s, gate);
            case 4: return launch_pipe_multi<float, ORDER, 4, FW, 2, 1, true, 1, 8>(p, c, pitch, gy, gs, n, e, xcfl, ycfl, chunk, 0, s, gate);
            case 5: return launch_pipe_multi<float, ORDER, 5, FW, 2, 1, true, 1, 8>(p, c, pitch, gy, gs, n, e, xcfl, ycfl, chunk, 0, s, gate);
            case 6: return launch_pipe_multi<float, ORDER, 6, FW, 2, 1, true, 1, 8>(p, c, pitch, gy, gs, n, e, xcfl, ycfl, chunk, 0, s, gate);
            default: return (int)hipErrorInvalidValue;
        }
    }
    switch (ns) {
        case 3: return launch_pipe_multi<float, ORDER, 3, FMA, 4, 1, true>(p, c, pitch, gy, gs, n, e, xcfl, ycfl, chunk, 0, s, gate);
        case 4: return launch_pipe_multi<float, ORDER, 4, FMA, 4, 1, true>(p, c, pitch, gy, gs, n, e, xcfl, ycfl, chunk, 0, s, gate);
        // 5 / 6 steps per pass: orders 2 / 4 are HBM-bound at 4 (profiles/heat_pipe_wide_r3.md)
        case 5: return launch_pipe_multi<float, ORDER, 5, FMA, 4, 1, true>(p, c, pitch, gy, gs, n, e, xcfl, ycfl, chunk, 0, s, gate);
        case 6: return launch_pipe_multi<float, ORDER, 6, FMA, 4, 1, true>(p, c, pitch, gy, gs, n, e, xcfl, ycfl, chunk, 0, s, gate);
        default: return (int)hipErrorInvalidValue;
    }
}
// poll bound of the fused schedule's gated border workgroups (PipeGate):
// CME_DIST_GATE_SPINS, read per call (a test forces the timeout path in-process)
unsigned gate_spin_limit() {
    const long v = cme::tune_get(cme::kTuneDistGateSpins);
    return v > 0 ? (unsigned)v : (1u << 24);
}

template <bool FMA>
int pipe_order(int order, const float* p, float* c, int pitch, int gy, const Region* gs, int n, Region e, int ns,
               float xcfl, float ycfl, int chunk, hipStream_t s, PipeGate gate = PipeGate{}) {
    switch (order) {
        case 2: return pipe_ns<2, FMA>(p, c, pitch, gy, gs, n, e, ns, xcfl, ycfl, chunk, s, gate);
        case 4: return pipe_ns<4, FMA>(p, c, pitch, gy, gs, n, e, ns, xcfl, ycfl, chunk, s, gate);
        case 8: return pipe_ns<8, FMA>(p, c, pitch, gy, gs, n, e, ns, xcfl, ycfl, chunk, s, gate);
        default: return (int)hipErrorInvalidValue;
    }
}
}  // namespace

CME_EXPORT int cme_heat_pipe_f32(const float* prev, float* curr, int pitch, int gy, const int* out, int nout,
                                 const int* ext, int order, int nsteps, float xcfl, float ycfl, int chunk, int fma,
                                 void* stream) {
    Region gs[kMaxS2Regions];
    if (nout < 1 || nout > kMaxS2Regions) return (int)hipErrorInvalidValue;
    for (int i = 0; i < nout; ++i) gs[i] = Region{out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]};
    const Region e{ext[0], ext[1], ext[2], ext[3]};
    return fma ? pipe_order<true>(order, prev, curr, pitch, gy, gs, nout, e, nsteps, xcfl, ycfl, chunk,
                                  as_stream(stream))
               : pipe_order<false>(order, prev, curr, pitch, gy, gs, nout, e, nsteps, xcfl, ycfl, chunk,
                                   as_stream(stream));
}

// fp64: the same pass on doubles (32 B per lane per row; RB = 2 rows per
// phase keeps the window + prefetch within ~128 VGPRs). The hw5 workload is
// double precision (hw/hw5/2dHeat_solution.cpp:63-84).
namespace {
template <int ORDER, bool FMA>
int pipe_ns_f64(const double* p, double* c, int pitch, int gy, const Region* gs, int n, Region e, int ns, double xcfl,
                double ycfl, int chunk, hipStream_t s, PipeGate gate) {
    // (a term-major chain order, the fp32 wide pass's, was measured here on
    // the hw5 shapes: 1000^2 / 2000^2 / 4000^2, orders 4 and 8, within 1 %
    // of this chain-major order -- profiles/heat_tile_r4.md -- and removed)
    switch (ns) {
        case 3: return launch_pipe_multi<double, ORDER, 3, FMA, 2, 1, false>(p, c, pitch, gy, gs, n, e, xcfl, ycfl, chunk, 0, s, gate);
        case 4: return launch_pipe_multi<double, ORDER, 4, FMA, 2, 1, false>(p, c, pitch, gy, gs, n, e, xcfl, ycfl, chunk, 0, s, gate);
        default: return (int)hipErrorInvalidValue;
    }
}
template <bool FMA>
int pipe_order_f64(int order, const double* p, double* c, int pitch, int gy, const Region* gs, int n, Region e,
                   int ns, double xcfl, double ycfl, int chunk, hipStream_t s, PipeGate gate = PipeGate{}) {
    switch (order) {
        case 2: return pipe_ns_f64<2, FMA>(p, c, pitch, gy, gs, n, e, ns, xcfl, ycfl, chunk, s, gate);
        case 4: return pipe_ns_f64<4, FMA>(p, c, pitch, gy, gs, n, e, ns, xcfl, ycfl, chunk, s, gate);
        case 8: return pipe_ns_f64<8, FMA>(p, c, pitch, gy, gs, n, e, ns, xcfl, ycfl, chunk, s, gate);
        default: return (int)hipErrorInvalidValue;
    }
}
}  // namespace

CME_EXPORT int cme_heat_pipe_f64(const double* prev, double* curr, int pitch, int gy, const int* out, int nout,
                                 const int* ext, int order, int nsteps, double xcfl, double ycfl, int chunk, int fma,
                                 void* stream) {
    Region gs[kMaxS2Regions];
    if (nout < 1 || nout > kMaxS2Regions) return (int)hipErrorInvalidValue;
    for (int i = 0; i < nout; ++i) gs[i] = Region{out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]};
    const Region e{ext[0], ext[1], ext[2], ext[3]};
    return fma ? pipe_order_f64<true>(order, prev, curr, pitch, gy, gs, nout, e, nsteps, xcfl, ycfl, chunk,
                                      as_stream(stream))
               : pipe_order_f64<false>(order, prev, curr, pitch, gy, gs, nout, e, nsteps, xcfl, ycfl, chunk,
                                       as_stream(stream));
}

// The same pass with regions [wait_from, nout) gated on *flag >= value (the
// fused distributed schedule: deep interior and border strips in ONE launch,
// the border workgroups waiting for the previous halo exchange).
CME_EXPORT int cme_heat_pipe_gated_f32(const float* prev, float* curr, int pitch, int gy, const int* out, int nout,
                                       const int* ext, int order, int nsteps, float xcfl, float ycfl, int fma,
                                       int wait_from, const unsigned* flag, unsigned value, unsigned* timeout,
                                       void* stream) {
    Region gs[kMaxS2Regions];
    if (nout < 1 || nout > kMaxS2Regions || (flag && !timeout)) return (int)hipErrorInvalidValue;
    for (int i = 0; i < nout; ++i) gs[i] = Region{out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]};
    const Region e{ext[0], ext[1], ext[2], ext[3]};
    PipeGate gate;
    gate.flag = flag;
    gate.val = value;
    gate.from = wait_from;
    gate.timeout = timeout;
    gate.spins = gate_spin_limit();
    return fma ? pipe_order<true>(order, prev, curr, pitch, gy, gs, nout, e, nsteps, xcfl, ycfl, 0, as_stream(stream),
                                  gate)
               : pipe_order<false>(order, prev, curr, pitch, gy, gs, nout, e, nsteps, xcfl, ycfl, 0,
                                   as_stream(stream), gate);
}

// fp64 twin of cme_heat_pipe_gated_f32 (the fused schedule on the hw5
// workload's doubles, hw/hw5/2dHeat_solution.cpp:63-84).
CME_EXPORT int cme_heat_pipe_gated_f64(const double* prev, double* curr, int pitch, int gy, const int* out, int nout,
                                       const int* ext, int order, int nsteps, double xcfl, double ycfl, int fma,
                                       int wait_from, const unsigned* flag, unsigned value, unsigned* timeout,
                                       void* stream) {
    Region gs[kMaxS2Regions];
    if (nout < 1 || nout > kMaxS2Regions || (flag && !timeout)) return (int)hipErrorInvalidValue;
    for (int i = 0; i < nout; ++i) gs[i] = Region{out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]};
    const Region e{ext[0], ext[1], ext[2], ext[3]};
    PipeGate gate;
    gate.flag = flag;
    gate.val = value;
    gate.from = wait_from;
    gate.timeout = timeout;
    gate.spins = gate_spin_limit();
    return fma ? pipe_order_f64<true>(order, prev, curr, pitch, gy, gs, nout, e, nsteps, xcfl, ycfl, 0,
                                      as_stream(stream), gate)
               : pipe_order_f64<false>(order, prev, curr, pitch, gy, gs, nout, e, nsteps, xcfl, ycfl, 0,
                                       as_stream(stream), gate);
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(heat_pipe3_fma_f32_o8, 192, heat_pipe_kernel<float, 8, 4, 3, true, 1, true>);
CME_REGISTER_KERNEL(heat_pipe4_fma_f32_o8, 256, heat_pipe_kernel<float, 8, 4, 4, true, 1, true>);
CME_REGISTER_KERNEL(heat_pipe3w_fma_f32_o8, 192, heat_pipe_kernel<float, 8, 2, 3, 4, 1, true, 1, 8>);
CME_REGISTER_KERNEL(heat_pipe4w_fma_f32_o8, 256, heat_pipe_kernel<float, 8, 2, 4, 4, 1, true, 1, 8>);
CME_REGISTER_KERNEL(heat_pipe4w_f32_o8, 256, heat_pipe_kernel<float, 8, 2, 4, false, 1, true, 1, 8>);
