// Tuning arms of the wave-pipelined heat pass (kernel: heat_pipe.h):
// rows per phase, prefetch depth, steps per pass, waves per role, wide lanes.
#include "../hip/heat_pipe.h"

// Tuning entry for the wave-pipelined NS-step pass (order 8, FMA): ns 3..6,
// rows per phase rb, input prefetch depth pd, explicit chunk or tasks per CU.
namespace {
template <int NS, int RB>
int tunep_pd(const float* p, float* c, int pitch, int gy, Region g, float xcfl, float ycfl, int chunk, int pd,
             int per_cu, hipStream_t s) {
    switch (pd) {
        case 1: return launch_pipe_multi<float, 8, NS, true, RB, 1>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl, chunk, per_cu, s);
        case 2: return launch_pipe_multi<float, 8, NS, true, RB, 2>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl, chunk, per_cu, s);
        case 11:  // depth 1, non-temporal output stores
            if constexpr (RB == 4)
                return launch_pipe_multi<float, 8, NS, true, RB, 1, true>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl, chunk,
                                                                         per_cu, s);
            return (int)hipErrorInvalidValue;
        case 12:  // depth 1, non-temporal stores, reassociated ("fast") arithmetic
            if constexpr (RB == 4)
                return launch_pipe_multi<float, 8, NS, 2, RB, 1, true>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl, chunk,
                                                                      per_cu, s);
            return (int)hipErrorInvalidValue;
        case 13:  // the same, registers capped for 4 waves per SIMD
            if constexpr (RB == 4)
                return launch_pipe_multi<float, 8, NS, 3, RB, 1, true>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl, chunk,
                                                                      per_cu, s);
            return (int)hipErrorInvalidValue;
        case 21:  // + two waves per role (seams through LDS)
            if constexpr (RB == 4)
                return launch_pipe_multi<float, 8, NS, true, RB, 1, true, 2>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                            chunk, per_cu, s);
            return (int)hipErrorInvalidValue;
        case 41:  // + four waves per role
            if constexpr (RB == 4 && NS <= 4)
                return launch_pipe_multi<float, 8, NS, true, RB, 1, true, 4>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                            chunk, per_cu, s);
            return (int)hipErrorInvalidValue;
        case 81:  // wide lanes: 8 columns per lane, non-temporal stores
            if constexpr (RB <= 4 && NS <= 5)
                return launch_pipe_multi<float, 8, NS, true, RB, 1, true, 1, 8>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                               chunk, per_cu, s);
            return (int)hipErrorInvalidValue;
        case 85:  // wide lanes, FMA chains interleaved across the lane's points (bitwise = 81)
            if constexpr (RB <= 4 && NS <= 5)
                return launch_pipe_multi<float, 8, NS, 4, RB, 1, true, 1, 8>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                            chunk, per_cu, s);
            return (int)hipErrorInvalidValue;
        case 86:  // wide lanes, term-major FMA chains, roles 1.. read x-neighbours from the LDS ring
            if constexpr (RB <= 4 && NS <= 4)
                return launch_pipe_multi<float, 8, NS, 4, RB, 1, true, 1, 8, 0, true>(p, c, pitch, gy, &g, 1, g, xcfl,
                                                                                     ycfl, chunk, per_cu, s);
            return (int)hipErrorInvalidValue;
        case 87:  // wide lanes, term-major, prefetch depth 2 (RB 1: 151 VGPRs; RB 2: 175 = 2 waves/SIMD)
            if constexpr (RB <= 2 && NS == 4)
                return launch_pipe_multi<float, 8, NS, 4, RB, 2, true, 1, 8>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                            chunk, per_cu, s);
            return (int)hipErrorInvalidValue;
        case 89:  // wide lanes, term-major, RB 1, prefetch depth 3
            if constexpr (RB == 1 && NS == 4)
                return launch_pipe_multi<float, 8, NS, 4, RB, 3, true, 1, 8>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                            chunk, per_cu, s);
            return (int)hipErrorInvalidValue;
        case 88:  // wide lanes, term-major, RB 1 capped at 4 waves per SIMD (128 VGPRs, 15 spilled)
            if constexpr (RB == 1 && NS == 4)
                return launch_pipe_multi<float, 8, NS, 4, RB, 1, true, 1, 8, 4>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                               chunk, per_cu, s);
            return (int)hipErrorInvalidValue;
        case 91:  // wide lanes, reassociated ("fast") arithmetic: 17 instead of 20 flop-instructions per point
            if constexpr (RB == 2 && NS <= 4)
                return launch_pipe_multi<float, 8, NS, 2, RB, 1, true, 1, 8>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                            chunk, per_cu, s);
            return (int)hipErrorInvalidValue;
        case 92:  // wide lanes, reassociated, registers capped for 3 waves per SIMD
            if constexpr (RB == 2 && NS <= 4)
                return launch_pipe_multi<float, 8, NS, 2, RB, 1, true, 1, 8, 3>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                               chunk, per_cu, s);
            return (int)hipErrorInvalidValue;
        case 95:  // wide lanes, reassociated, terms interleaved across the lane's points (bitwise = 91)
            if constexpr (RB == 2 && NS <= 4)
                return launch_pipe_multi<float, 8, NS, 5, RB, 1, true, 1, 8>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                            chunk, per_cu, s);
            return (int)hipErrorInvalidValue;
        case 96:  // the same, capped for 3 waves per SIMD
            if constexpr (RB == 2 && NS <= 4)
                return launch_pipe_multi<float, 8, NS, 5, RB, 1, true, 1, 8, 3>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                               chunk, per_cu, s);
            return (int)hipErrorInvalidValue;
        case 97:  // wide lanes, reassociated term-major, ONE row per phase, 3 waves per SIMD (168 VGPRs, no spill)
            if constexpr (RB == 1 && NS == 4)
                return launch_pipe_multi<float, 8, NS, 5, RB, 1, true, 1, 8, 3>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                               chunk, per_cu, s);
            return (int)hipErrorInvalidValue;
        case 83:  // wide lanes, registers capped for 3 / 4 waves per SIMD
        case 84:
            if constexpr (RB == 2 && NS == 4) {
                if (pd == 83)
                    return launch_pipe_multi<float, 8, NS, true, RB, 1, true, 1, 8, 3>(p, c, pitch, gy, &g, 1, g, xcfl,
                                                                                      ycfl, chunk, per_cu, s);
                return launch_pipe_multi<float, 8, NS, true, RB, 1, true, 1, 8, 4>(p, c, pitch, gy, &g, 1, g, xcfl, ycfl,
                                                                                  chunk, per_cu, s);
            }
            return (int)hipErrorInvalidValue;
        default: return (int)hipErrorInvalidValue;
    }
}
template <int NS>
int tunep_rb(const float* p, float* c, int pitch, int gy, Region g, float xcfl, float ycfl, int chunk, int rb, int pd,
             int per_cu, hipStream_t s) {
    if (rb == 4) return tunep_pd<NS, 4>(p, c, pitch, gy, g, xcfl, ycfl, chunk, pd, per_cu, s);
    if constexpr (NS == 4) {
        if (rb == 1 && pd >= 85) return tunep_pd<NS, 1>(p, c, pitch, gy, g, xcfl, ycfl, chunk, pd, per_cu, s);
    }
    if constexpr (NS <= 4) {
        if (rb == 2) return tunep_pd<NS, 2>(p, c, pitch, gy, g, xcfl, ycfl, chunk, pd, per_cu, s);
        if (rb == 8) return tunep_pd<NS, 8>(p, c, pitch, gy, g, xcfl, ycfl, chunk, pd, per_cu, s);
    }
    return (int)hipErrorInvalidValue;
}
}  // namespace

CME_EXPORT int cme_heat_pipe_tune(const float* prev, float* curr, int pitch, int gy, int xb, int xe, int yb, int ye,
                                  float xcfl, float ycfl, int chunk, int rb, int ns, int pd, int per_cu,
                                  void* stream) {
    hipStream_t s = as_stream(stream);
    const Region g{xb, xe, yb, ye};
    switch (ns) {
        case 3: return tunep_rb<3>(prev, curr, pitch, gy, g, xcfl, ycfl, chunk, rb, pd, per_cu, s);
        case 4: return tunep_rb<4>(prev, curr, pitch, gy, g, xcfl, ycfl, chunk, rb, pd, per_cu, s);
        case 5: return tunep_rb<5>(prev, curr, pitch, gy, g, xcfl, ycfl, chunk, rb, pd, per_cu, s);
        case 6: return tunep_rb<6>(prev, curr, pitch, gy, g, xcfl, ycfl, chunk, rb, pd, per_cu, s);
        default: return (int)hipErrorInvalidValue;
    }
}

// Profiling entry (benchmarks/trace_pipe_tasks.py): the production fp32
// wide-lane pass (FMA, term-major chains, RB 2) over `nout` regions as the
// fused distributed schedule launches them (deep interior first, then the
// border strips), with every workgroup recording {start, end} wall-clock
// ticks and {region << 40 | XCC_ID << 32 | HW_ID} into trace (3 x u64 per
// workgroup; the caller sizes it for the grid and zeroes it). chunk /
// per_cu: the chunk rule's overrides (0 = production rule).
CME_EXPORT int cme_heat_pipe_trace(const float* prev, float* curr, int pitch, int gy, const int* out, int nout,
                                   const int* ext, int ns, float xcfl, float ycfl, int chunk, int per_cu,
                                   unsigned long long* trace, void* stream) {
    Region gs[kMaxS2Regions];
    if (nout < 1 || nout > kMaxS2Regions || !trace) return (int)hipErrorInvalidValue;
    for (int i = 0; i < nout; ++i) gs[i] = Region{out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]};
    const Region e{ext[0], ext[1], ext[2], ext[3]};
    PipeGate gate;
    gate.trace = trace;
    hipStream_t s = as_stream(stream);
    switch (ns) {
        case 3: return launch_pipe_multi<float, 8, 3, 4, 2, 1, true, 1, 8>(prev, curr, pitch, gy, gs, nout, e, xcfl, ycfl, chunk, per_cu, s, gate);
        case 4: return launch_pipe_multi<float, 8, 4, 4, 2, 1, true, 1, 8>(prev, curr, pitch, gy, gs, nout, e, xcfl, ycfl, chunk, per_cu, s, gate);
        default: return (int)hipErrorInvalidValue;
    }
}
