// Wave-pipelined temporal blocking for the 2-D heat stencil (gfx950).
//
// Same capability as the NS-step streamN pass of heat2d.hip -- NS FTCS
// timesteps of the reference's stencil (hw/hw2/solution/2dHeat_solution.cu:
// 344-369, hw/hw5/2dHeat_solution.cpp:501-628 loops) per HBM pass, over up to
// four output regions with a shared intermediate-step region -- with the
// timesteps of one strip-chunk split across the waves of a workgroup.
#include <stdlib.h>

#include "cme213/common.h"
#include "cme213/heat_region.h"
#include "cme213/heat_stencil.h"
#include "cme213/vec.h"

using namespace cme;

// a wave-uniform float moved to an SGPR (usable as the scalar operand of VALU ops)
__device__ __forceinline__ float uniform_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}

// ---------------------------------------------------------------- pipe
// Wave-pipelined temporal blocking: NS (2..6) timesteps per HBM pass with the
// steps split ACROSS the waves of a workgroup instead of stacked in one wave.
//
// A streamN wave keeps all NS step windows in its own VGPRs (210 at NS = 3:
// two waves per SIMD) and re-computes 2(NS-1)B warm-up rows at the top of its
// chunk -- a fixed cost per wave that grows to a third of the pass when a
// strong-scaled subdomain hands every wave a short chunk (profiles/
// dist_rank_r2.md). Here a workgroup of NS waves shares ONE strip-chunk: wave
// k holds only the window of step-k rows (k = 0: input), computes step k+1 on
// lanes k+1..62-k and hands every block of RB rows to wave k+1 through a
// double-buffered LDS ring (16 B per lane, conflict-free); wave 0 streams the
// input from HBM with PD phases of loads in flight, wave NS-1 stores the
// result. One workgroup barrier per phase orders the hand-offs, wave k running
// k phases behind wave 0. Each wave then needs one (RB+2B)-row window (~100
// VGPRs), and for a given occupancy a workgroup's chunk is NS times taller
// than a streamN wave's, so the warm-up share per pass drops NS-fold. The
// arithmetic per cell, the region masks and hence the result are those of
// StreamN / NS single steps, bit for bit.
//
// WPR > 1 (waves per role): a role is WPR waves side by side, so a strip is
// 64*WPR lanes wide and the 2*NS lanes each strip loses to the shrinking
// valid range are amortised over WPR times more output columns (12.5 % of the
// lanes at NS = 4, WPR = 1; 6.25 % at WPR = 2). The x-neighbours across the
// seam between two waves of a role come from the LDS edge buffer: every wave
// publishes the edge lanes (0 and 63) of the rows it receives in phase q; they
// are the centre rows of phase q+1 (needs RB == B), which the neighbour wave
// reads back as the `old` operand of its DPP shifts (the lane with no DPP
// source keeps it). Three edge buffers, one barrier per phase.
template <typename T, int ORDER, int RB, int NS, int FMA, bool CHECK, int PD, bool NT, int WPR = 1>
struct PipeN {
    static constexpr int B = HeatOrder<ORDER>::B;
    static constexpr int NW = RB + 2 * B;
    static constexpr int P = NW / cgcd(NW, RB);
    static constexpr int Q = P * PD / cgcd(P, PD);
    static constexpr int LW = 64 * WPR;  // lanes per role (strip width / 4)
    static_assert(WPR == 1 || (RB == B && sizeof(T) == 4), "pipe: WPR > 1 needs RB == B (order 8, RB 4), fp32");
    using Ring = V4<T>[2][RB][LW];
    using Edge = V4<T>[3][RB][WPR][2];

    V4<T> w[NW];        // window of step-k rows (k = this wave's role); slot j = row r0 - (k+1)B + j
    V4<T> nxt[PD][RB];  // role 0: input rows of the next PD phases, in flight
    Ring* ring;         // ring[k]: step-(k+1) rows from role k to role k+1
    Edge* edge;         // edge[k]: seam lanes of the step-k rows role k received (WPR > 1)
    const T* src;
    T* dst;
    int pitch, gy, xbase, lane, sub, glane, e3;
    bool out_lane, full_vec;
    int y0, y1, xb, xe, xb1, xe1, yb1, ye1;
    T xcfl, ycfl;
    HeatFast<ORDER, T> fc;  // FMA >= 2 (3: capped at 4 waves/SIMD): folded weights, wave-uniform
    int r0, q;

    __device__ __forceinline__ const T* row_ptr(int r) const {
        r = r < 0 ? 0 : (r >= gy ? gy - 1 : r);
        return src + (size_t)r * pitch;
    }

    template <bool MASK>
    __device__ __forceinline__ V4<T> upd(int s_lo, int row, const V4<T>& ev) const {
        const V4<T> c = w[(s_lo + B) % NW];
        V4<T> L, R;
        if constexpr (WPR == 1) {
            L = wave_shr1(c);
            R = wave_shl1(c);
        } else {  // lane 0 / 63 keep the neighbour wave's seam value
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                L[j] = dpp_move<kDppWaveShr1>(ev[j], c[j]);
                R[j] = dpp_move<kDppWaveShl1>(ev[j], c[j]);
            }
        }
        T rowv[12];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            rowv[j] = L[j];
            rowv[4 + j] = c[j];
            rowv[8 + j] = R[j];
        }
        bool row_in = true;
        if constexpr (MASK) row_in = row >= yb1 && row < ye1;
        V4<T> o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            T xm[B], xp[B], ym[B], yp[B];
#pragma unroll
            for (int k = 0; k < B; ++k) {
                xm[k] = rowv[4 + j - (k + 1)];
                xp[k] = rowv[4 + j + (k + 1)];
                ym[k] = w[(s_lo + B - (k + 1)) % NW][j];
                yp[k] = w[(s_lo + B + (k + 1)) % NW][j];
            }
            T u;
            if constexpr (FMA >= 2)
                u = heat_update_fast<ORDER>(c[j], xm, xp, ym, yp, fc);
            else
                u = heat_update_sel<ORDER, FMA != 0>(c[j], xm, xp, ym, yp, xcfl, ycfl);
            if constexpr (MASK) {
                const int x = xbase + j;
                o[j] = (row_in && x >= xb1 && x < xe1) ? u : c[j];
            } else {
                o[j] = u;
            }
        }
        return o;
    }

    __device__ __forceinline__ void store_out(T* d, const V4<T>& o) const {
        if constexpr (NT && sizeof(T) == 4) {
            typedef float f32x4 __attribute__((ext_vector_type(4)));
            const f32x4 ov = {o[0], o[1], o[2], o[3]};
            __builtin_nontemporal_store(ov, reinterpret_cast<f32x4*>(d));
        } else {
            store4(d, o);
        }
    }

    // local phase q of role K: new step-K rows r0 - (K-1)B + i into the
    // window, step-(K+1) rows r0 - KB + i out (to the ring, or to HBM)
    template <int K, int PH>
    __device__ __forceinline__ bool phase() {
        if (r0 - (NS - 1) * B >= y1) return false;
        constexpr int S = (PH * RB) % NW;
        constexpr int ST = K + 1;  // the timestep this role computes
        const int par = q & 1;
        if constexpr (K == 0) {
            constexpr int F = PH % PD;
#pragma unroll
            for (int i = 0; i < RB; ++i) w[(S + 2 * B + i) % NW] = nxt[F][i];
            // unconditional (row_ptr clamps to the grid): a guarded prefetch
            // becomes a phi whose register copies wait on the loads just issued
#pragma unroll
            for (int i = 0; i < RB; ++i) nxt[F][i] = load4(row_ptr(r0 + PD * RB + B + i));
        } else {
#pragma unroll
            for (int i = 0; i < RB; ++i) w[(S + 2 * B + i) % NW] = ring[K - 1][par][i][glane];
        }
        V4<T> ev[RB];
        if constexpr (WPR > 1) {
            // seam values of this phase's centre rows (received last phase),
            // then publish the seam lanes of the rows just received
            const int ns = lane == 0 ? (sub > 0 ? sub - 1 : 0) : (sub + 1 < WPR ? sub + 1 : sub);
            const int pe = e3 == 0 ? 2 : e3 - 1;
#pragma unroll
            for (int i = 0; i < RB; ++i) ev[i] = edge[K][pe][i][ns][lane == 0 ? 1 : 0];
            if (lane == 0 || lane == 63) {
#pragma unroll
                for (int i = 0; i < RB; ++i) edge[K][e3][i][sub][lane == 63 ? 1 : 0] = w[(S + 2 * B + i) % NW];
            }
        }
#pragma unroll
        for (int i = 0; i < RB; ++i) {
            const int row = r0 - (ST - 1) * B + i;
            if constexpr (ST < NS) {
                if (row >= y0 - (NS - ST) * B && row < y1 + (NS - ST) * B)
                    ring[K][par][i][glane] = upd<CHECK>((S + i) % NW, row, ev[i]);
            } else if (row >= y0 && row < y1) {
                const V4<T> o = upd<false>((S + i) % NW, row, ev[i]);
                T* d = dst + (size_t)row * pitch;
                if constexpr (!CHECK) {
                    if (out_lane) store_out(d, o);
                } else if (out_lane) {
                    if (full_vec) {
                        store_out(d, o);
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if (xbase + j >= xb && xbase + j < xe) d[j] = o[j];
                    }
                }
            }
        }
        r0 += RB;
        ++q;
        if constexpr (WPR > 1) e3 = e3 == 2 ? 0 : e3 + 1;
        __syncthreads();
        if constexpr (PH + 1 < Q)
            return phase<K, PH + 1>();
        else
            return true;
    }

    // every role passes the same number of barriers: K (pipeline fill), one
    // per active phase, NS-1-K (drain)
    template <int K>
    __device__ __forceinline__ void run() {
        r0 = y0 - (NS - 1) * B;
        q = 0;
        e3 = 0;
        if constexpr (K == 0) {
#pragma unroll
            for (int i = 0; i < 2 * B; ++i) w[i] = load4(row_ptr(r0 - B + i));
#pragma unroll
            for (int f = 0; f < PD; ++f)
#pragma unroll
                for (int i = 0; i < RB; ++i) nxt[f][i] = load4(row_ptr(r0 + f * RB + B + i));
            if constexpr (WPR > 1) {  // seams of the first phase's centre rows (window slots B..2B-1)
                if (lane == 0 || lane == 63) {
#pragma unroll
                    for (int i = 0; i < RB; ++i) edge[0][2][i][sub][lane == 63 ? 1 : 0] = w[B + i];
                }
            }
        }
        if constexpr (WPR > 1) __syncthreads();
#pragma unroll
        for (int i = 0; i < K; ++i) __syncthreads();
        while (phase<K, 0>()) {
        }
#pragma unroll
        for (int i = K; i < NS - 1; ++i) __syncthreads();
    }

    template <int K = 0>
    __device__ __forceinline__ void run_role(int k) {
        if constexpr (K < NS) {
            if (k == K)
                run<K>();
            else
                run_role<K + 1>(k);
        }
    }
};

template <typename T, int ORDER, int RB, int NS, int FMA, bool CHECK, int PD, bool NT, int WPR>
__device__ __forceinline__ void pipen_run(V4<T> (*ring)[2][RB][64 * WPR], V4<T> (*edge)[3][RB][WPR][2], int k,
                                          int sub, const T* src, T* dst, int pitch, int gy, int xbase, int lane,
                                          bool out_lane, bool full_vec, int y0, int y1, int xb, int xe, int xb1,
                                          int xe1, int yb1, int ye1, T xcfl, T ycfl) {
    PipeN<T, ORDER, RB, NS, FMA, CHECK, PD, NT, WPR> st;
    st.ring = ring;
    st.edge = edge;
    st.sub = sub;
    st.glane = sub * 64 + lane;
    st.src = src;
    st.dst = dst;
    st.pitch = pitch;
    st.gy = gy;
    st.xbase = xbase;
    st.lane = lane;
    st.out_lane = out_lane;
    st.full_vec = full_vec;
    st.y0 = y0;
    st.y1 = y1;
    st.xb = xb;
    st.xe = xe;
    st.xb1 = xb1;
    st.xe1 = xe1;
    st.yb1 = yb1;
    st.ye1 = ye1;
    st.xcfl = xcfl;
    st.ycfl = ycfl;
    if constexpr (FMA >= 2) {
        const HeatFast<ORDER, T> f = heat_fast_coefs<ORDER>(xcfl, ycfl);
        st.fc.c0 = uniform_f(f.c0);
#pragma unroll
        for (int i = 0; i < HeatOrder<ORDER>::B; ++i) {
            st.fc.ax[i] = uniform_f(f.ax[i]);
            st.fc.ay[i] = uniform_f(f.ay[i]);
        }
    }
    st.run_role(k);
}

// one workgroup (NS roles x WPR waves) per strip-chunk task; regions as for streamN
template <typename T, int ORDER, int RB, int NS, int FMA, int PD = 1, bool NT = false, int WPR = 1>
__global__ __launch_bounds__(NS * WPR * 64, (FMA == 3 ? 16 / NS : 1)) void heat_pipe_kernel(
    const T* __restrict__ prev, T* __restrict__ curr, int pitch, int gy, S2Regions R, int xb1, int xe1, int yb1,
    int ye1, T xcfl, T ycfl, PipeGate gate) {
    static_assert(NS >= 2 && NS <= 6, "pipe: 2..6 steps per pass");
    __shared__ V4<T> ring[NS - 1][2][RB][64 * WPR];
    __shared__ V4<T> edge[WPR > 1 ? NS : 1][3][RB][WPR][2];
    constexpr int B = HeatOrder<ORDER>::B;
    constexpr int OUT = PipeOut<NS, WPR>::kOut;
    constexpr int LW = 64 * WPR;
    const int lane = lane_id();
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
    const int k = wv / WPR, sub = wv % WPR;
    int task = (int)blockIdx.x;
    if (task >= R.wave_end[R.n - 1]) return;  // whole workgroup
    int r = 0;
    while (task >= R.wave_end[r]) ++r;
    if (r > 0) task -= R.wave_end[r - 1];
    if (gate.flag && r >= gate.from) {  // border strips of the fused schedule: halos of the previous exchange
        if (threadIdx.x == 0 && __hip_atomic_load(gate.timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
            // ~2^24 polls (tens of seconds: an exchange that includes RCCL's
            // first-use connection setup must not trip it); sticky -- once one
            // workgroup gives up, the others stop at their next check
            for (unsigned spins = 0;; ++spins) {
                const unsigned v = __hip_atomic_load(gate.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((int)(v - gate.val) >= 0) break;
                if (spins >= (1u << 24)) {
                    __hip_atomic_store(gate.timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                if ((spins & 1023u) == 1023u &&
                    __hip_atomic_load(gate.timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)
                    break;
                __builtin_amdgcn_s_sleep(8);
            }
        }
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the halo rows the exchange wrote, not stale L1 lines
    }
    const int xb = R.xb[r], xe = R.xe[r], yb = R.yb[r], ye = R.ye[r];
    const int strips = R.strips[r], chunk = R.chunk[r];
    const int strip = task % strips;
    const int ck = task / strips;
    const int y0 = yb + ck * chunk;
    const int y1 = min(ye, y0 + chunk);
    const int xs = (xb & ~3) + strip * OUT;
    const int gl = sub * 64 + lane;
    const int xbase = xs - 4 * NS + 4 * gl;
    const int xl = min(max(xbase, 0), pitch - 4);
    const bool out_lane = (gl >= NS) && (gl <= LW - 1 - NS) && (xbase < xe) && (xbase + 4 > xb);
    const bool full_vec = (xbase >= xb) && (xbase + 4 <= xe);
    constexpr int reach = 4 * (NS - 1);
    const bool inside = (xs - reach >= xb1) && (xs + OUT + reach <= xe1) && (y0 - (NS - 1) * B >= yb1) &&
                        (y1 + (NS - 1) * B <= ye1) && (xs >= xb) && (xs + OUT <= xe);
    if (inside)
        pipen_run<T, ORDER, RB, NS, FMA, false, PD, NT, WPR>(ring, edge, k, sub, prev + xl, curr + xl, pitch, gy,
                                                             xbase, lane, out_lane, full_vec, y0, y1, xb, xe, xb1,
                                                             xe1, yb1, ye1, xcfl, ycfl);
    else
        pipen_run<T, ORDER, RB, NS, FMA, true, PD, NT, WPR>(ring, edge, k, sub, prev + xl, curr + xl, pitch, gy,
                                                            xbase, lane, out_lane, full_vec, y0, y1, xb, xe, xb1,
                                                            xe1, yb1, ye1, xcfl, ycfl);
}

// Chunk rule for the pipelined pass, in workgroup tasks: a whole number of
// rounds of the device's resident workgroups (every strip cut into the same
// number of chunks, each chunk paying its warm-up rows once). The floor
// keeps a partial second round from forming (16384^2, 74 strips, 1024
// resident: 13 chunks of 1261 rows = 962 tasks, not 14 = 1036). Thin regions
// (border strips) use ~1024 tasks. CME_PIPE_CHUNK / CME_PIPE_PER_CU override
// for sweeps (per_cu = task target per CU).
template <int NS, int RB>
int pipe_chunk(int strips, int H, int chunk_hint, int per_cu_hint, long resident, bool thin_floor) {
    static const int env_chunk = [] {
        const char* e = getenv("CME_PIPE_CHUNK");
        return e ? atoi(e) : 0;
    }();
    static const int env_per_cu = [] {
        const char* e = getenv("CME_PIPE_PER_CU");
        return e ? atoi(e) : 0;
    }();
    static const int thin_min = [] {
        const char* e = getenv("CME_PIPE_THIN_MIN");
        return e ? atoi(e) : 64;
    }();
    int chunk = chunk_hint > 0 ? chunk_hint : env_chunk;
    if (chunk <= 0) {
        const int per_cu = per_cu_hint > 0 ? per_cu_hint : env_per_cu;
        const long target = per_cu > 0 ? (long)per_cu * device_cu_count() : resident;
        const long lo = 4 * RB > 16 ? 4 * RB : 16;
        long rows;
        if ((long)strips * cdiv(H, lo) < 1024) {
            // thin regions (a distributed subdomain's border strips): every
            // chunk pays 2(NS-1)B warm-up + (NS-1)RB fill rows, so chunks are
            // at least thin_min rows (or the whole height) -- 4-row chunks
            // made the 16-row border strips of an N = 8 rank cost 10x their
            // rows, running 85 us beside the interior (profiles/
            // dist_fused_r2.md)
            // (multi-region launches only: a lone small region -- a whole
            // 1000^2 grid -- is latency-bound and wants many short chunks)
            rows = ((long)strips * H + 1023) / 1024;
            if (thin_floor) {
                rows = rows < thin_min ? thin_min : rows;
                rows = rows > H ? H : rows;
            }
            rows = rows < RB ? RB : rows;
        } else {
            // default, measured on the bench's field (benchmarks/
            // tune_heat_pipe.py, profiles/heat_pipe_chunk_r2.md): 14 tasks
            // per CU for tall regions (>= 8192 rows: ~340 / 170-row chunks
            // at 16384 / 8192 rows), 8 at >= 4096 rows, one round of the
            // resident workgroups below that (2048 rows: ~100-row chunks)
            long tasks = target;
            if (per_cu <= 0) tasks = H >= 8192 ? 14L * device_cu_count() : (H >= 4096 ? 8L * device_cu_count() : resident);
            long per_strip = tasks / strips;
            per_strip = per_strip < 1 ? 1 : per_strip;
            rows = (H + per_strip - 1) / per_strip;
            rows = rows < lo ? lo : rows;
        }
        chunk = (int)rows;
    }
    return ((chunk + RB - 1) / RB) * RB;
}

template <typename T, int ORDER, int NS, int FMA, int RB, int PD = 1, bool NT = false, int WPR = 1>
int launch_pipe_multi(const T* prev, T* curr, int pitch, int gy, const Region* gs, int n, Region g1, T xcfl, T ycfl,
                      int chunk_hint, int per_cu, hipStream_t s, PipeGate gate = PipeGate{}) {
    if (n < 1 || n > kMaxS2Regions) return (int)hipErrorInvalidValue;
    if ((pitch & 63) != 0) return (int)hipErrorInvalidValue;
    static const long resident = [] {
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, heat_pipe_kernel<T, ORDER, RB, NS, FMA, PD, NT, WPR>,
                                                         NS * WPR * 64, 0) != hipSuccess || per_cu < 1)
            per_cu = 1;
        return (long)per_cu * device_cu_count();
    }();
    S2Regions R{};
    int tasks = 0;
    const int gate_from = gate.from;
    gate.from = kMaxS2Regions;  // region index in R of the first gated input region
    for (int i = 0; i < n; ++i) {
        const Region& g = gs[i];
        const int H = g.ye - g.yb;
        if (i >= gate_from && gate.from == kMaxS2Regions) gate.from = R.n;
        if (H <= 0 || g.xe <= g.xb) continue;
        const int strips = (int)cdiv(g.xe - (g.xb & ~3), PipeOut<NS, WPR>::kOut);
        const int chunk = pipe_chunk<NS, RB>(strips, H, chunk_hint, per_cu, resident, n > 1);
        const int k = R.n++;
        R.xb[k] = g.xb, R.xe[k] = g.xe, R.yb[k] = g.yb, R.ye[k] = g.ye;
        R.strips[k] = strips;
        R.chunk[k] = chunk;
        tasks += strips * (int)cdiv(H, chunk);
        R.wave_end[k] = tasks;
    }
    if (R.n == 0) return 0;
    if (gate.flag && gate.from < R.n) {
        // the gated (border) workgroups spin until the comm stream's exchange
        // lands; they are dispatched last, and must leave most resident slots
        // to the interior and to the exchange's own kernels --
        // else refuse (the caller falls back to the event schedule)
        const long gated = tasks - (gate.from > 0 ? R.wave_end[gate.from - 1] : 0);
        if (2 * gated > resident) return (int)hipErrorInvalidConfiguration;
    }
    hipLaunchKernelGGL((heat_pipe_kernel<T, ORDER, RB, NS, FMA, PD, NT, WPR>), dim3(tasks), dim3(NS * WPR * 64), 0, s,
                       prev, curr, pitch, gy, R, g1.xb, g1.xe, g1.yb, g1.ye, xcfl, ycfl, gate);
    CME_LAUNCH_STATUS();
}


// Production entry: NS (3, 4) timesteps in one pass, like cme_heat_stepn_f32
// (intermediate steps over `ext`, the last writes `out`, nout <= 4 regions).
// RB = 4 rows per phase, one phase of input loads in flight, non-temporal
// output stores (benchmarks/tune_heat_pipe.py, profiles/heat_pipe_r2.md).
namespace {
template <int ORDER, bool FMA>
int pipe_ns(const float* p, float* c, int pitch, int gy, const Region* gs, int n, Region e, int ns, float xcfl,
            float ycfl, int chunk, hipStream_t s, PipeGate gate) {
    switch (ns) {
        case 3: return launch_pipe_multi<float, ORDER, 3, FMA, 4, 1, true>(p, c, pitch, gy, gs, n, e, xcfl, ycfl, chunk, 0, s, gate);
        case 4: return launch_pipe_multi<float, ORDER, 4, FMA, 4, 1, true>(p, c, pitch, gy, gs, n, e, xcfl, ycfl, chunk, 0, s, gate);
        default: return (int)hipErrorInvalidValue;
    }
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
    return fma ? pipe_order_f64<true>(order, prev, curr, pitch, gy, gs, nout, e, nsteps, xcfl, ycfl, 0,
                                      as_stream(stream), gate)
               : pipe_order_f64<false>(order, prev, curr, pitch, gy, gs, nout, e, nsteps, xcfl, ycfl, 0,
                                       as_stream(stream), gate);
}

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
        default: return (int)hipErrorInvalidValue;
    }
}
template <int NS>
int tunep_rb(const float* p, float* c, int pitch, int gy, Region g, float xcfl, float ycfl, int chunk, int rb, int pd,
             int per_cu, hipStream_t s) {
    if (rb == 4) return tunep_pd<NS, 4>(p, c, pitch, gy, g, xcfl, ycfl, chunk, pd, per_cu, s);
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

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(heat_pipe3_fma_f32_o8, 192, heat_pipe_kernel<float, 8, 4, 3, true, 1, true>);
CME_REGISTER_KERNEL(heat_pipe4_fma_f32_o8, 256, heat_pipe_kernel<float, 8, 4, 4, true, 1, true>);
