// Wave-pipelined temporal blocking for the 2-D heat stencil (gfx950).
//
// Same capability as the NS-step streamN pass of heat2d.hip -- NS FTCS
// timesteps of the reference's stencil (hw/hw2/solution/2dHeat_solution.cu:
// 344-369, hw/hw5/2dHeat_solution.cpp:501-628 loops) per HBM pass, over up to
// four output regions with a shared intermediate-step region -- with the
// timesteps of one strip-chunk split across the waves of a workgroup.
//
// Kernel template, chunk rule and launcher; the C entry points are in
// heat_pipe.hip (production) and heat_pipe_tune.hip (tuning arms).
#pragma once
#include <limits.h>
#include <stdlib.h>

#include "cme213/common.h"
#include "cme213/tuning.h"
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
//
// VW = 8 (wide lanes, the order-8 fp32 production pass): each lane holds 8
// consecutive columns, so the 2B DPP moves of the x-neighbours serve 8 points
// instead of 4, more packed-FMA operand pairs lie inside one lane, and a strip
// loses ceil(NS*B/8) lanes per side instead of NS (60 of 64 lanes write at
// NS = 4). 156 VGPRs at RB = 2: three waves per SIMD. Strips start on
// 8-column boundaries so no lane straddles the grid edge (profiles/
// heat_pipe_wide_r3.md). FMA = 4 issues the FMA chains of the lane's points
// term by term (heat_d2_fma_n): the same operations per point, interleaved.
//
// LX (x-neighbours from LDS): roles 1..NS-1 read the B edge columns of the
// lanes on either side of their centre rows back from the ring (two 16-B LDS
// reads per row) instead of shifting them across lanes with 2B DPP moves on
// the VALU; the centre rows arrived B/RB phases earlier, so the ring keeps
// 2 + B/RB slots. Role 0 (rows from HBM) keeps the DPP shifts.
template <typename T, int ORDER, int RB, int NS, int FMA, bool CHECK, int PD, bool NT, int WPR = 1, int VW = 4,
          bool LX = false, int OST = 0>
struct PipeN {
    static constexpr int B = HeatOrder<ORDER>::B;
    static constexpr int NW = RB + 2 * B;
    static constexpr int P = NW / cgcd(NW, RB);
    static constexpr int Q = P * PD / cgcd(P, PD);
    static constexpr int LW = 64 * WPR;  // lanes per role
    static constexpr int NH = VW / 4;    // 16-B (fp32) pieces per lane and row
    static_assert(WPR == 1 || (RB == B && sizeof(T) == 4 && VW == 4),
                  "pipe: WPR > 1 needs RB == B (order 8, RB 4), fp32, 4 columns per lane");
    static_assert(VW == 4 || (VW == 8 && sizeof(T) == 4 && B <= VW), "pipe: wide lanes are fp32, 8 columns");
    static_assert(!LX || (WPR == 1 && B % RB == 0), "pipe: LDS x-neighbours need one wave per role, RB | B");
    static constexpr int NSLOT = LX ? 2 + B / RB : 2;  // ring slots per role hand-off
    // FMA: 0 exact, 1 FMA-contracted (the reference's nvcc -fmad code), 2 / 3
    // reassociated ("fast"; 3 capped at 4 waves/SIMD), 4 FMA-contracted with
    // the chains of the lane's VW points interleaved term by term (bitwise 1),
    // 5 reassociated with the terms interleaved across the points (bitwise 2)
    static constexpr bool kFast = FMA == 2 || FMA == 3 || FMA == 5;
    static constexpr bool kTermMajor = FMA == 4;
    static constexpr bool kFastTM = FMA == 5;  // reassociated, terms issued across the lane's points
    using VT = VecN<T, VW>;
    using Ring = V4<T>[NSLOT][RB][NH][LW];
    using Edge = V4<T>[3][RB][WPR][2];

    VT w[NW];           // window of step-k rows (k = this wave's role); slot j = row r0 - (k+1)B + j
    VT nxt[PD][RB];     // role 0: input rows of the next PD phases, in flight
    Ring* ring;         // ring[k]: step-(k+1) rows from role k to role k+1
    Edge* edge;         // edge[k]: seam lanes of the step-k rows role k received (WPR > 1)
    const T* src;
    T* dst;
    // OST = 1 / 2 (the dataflow launch's hand-off, heat_flow.hip): every
    // output row / the rows outside [wt_lo, wt_hi) are stored write-through
    // (sc1 buffer stores) from the uniform base `obase` at lane column `oxl`,
    // so a completion flag needs no L2 write-back fence behind them for a
    // reader on another XCD (cdna_hip_programming.md §6 Guideline 16, R1)
    T* obase;
    int oxl;
    int wt_lo, wt_hi;  // OST = 2: rows outside [wt_lo, wt_hi) write-through, the rest as NT says
    int pitch, gy, xbase, lane, sub, glane, e3;
    int gl_l, gl_r;  // LX: the neighbour lanes (clamped into the strip; edge lanes are margin lanes)
    bool out_lane, full_vec;
    int y0, y1, xb, xe, xb1, xe1, yb1, ye1;
    T xcfl, ycfl;
    HeatFast<ORDER, T> fc;  // kFast: folded weights, wave-uniform
    int r0, q;

    __device__ __forceinline__ const T* row_ptr(int r) const {
        r = r < 0 ? 0 : (r >= gy ? gy - 1 : r);
        return src + (size_t)r * pitch;
    }

    // One output row of VW columns. The x-neighbours beyond the lane are the
    // B edge columns of the lanes on either side (DPP wave shifts; a wave
    // seam of WPR > 1 takes the neighbour wave's value from `ev`). VW = 8
    // moves 2B = 8 values per 8 points instead of per 4, and pairs more of the
    // x operands inside one lane for the packed FMAs.
    template <bool MASK, bool FROM_LDS = false>
    __device__ __forceinline__ VT upd(int s_lo, int row, const V4<T>& ev, const V4<T>& xl = V4<T>{},
                                      const V4<T>& xr = V4<T>{}) const {
        const VT c = w[(s_lo + B) % NW];
        T rowv[VW + 2 * B];
        if constexpr (FROM_LDS) {  // the left lane's last B columns, the right lane's first B
#pragma unroll
            for (int k = 0; k < B; ++k) {
                rowv[k] = xl[4 - B + k];
                rowv[B + VW + k] = xr[k];
            }
        } else if constexpr (WPR == 1) {
#pragma unroll
            for (int k = 0; k < B; ++k) {
                rowv[k] = dpp_shift<kDppWaveShr1>(c[VW - B + k]);
                rowv[B + VW + k] = dpp_shift<kDppWaveShl1>(c[k]);
            }
        } else {  // lane 0 / 63 keep the neighbour wave's seam value
#pragma unroll
            for (int k = 0; k < B; ++k) {
                rowv[k] = dpp_move<kDppWaveShr1>(ev[VW - B + k], c[VW - B + k]);
                rowv[B + VW + k] = dpp_move<kDppWaveShl1>(ev[k], c[k]);
            }
        }
#pragma unroll
        for (int j = 0; j < VW; ++j) rowv[B + j] = c[j];
        bool row_in = true;
        if constexpr (MASK) row_in = row >= yb1 && row < ye1;
        VT o;
        if constexpr (kFastTM) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
            // heat_update_fast per point (c0 c, then the x pairs, then the y
            // pairs, k = B-1..0), each term issued for all VW points first
            T u[VW];
#pragma unroll
            for (int j = 0; j < VW; ++j) u[j] = fc.c0 * c[j];
#pragma unroll
            for (int k = B - 1; k >= 0; --k)
#pragma unroll
                for (int j = 0; j < VW; ++j)
                    u[j] = fmaT<T>(fc.ax[k], rowv[B + j + (k + 1)] + rowv[B + j - (k + 1)], u[j]);
#pragma unroll
            for (int k = B - 1; k >= 0; --k)
#pragma unroll
                for (int j = 0; j < VW; ++j)
                    u[j] = fmaT<T>(fc.ay[k], w[(s_lo + B + (k + 1)) % NW][j] + w[(s_lo + B - (k + 1)) % NW][j], u[j]);
#pragma unroll
            for (int j = 0; j < VW; ++j) {
                if constexpr (MASK) {
                    const int x = xbase + j;
                    o[j] = (row_in && x >= xb1 && x < xe1) ? u[j] : c[j];
                } else {
                    o[j] = u[j];
                }
            }
            return o;
        } else if constexpr (kTermMajor) {
            T cc[VW], xm[B][VW], xp[B][VW], ym[B][VW], yp[B][VW], dx[VW], dy[VW];
#pragma unroll
            for (int j = 0; j < VW; ++j) {
                cc[j] = c[j];
#pragma unroll
                for (int k = 0; k < B; ++k) {
                    xm[k][j] = rowv[B + j - (k + 1)];
                    xp[k][j] = rowv[B + j + (k + 1)];
                    ym[k][j] = w[(s_lo + B - (k + 1)) % NW][j];
                    yp[k][j] = w[(s_lo + B + (k + 1)) % NW][j];
                }
            }
            heat_d2_fma_n<ORDER, VW>(dx, cc, xm, xp);
            heat_d2_fma_n<ORDER, VW>(dy, cc, ym, yp);
#pragma unroll
            for (int j = 0; j < VW; ++j) dx[j] = fmaT<T>(xcfl, dx[j], cc[j]);
#pragma unroll
            for (int j = 0; j < VW; ++j) {
                const T u = fmaT<T>(ycfl, dy[j], dx[j]);
                if constexpr (MASK) {
                    const int x = xbase + j;
                    o[j] = (row_in && x >= xb1 && x < xe1) ? u : c[j];
                } else {
                    o[j] = u;
                }
            }
            return o;
        }
#pragma unroll
        for (int j = 0; j < VW; ++j) {
            T xm[B], xp[B], ym[B], yp[B];
#pragma unroll
            for (int k = 0; k < B; ++k) {
                xm[k] = rowv[B + j - (k + 1)];
                xp[k] = rowv[B + j + (k + 1)];
                ym[k] = w[(s_lo + B - (k + 1)) % NW][j];
                yp[k] = w[(s_lo + B + (k + 1)) % NW][j];
            }
            T u;
            if constexpr (kFast)
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

    // OST = 1: write-through stores of output row `row` (byte offsets fit 32
    // bits: the launcher checks the buffer size)
    __device__ __forceinline__ __amdgpu_buffer_rsrc_t out_rsrc() const {
        return __builtin_amdgcn_make_buffer_rsrc(obase, (short)0, 0x7fffffff, 0x00020000);
    }
    __device__ __forceinline__ void store_out_wt(int row, const VT& o) const {
        static_assert(sizeof(T) == 4, "write-through output stores: fp32");
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const __amdgpu_buffer_rsrc_t rs = out_rsrc();
        const int off = (int)(((size_t)row * pitch + oxl) * sizeof(T));
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            const u32x4 v = {__builtin_bit_cast(unsigned, o[4 * h]), __builtin_bit_cast(unsigned, o[4 * h + 1]),
                             __builtin_bit_cast(unsigned, o[4 * h + 2]), __builtin_bit_cast(unsigned, o[4 * h + 3])};
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, off + 16 * h, 0, 16);
        }
    }
    __device__ __forceinline__ void store_one_wt(int row, int j, T v) const {
        const int off = (int)(((size_t)row * pitch + oxl + j) * sizeof(T));
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), out_rsrc(), off, 0, 16);
    }

    __device__ __forceinline__ void store_out(T* d, const VT& o) const {
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            if constexpr (NT && sizeof(T) == 4) {
                typedef float f32x4 __attribute__((ext_vector_type(4)));
                const f32x4 ov = {o[4 * h], o[4 * h + 1], o[4 * h + 2], o[4 * h + 3]};
                __builtin_nontemporal_store(ov, reinterpret_cast<f32x4*>(d + 4 * h));
            } else {
                store4(d + 4 * h, piece4(o, h));
            }
        }
    }

    // local phase q of role K: new step-K rows r0 - (K-1)B + i into the
    // window, step-(K+1) rows r0 - KB + i out (to the ring, or to HBM)
    template <int K, int PH>
    __device__ __forceinline__ bool phase() {
        if (r0 - (NS - 1) * B >= y1) return false;
        constexpr int S = (PH * RB) % NW;
        constexpr int ST = K + 1;  // the timestep this role computes
        const int par = q % NSLOT;
        const int cslot = (q + NSLOT - B / RB) % NSLOT;  // LX: slot of this phase's centre rows
        if constexpr (K == 0) {
            constexpr int F = PH % PD;
#pragma unroll
            for (int i = 0; i < RB; ++i) w[(S + 2 * B + i) % NW] = nxt[F][i];
            // unconditional (row_ptr clamps to the grid): a guarded prefetch
            // becomes a phi whose register copies wait on the loads just issued
#pragma unroll
            for (int i = 0; i < RB; ++i) nxt[F][i] = load_n<VW>(row_ptr(r0 + PD * RB + B + i));
        } else {
#pragma unroll
            for (int i = 0; i < RB; ++i)
#pragma unroll
                for (int h = 0; h < NH; ++h) {
                    const V4<T> v = ring[K - 1][par][i][h][glane];
#pragma unroll
                    for (int j = 0; j < 4; ++j) w[(S + 2 * B + i) % NW][4 * h + j] = v[j];
                }
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
                for (int i = 0; i < RB; ++i)
                    edge[K][e3][i][sub][lane == 63 ? 1 : 0] = piece4(w[(S + 2 * B + i) % NW], 0);
            }
        }
#pragma unroll
        for (int i = 0; i < RB; ++i) {
            const int row = r0 - (ST - 1) * B + i;
            if constexpr (ST < NS) {
                if (row >= y0 - (NS - ST) * B && row < y1 + (NS - ST) * B) {
                    VT o;
                    if constexpr (LX && K > 0)
                        o = upd<CHECK, true>((S + i) % NW, row, ev[i], ring[K - 1][cslot][i][NH - 1][gl_l],
                                             ring[K - 1][cslot][i][0][gl_r]);
                    else
                        o = upd<CHECK>((S + i) % NW, row, ev[i]);
#pragma unroll
                    for (int h = 0; h < NH; ++h) ring[K][par][i][h][glane] = piece4(o, h);
                }
            } else if (row >= y0 && row < y1) {
                VT o;
                if constexpr (LX && K > 0)
                    o = upd<false, true>((S + i) % NW, row, ev[i], ring[K - 1][cslot][i][NH - 1][gl_l],
                                         ring[K - 1][cslot][i][0][gl_r]);
                else
                    o = upd<false>((S + i) % NW, row, ev[i]);
                T* d = dst + (size_t)row * pitch;
                bool wt = false;
                if constexpr (OST != 0) wt = OST == 1 || row < wt_lo || row >= wt_hi;
                if (wt) {
                    if constexpr (OST != 0) {
                        if (out_lane) {
                            if (!CHECK || full_vec) {
                                store_out_wt(row, o);
                            } else {
#pragma unroll
                                for (int j = 0; j < VW; ++j)
                                    if (xbase + j >= xb && xbase + j < xe) store_one_wt(row, j, o[j]);
                            }
                        }
                    }
                } else if constexpr (!CHECK) {
                    if (out_lane) store_out(d, o);
                } else if (out_lane) {
                    if (full_vec) {
                        store_out(d, o);
                    } else {
#pragma unroll
                        for (int j = 0; j < VW; ++j)
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
            for (int i = 0; i < 2 * B; ++i) w[i] = load_n<VW>(row_ptr(r0 - B + i));
#pragma unroll
            for (int f = 0; f < PD; ++f)
#pragma unroll
                for (int i = 0; i < RB; ++i) nxt[f][i] = load_n<VW>(row_ptr(r0 + f * RB + B + i));
            if constexpr (WPR > 1) {  // seams of the first phase's centre rows (window slots B..2B-1)
                if (lane == 0 || lane == 63) {
#pragma unroll
                    for (int i = 0; i < RB; ++i) edge[0][2][i][sub][lane == 63 ? 1 : 0] = piece4(w[B + i], 0);
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

template <typename T, int ORDER, int RB, int NS, int FMA, bool CHECK, int PD, bool NT, int WPR, int VW, bool LX,
          int NSLOT, int OST = 0>
__device__ __forceinline__ void pipen_run(V4<T> (*ring)[NSLOT][RB][VW / 4][64 * WPR], V4<T> (*edge)[3][RB][WPR][2],
                                          int k, int sub, const T* src, T* dst, int pitch, int gy, int xbase,
                                          int lane, bool out_lane, bool full_vec, int y0, int y1, int xb, int xe,
                                          int xb1, int xe1, int yb1, int ye1, T xcfl, T ycfl, T* obase = nullptr,
                                          int oxl = 0, int wt_lo = 0, int wt_hi = 0) {
    PipeN<T, ORDER, RB, NS, FMA, CHECK, PD, NT, WPR, VW, LX, OST> st;
    static_assert(decltype(st)::NSLOT == NSLOT, "pipe: ring slots");
    st.obase = obase;
    st.oxl = oxl;
    st.wt_lo = wt_lo;
    st.wt_hi = wt_hi;
    st.ring = ring;
    st.edge = edge;
    st.sub = sub;
    st.glane = sub * 64 + lane;
    st.gl_l = st.glane > 0 ? st.glane - 1 : 0;
    st.gl_r = st.glane < 64 * WPR - 1 ? st.glane + 1 : 64 * WPR - 1;
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
    if constexpr (FMA == 2 || FMA == 3 || FMA == 5) {
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

// One strip-chunk task of region r of R (the whole workgroup): rows and
// columns of the task, the interior / edge instantiation, the pass itself.
// Shared by the one-pass launch (heat_pipe_kernel) and the persistent
// multi-pass dataflow launch (heat_flow.hip).
template <typename T, int ORDER, int RB, int NS, int FMA, int PD, bool NT, int WPR, int VW, bool LX, int NSLOT,
          int OST = 0>
__device__ __forceinline__ void pipe_task(V4<T> (*ring)[NSLOT][RB][VW / 4][64 * WPR],
                                          V4<T> (*edge)[3][RB][WPR][2], const S2Regions& R, int r, int task,
                                          const T* prev, T* curr, int pitch, int gy, int xb1, int xe1, int yb1,
                                          int ye1, T xcfl, T ycfl, int k, int sub, int lane, int wt_lo = 0,
                                          int wt_hi = 0) {
    constexpr int B = HeatOrder<ORDER>::B;
    using G = PipeOut<NS, WPR, VW, B>;
    constexpr int OUT = G::kOut;
    constexpr int M = G::kMargin;
    constexpr int LW = 64 * WPR;
    const int xb = R.xb[r], xe = R.xe[r], yb = R.yb[r], ye = R.ye[r];
    const int strips = R.strips[r];
    // chunk word: rows per chunk in the low 16 bits; a tapered region
    // (pipe_taper) keeps n1 = bits 16.. full chunks per strip and cuts the
    // rest -- the tasks dispatched last -- to half height
    const int chunk = R.chunk[r] & 0xffff, n1 = R.chunk[r] >> 16;
    const int strip = task % strips;
    const int ck = task / strips;
    const bool half = n1 > 0 && ck >= n1;
    const int y0 = half ? yb + n1 * chunk + (ck - n1) * (chunk >> 1) : yb + ck * chunk;
    const int y1 = min(ye, y0 + (half ? chunk >> 1 : chunk));
    const int xs = (xb & ~(VW - 1)) + strip * OUT;
    const int gl = sub * 64 + lane;
    const int xbase = xs - VW * M + VW * gl;
    const int xl = min(max(xbase, 0), pitch - VW);
    const bool out_lane = (gl >= M) && (gl <= LW - 1 - M) && (xbase < xe) && (xbase + VW > xb);
    const bool full_vec = (xbase >= xb) && (xbase + VW <= xe);
    constexpr int reach = 4 * (NS - 1);
    const bool inside = (xs - reach >= xb1) && (xs + OUT + reach <= xe1) && (y0 - (NS - 1) * B >= yb1) &&
                        (y1 + (NS - 1) * B <= ye1) && (xs >= xb) && (xs + OUT <= xe);
    if (inside)
        pipen_run<T, ORDER, RB, NS, FMA, false, PD, NT, WPR, VW, LX, NSLOT, OST>(
            ring, edge, k, sub, prev + xl, curr + xl, pitch, gy, xbase, lane, out_lane, full_vec, y0, y1, xb, xe, xb1,
            xe1, yb1, ye1, xcfl, ycfl, curr, xl, wt_lo, wt_hi);
    else
        pipen_run<T, ORDER, RB, NS, FMA, true, PD, NT, WPR, VW, LX, NSLOT, OST>(
            ring, edge, k, sub, prev + xl, curr + xl, pitch, gy, xbase, lane, out_lane, full_vec, y0, y1, xb, xe, xb1,
            xe1, yb1, ye1, xcfl, ycfl, curr, xl, wt_lo, wt_hi);
}

// one workgroup (NS roles x WPR waves) per strip-chunk task; regions as for
// streamN. VW = 8: strips start on 8-column boundaries, so every lane's
// columns lie wholly inside or wholly outside the grid (the edge lanes' loads
// are clamped into the row).
template <typename T, int ORDER, int RB, int NS, int FMA, int PD = 1, bool NT = false, int WPR = 1, int VW = 4,
          int OCC = (FMA == 3 ? 4 : 0), bool LX = false>
__global__ __launch_bounds__(NS * WPR * 64, (OCC > 0 ? 4 * OCC / NS : 1)) void heat_pipe_kernel(
    const T* __restrict__ prev, T* __restrict__ curr, int pitch, int gy, S2Regions R, int xb1, int xe1, int yb1,
    int ye1, T xcfl, T ycfl, PipeGate gate) {
    static_assert(NS >= 2 && NS <= 6, "pipe: 2..6 steps per pass");
    constexpr int NSLOT = PipeN<T, ORDER, RB, NS, FMA, false, PD, NT, WPR, VW, LX>::NSLOT;
    __shared__ V4<T> ring[NS - 1][NSLOT][RB][VW / 4][64 * WPR];
    __shared__ V4<T> edge[WPR > 1 ? NS : 1][3][RB][WPR][2];
    const int lane = lane_id();
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
    const int k = wv / WPR, sub = wv % WPR;
    int task = (int)blockIdx.x;
    if (task >= R.wave_end[R.n - 1]) return;  // whole workgroup
    unsigned long long t_start = 0;
    if (gate.trace && threadIdx.x == 0) t_start = wall_clock64();
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
                if (spins >= gate.spins) {
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
    pipe_task<T, ORDER, RB, NS, FMA, PD, NT, WPR, VW, LX, NSLOT>(ring, edge, R, r, task, prev, curr, pitch, gy, xb1, xe1,
                                                             yb1, ye1, xcfl, ycfl, k, sub, lane);
    if (gate.trace) {  // profiling: the whole workgroup's span (vector stores)
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_REG_HW_ID
            const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // HW_REG_XCC_ID
            unsigned long long* t = gate.trace + 3ull * blockIdx.x;
            t[0] = t_start;
            t[1] = wall_clock64();
            t[2] = ((unsigned long long)r << 40) | ((unsigned long long)(xcc & 0xff) << 32) | hw;
        }
    }
}

// Chunk rule for the pipelined pass, in workgroup tasks: a whole number of
// rounds of the device's resident workgroups (every strip cut into the same
// number of chunks, each chunk paying its warm-up rows once). The floor
// keeps a partial second round from forming (16384^2, 74 strips, 1024
// resident: 13 chunks of 1261 rows = 962 tasks, not 14 = 1036). Thin regions
// (border strips) use ~1024 tasks. CME_PIPE_CHUNK / CME_PIPE_PER_CU override
// for sweeps (per_cu = task target per CU).
// `reserve` < 0: take that many tasks off the bulk rule (so that the thin
// regions sharing the launch -- the fused schedule's border strips, last in
// the grid -- fit in the bulk's last round of resident workgroups). Measured
// on one N = 4 / 8 rank (profiles/dist_rank_trace_r4.md): every task then
// starts at once, but the pass got 5 / 2 % SLOWER (the span is set by the
// slowest interior tasks, which got taller), so launch_pipe_multi passes 0.
template <int NS, int RB, int VW = 4>
int pipe_chunk(int strips, int H, int chunk_hint, int per_cu_hint, long resident, bool thin_floor, long reserve = 0) {
    const int env_chunk = (int)cme::tune_get(cme::kTunePipeChunk);
    const int env_per_cu = (int)cme::tune_get(cme::kTunePipePerCU);
    const int thin_min = (int)cme::tune_get(cme::kTunePipeThinMin);
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
            // (wide lanes, 3 workgroups per CU: 8 per CU at >= 8192 rows,
            // ~280-row chunks at 16384; 6 at >= 4096 rows; profiles/
            // heat_pipe_wide_r3.md)
            if (per_cu <= 0) {
                tasks = H >= 8192 ? (VW == 8 ? 8L : 14L) * device_cu_count()
                                  : (H >= 4096 ? (VW == 8 ? 6L : 8L) * device_cu_count() : resident);
                if (reserve < 0) tasks = tasks + reserve < tasks / 2 ? tasks / 2 : tasks + reserve;
            }
            long per_strip = tasks / strips;
            per_strip = per_strip < 1 ? 1 : per_strip;
            rows = (H + per_strip - 1) / per_strip;
            rows = rows < lo ? lo : rows;
        }
        chunk = (int)rows;
    }
    return ((chunk + RB - 1) / RB) * RB;
}

template <typename T, int ORDER, int NS, int FMA, int RB, int PD = 1, bool NT = false, int WPR = 1, int VW = 4,
          int OCC = (FMA == 3 ? 4 : 0), bool LX = false>
int launch_pipe_multi(const T* prev, T* curr, int pitch, int gy, const Region* gs, int n, Region g1, T xcfl, T ycfl,
                      int chunk_hint, int per_cu, hipStream_t s, PipeGate gate = PipeGate{}) {
    if (n < 1 || n > kMaxS2Regions) return (int)hipErrorInvalidValue;
    if ((pitch & 63) != 0) return (int)hipErrorInvalidValue;
    static const long resident = [] {
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, heat_pipe_kernel<T, ORDER, RB, NS, FMA, PD, NT, WPR, VW, OCC, LX>,
                                                         NS * WPR * 64, 0) != hipSuccess || per_cu < 1)
            per_cu = 1;
        return (long)per_cu * device_cu_count();
    }();
    S2Regions R{};
    int tasks = 0;
    const int gate_from = gate.from;
    gate.from = kMaxS2Regions;  // region index in R of the first gated input region
    constexpr int kOut = PipeOut<NS, WPR, VW, HeatOrder<ORDER>::B>::kOut;
    const long reserve = 0;  // see pipe_chunk
    for (int i = 0; i < n; ++i) {
        const Region& g = gs[i];
        const int H = g.ye - g.yb;
        if (i >= gate_from && gate.from == kMaxS2Regions) gate.from = R.n;
        if (H <= 0 || g.xe <= g.xb) continue;
        const int strips = (int)cdiv(g.xe - (g.xb & ~(VW - 1)), kOut);
        int chunk = pipe_chunk<NS, RB, VW>(strips, H, chunk_hint, per_cu, resident, n > 1, reserve);
        int nchunks = (int)cdiv(H, chunk), n1 = 0;
        // taper (pipe_taper): a region of several rounds of resident tasks
        // ends in shorter tasks, so the last round drains sooner (the
        // per-task trace had the N = 1 pass at 84 % slot utilisation,
        // profiles/dist_rank_trace_r4.md). m2 half-height chunks per strip
        // (-1: enough to fill one round of the resident workgroups)
        const long taper = cme::tune_get(cme::kTunePipeTaper);
        if (taper != 0 && chunk_hint <= 0 && (long)strips * nchunks > 2 * resident) {
            const int c1 = ((chunk + 2 * RB - 1) / (2 * RB)) * (2 * RB), c2 = c1 / 2;
            const long m2 = taper > 0 ? taper : cdiv(resident, strips);
            const long full = ((long)H - m2 * c2) / c1;
            if (full >= 1 && c1 < 65536) {
                n1 = (int)full;
                chunk = c1;
                nchunks = n1 + (int)cdiv(H - n1 * c1, c2);
            }
        }
        const int k = R.n++;
        R.xb[k] = g.xb, R.xe[k] = g.xe, R.yb[k] = g.yb, R.ye[k] = g.ye;
        R.strips[k] = strips;
        R.chunk[k] = chunk | (n1 << 16);
        tasks += strips * nchunks;
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
    hipLaunchKernelGGL((heat_pipe_kernel<T, ORDER, RB, NS, FMA, PD, NT, WPR, VW, OCC, LX>), dim3(tasks), dim3(NS * WPR * 64), 0, s,
                       prev, curr, pitch, gy, R, g1.xb, g1.xe, g1.yb, g1.ye, xcfl, ycfl, gate);
    CME_LAUNCH_STATUS();
}
