// Kernel templates and launchers of the 2-D heat family (entry points:
// heat2d.hip production, hip_tune/heat2d_tune.hip tuning arms).
#pragma once
// 2-D heat diffusion (explicit FTCS), orders 2/4/8, fp32/fp64, on gfx950.
//
// Capability parity with the reference's single-GPU hw2 kernels
// (hw/hw2/solution/2dHeat_solution.cu:413-530 global + gpuShared) and the
// distributed hw5 compute loops (hw/hw5/2dHeat_solution.cpp:501-628), which
// are expressed here as one kernel family over an arbitrary compute REGION so
// the same code serves full sweeps, async "interior only" sweeps and the
// border strips computed after the halo exchange.
//
// Device grid layout: rows of `pitch` elements (pitch % 64 == 0, pitch >= gx),
// row y at base + y*pitch; the region [xb,xe) x [yb,ye) is updated from prev.
//
// Three variants (the lecture's optimisation ladder, re-derived for wave64):
//   naive  : 1 thread / point, 64x4 blocks, every neighbour a global load.
//   lds    : 2-D LDS tile (64+2B) x (TY+2B) with +1 padding, 4 waves, each
//            thread marches TY/4 rows (the reference's gpuShared idea).
//   stream : register sliding window. Each wave owns a 248-column strip
//            (62 output lanes + 1 halo lane per side, 4 elements per lane =
//            16 B fp32 / 32 B fp64 accesses) and marches down `chunk` rows,
//            holding the 2B+1 row window in VGPRs. x-neighbours come from the
//            adjacent lanes through DPP wave_shr/wave_shl (no LDS), and the
//            next RB rows are prefetched while the current RB are computed.
//            Each input element is fetched from HBM ~once: 8 B/pt fp32.
#include "cme213/common.h"
#include "cme213/tuning.h"
#include "cme213/heat_region.h"
#include "cme213/heat_stencil.h"
#include "cme213/vec.h"

using namespace cme;

// ---------------------------------------------------------------- naive
template <typename T, int ORDER>
__global__ __launch_bounds__(256) void heat_naive_kernel(const T* __restrict__ prev, T* __restrict__ curr, int pitch,
                                                         int xb, int xe, int yb, int ye, T xcfl, T ycfl) {
    constexpr int B = HeatOrder<ORDER>::B;
    const int x = xb + (int)(blockIdx.x * 64 + threadIdx.x % 64);
    const int y = yb + (int)(blockIdx.y * 4 + threadIdx.x / 64);
    if (x >= xe || y >= ye) return;
    const T* p = prev + (size_t)y * pitch + x;
    T xm[B], xp[B], ym[B], yp[B];
#pragma unroll
    for (int k = 0; k < B; ++k) {
        xm[k] = p[-(k + 1)];
        xp[k] = p[k + 1];
        ym[k] = p[-(ptrdiff_t)(k + 1) * pitch];
        yp[k] = p[(ptrdiff_t)(k + 1) * pitch];
    }
    curr[(size_t)y * pitch + x] = heat_update<ORDER>(p[0], xm, xp, ym, yp, xcfl, ycfl);
}

// ---------------------------------------------------------------- lds tile
// Block: 256 threads = 64 columns x 4 row-groups; tile TX=64 x TY rows.
template <typename T, int ORDER, int TY, int PAD>
__global__ __launch_bounds__(256) void heat_lds_kernel(const T* __restrict__ prev, T* __restrict__ curr, int pitch,
                                                       int gy, int xb, int xe, int yb, int ye, T xcfl, T ycfl) {
    constexpr int B = HeatOrder<ORDER>::B;
    constexpr int TX = 64;
    constexpr int LW = TX + 2 * B + PAD;  // LDS row length (PAD breaks the power-of-2 stride)
    constexpr int LH = TY + 2 * B;
    __shared__ T tile[LH * LW];
    const int tx = threadIdx.x % 64, ty = threadIdx.x / 64;
    const int x0 = xb + (int)blockIdx.x * TX;
    const int y0 = yb + (int)blockIdx.y * TY;
    // Cooperative load of the haloed tile (rows/cols outside the allocation are
    // clamped; they only feed points outside the region).
    for (int i = threadIdx.x; i < LH * (TX + 2 * B); i += 256) {
        const int r = i / (TX + 2 * B), c = i % (TX + 2 * B);
        int gyy = y0 - B + r;
        int gxx = x0 - B + c;
        gyy = gyy < 0 ? 0 : (gyy >= gy ? gy - 1 : gyy);
        gxx = gxx < 0 ? 0 : (gxx >= pitch ? pitch - 1 : gxx);
        tile[r * LW + c] = prev[(size_t)gyy * pitch + gxx];
    }
    __syncthreads();
    const int x = x0 + tx;
    if (x >= xe) return;
#pragma unroll 4
    for (int r = ty; r < TY; r += 4) {
        const int y = y0 + r;
        if (y >= ye) break;
        const T* t = &tile[(r + B) * LW + tx + B];
        T xm[B], xp[B], ym[B], yp[B];
#pragma unroll
        for (int k = 0; k < B; ++k) {
            xm[k] = t[-(k + 1)];
            xp[k] = t[k + 1];
            ym[k] = t[-(k + 1) * LW];
            yp[k] = t[(k + 1) * LW];
        }
        curr[(size_t)y * pitch + x] = heat_update<ORDER>(t[0], xm, xp, ym, yp, xcfl, ycfl);
    }
}

// ---------------------------------------------------------------- stream
constexpr int kStripOut = 62 * 4;  // output columns per wave strip

template <typename T, int ORDER, int RB, int WPB = 4, bool NT = false, bool FMA = false>
__global__ __launch_bounds__(WPB * 64) void heat_stream_kernel(const T* __restrict__ prev, T* __restrict__ curr, int pitch,
                                                          int gy, int xb, int xe, int yb, int ye, int strips, int chunk,
                                                          int total_waves, T xcfl, T ycfl) {
    constexpr int B = HeatOrder<ORDER>::B;
    constexpr int NW = RB + 2 * B;  // rows held in the window
    const int lane = lane_id();
    const int wave = (int)blockIdx.x * WPB + (int)(threadIdx.x / 64);
    if (wave >= total_waves) return;
    const int strip = wave % strips;
    const int ck = wave / strips;
    const int y0 = yb + ck * chunk;
    const int y1 = min(ye, y0 + chunk);
    const int xs = (xb & ~3) + strip * kStripOut;
    const int xbase = xs - 4 + 4 * lane;
    const int xl = min(max(xbase, 0), pitch - 4);
    const bool out_lane = (lane >= 1) && (lane <= 62) && (xbase < xe) && (xbase + 4 > xb);
    const bool full_vec = (xbase >= xb) && (xbase + 4 <= xe);
    const T* src = prev + xl;
    T* dst = curr + xl;

    auto row_ptr = [&](int r) -> const T* {
        r = r < 0 ? 0 : (r >= gy ? gy - 1 : r);
        return src + (size_t)r * pitch;
    };

    V4<T> win[NW];
    V4<T> nxt[RB];
#pragma unroll
    for (int i = 0; i < 2 * B; ++i) win[i] = load4(row_ptr(y0 - B + i));
#pragma unroll
    for (int i = 0; i < RB; ++i) nxt[i] = load4(row_ptr(y0 + B + i));

    for (int y = y0; y < y1; y += RB) {
#pragma unroll
        for (int i = 0; i < RB; ++i) win[2 * B + i] = nxt[i];
        // unconditional prefetch (row_ptr clamps): a guarded one compiles to a
        // phi whose register copies wait on the loads just issued
#pragma unroll
        for (int i = 0; i < RB; ++i) nxt[i] = load4(row_ptr(y + RB + B + i));
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            const V4<T> c = win[r + B];
            const V4<T> L = wave_shr1(c);  // lane-1's 4 columns
            const V4<T> R = wave_shl1(c);  // lane+1's 4 columns
            T row[12];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                row[j] = L[j];
                row[4 + j] = c[j];
                row[8 + j] = R[j];
            }
            V4<T> o;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                T xm[B], xp[B], ym[B], yp[B];
#pragma unroll
                for (int k = 0; k < B; ++k) {
                    xm[k] = row[4 + j - (k + 1)];
                    xp[k] = row[4 + j + (k + 1)];
                    ym[k] = win[r + B - (k + 1)][j];
                    yp[k] = win[r + B + (k + 1)][j];
                }
                o[j] = heat_update_sel<ORDER, FMA>(c[j], xm, xp, ym, yp, xcfl, ycfl);
            }
            const int yy = y + r;
            if (out_lane && yy < y1) {
                T* d = dst + (size_t)yy * pitch;
                if (full_vec) {
                    if constexpr (NT && sizeof(T) == 4) {
                        typedef float f32x4 __attribute__((ext_vector_type(4)));
                        f32x4 ov = {o[0], o[1], o[2], o[3]};
                        __builtin_nontemporal_store(ov, reinterpret_cast<f32x4*>(d));
                    } else {
                        store4(d, o);
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (xbase + j >= xb && xbase + j < xe) d[j] = o[j];
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 2 * B; ++i) win[i] = win[RB + i];
    }
}


// ---------------------------------------------------------------- stream2
// Temporal blocking: TWO timesteps per pass over HBM. The wave keeps an input
// row window AND a window of step-1 rows in VGPRs; step-1 rows are produced
// on lanes 1..62 (x-neighbours through DPP), step-2 rows on lanes 2..61
// (4 x 60 = 240 output columns per strip). Cells outside the step-1 region
// keep their input value in the intermediate state (fixed boundary cells), so
// the result is bitwise identical to two single steps.
//
// Instruction diet (the kernel is VALU-bound once two steps share a pass):
//  * both windows are rings indexed by compile-time slots; the main loop is
//    unrolled over P = NW / gcd(NW, RB) phases, so advancing the window costs
//    no register moves;
//  * waves whose step-1 cells all lie inside the region skip the per-cell
//    region select (wave-uniform branch into a CHECK=false instance); the
//    step-2 value needs no select at all since only in-region cells are
//    stored;
//  * FMA=true evaluates the FMA-contracted stencil (heat_update_fma).
constexpr int kStrip2Out = 60 * 4;


template <typename T, int ORDER, int RB, bool FMA, bool CHECK>
struct Stream2 {
    static constexpr int B = HeatOrder<ORDER>::B;
    static constexpr int NW = RB + 2 * B;           // rows per window
    static constexpr int P = NW / cgcd(NW, RB);     // phases until the ring realigns

    V4<T> in[NW];   // input rows; logical j = row r0 - B + j
    V4<T> s1[NW];   // step-1 rows; logical j = row r0 - 2B + j
    V4<T> nxt[RB];  // prefetched input rows
    const T* src;
    T* dst;
    int pitch, gy, xbase;
    bool out_lane, full_vec;
    int y0, y1, xb, xe, xb1, xe1, yb1, ye1;
    T xcfl, ycfl;
    int r0;

    __device__ __forceinline__ const T* row_ptr(int r) const {
        r = r < 0 ? 0 : (r >= gy ? gy - 1 : r);
        return src + (size_t)r * pitch;
    }

    // FTCS update of this lane's 4 columns for the row centred on ring slot
    // (s_lo + B) % NW of window w.
    template <bool MASK>
    __device__ __forceinline__ V4<T> upd(const V4<T> (&w)[NW], int s_lo, int row) const {
        const V4<T> c = w[(s_lo + B) % NW];
        const V4<T> L = wave_shr1(c);
        const V4<T> R = wave_shl1(c);
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
            const T u = heat_update_sel<ORDER, FMA>(c[j], xm, xp, ym, yp, xcfl, ycfl);
            if constexpr (MASK) {
                const int x = xbase + j;
                o[j] = (row_in && x >= xb1 && x < xe1) ? u : c[j];
            } else {
                o[j] = u;
            }
        }
        return o;
    }

    template <int PH>
    __device__ __forceinline__ bool phase() {
        if (r0 - B >= y1) return false;
        constexpr int S = (PH * RB) % NW;  // ring slot of logical row 0
#pragma unroll
        for (int i = 0; i < RB; ++i) in[(S + 2 * B + i) % NW] = nxt[i];
#pragma unroll
        for (int i = 0; i < RB; ++i) nxt[i] = load4(row_ptr(r0 + RB + B + i));  // unguarded, as above
#pragma unroll
        for (int i = 0; i < RB; ++i) s1[(S + 2 * B + i) % NW] = upd<CHECK>(in, (S + i) % NW, r0 + i);
#pragma unroll
        for (int i = 0; i < RB; ++i) {
            const int y = r0 - B + i;
            // wave-uniform: the first 2B step-2 rows of a chunk are warm-up
            // (their step-1 window is incomplete) -- skip their arithmetic
            if (y >= y0 && y < y1) {
                const V4<T> o = upd<false>(s1, (S + i) % NW, y);
                T* d = dst + (size_t)y * pitch;
                if constexpr (!CHECK) {
                    // interior strip: every output lane holds 4 in-region cells
                    if (out_lane) store4(d, o);
                } else if (out_lane) {
                    if (full_vec) {
                        store4(d, o);
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if (xbase + j >= xb && xbase + j < xe) d[j] = o[j];
                    }
                }
            }
        }
        r0 += RB;
        if constexpr (PH + 1 < P)
            return phase<PH + 1>();
        else
            return true;
    }

    __device__ __forceinline__ void run() {
        r0 = y0 - B;
#pragma unroll
        for (int i = 0; i < 2 * B; ++i) in[i] = load4(row_ptr(r0 - B + i));
#pragma unroll
        for (int i = 0; i < RB; ++i) nxt[i] = load4(row_ptr(r0 + B + i));
        while (phase<0>()) {
        }
    }
};

template <typename T, int ORDER, int RB, bool FMA, bool CHECK>
__device__ __forceinline__ void stream2_run(const T* src, T* dst, int pitch, int gy, int xbase, bool out_lane,
                                            bool full_vec, int y0, int y1, int xb, int xe, int xb1, int xe1, int yb1,
                                            int ye1, T xcfl, T ycfl) {
    Stream2<T, ORDER, RB, FMA, CHECK> st;
    st.src = src;
    st.dst = dst;
    st.pitch = pitch;
    st.gy = gy;
    st.xbase = xbase;
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
    st.run();
}


template <typename T, int ORDER, int RB, bool FMA, int WPE = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void heat_stream2_kernel(
    const T* __restrict__ prev, T* __restrict__ curr, int pitch, int gy, S2Regions R, int xb1, int xe1, int yb1,
    int ye1, T xcfl, T ycfl) {
    constexpr int B = HeatOrder<ORDER>::B;
    const int lane = lane_id();
    int wave = (int)blockIdx.x * 4 + (int)(threadIdx.x / 64);
    if (wave >= R.wave_end[R.n - 1]) return;
    int r = 0;
    while (wave >= R.wave_end[r]) ++r;  // wave-uniform, <= 3 steps
    if (r > 0) wave -= R.wave_end[r - 1];
    const int xb = R.xb[r], xe = R.xe[r], yb = R.yb[r], ye = R.ye[r];
    const int strips = R.strips[r], chunk = R.chunk[r];
    const int strip = wave % strips;
    const int ck = wave / strips;
    const int y0 = yb + ck * chunk;
    const int y1 = min(ye, y0 + chunk);
    const int xs = (xb & ~3) + strip * kStrip2Out;
    const int xbase = xs - 8 + 4 * lane;
    const int xl = min(max(xbase, 0), pitch - 4);
    const bool out_lane = (lane >= 2) && (lane <= 61) && (xbase < xe) && (xbase + 4 > xb);
    const bool full_vec = (xbase >= xb) && (xbase + 4 <= xe);
    // step-1 cells that matter: columns xs-4 .. xs+243 (lanes 1..62), rows
    // y0-B .. y1+B-1; all inside the step-1 region -> no per-cell select; and
    // output columns xs .. xs+239 all inside [xb, xe) -> plain vector stores
    const bool inside = (xs - 4 >= xb1) && (xs + 244 <= xe1) && (y0 - B >= yb1) && (y1 + B <= ye1) &&
                        (xs >= xb) && (xs + kStrip2Out <= xe);
    if (inside)
        stream2_run<T, ORDER, RB, FMA, false>(prev + xl, curr + xl, pitch, gy, xbase, out_lane, full_vec, y0, y1, xb,
                                              xe, xb1, xe1, yb1, ye1, xcfl, ycfl);
    else
        stream2_run<T, ORDER, RB, FMA, true>(prev + xl, curr + xl, pitch, gy, xbase, out_lane, full_vec, y0, y1, xb,
                                             xe, xb1, xe1, yb1, ye1, xcfl, ycfl);
}

// ---------------------------------------------------------------- streamN
// Deeper temporal blocking: NS (3 or 4) timesteps per HBM pass, the stream2
// design generalised. The two-step kernel moves 4 B/pt/step and runs at
// ~4.4 TB/s on 16384^2, short of loads in flight rather than of VALU issue,
// so the lever is fewer HBM bytes per timestep: NS steps per pass move
// 8/NS B/pt.
//
// Window k (0 = input, k = 1..NS-1 = step-k rows) holds NW = RB + 2B rows in a
// ring; logical slot j of window k is row r0 - (k+1)B + j. A phase loads RB
// new input rows, produces RB rows of every step k from window k-1 (rows
// r0 - (k-1)B + i) and stores RB final rows (y = r0 - (NS-1)B + i). Step k is
// valid on lanes k..63-k (x-neighbours arrive through DPP), so a strip emits
// (64 - 2NS) x 4 columns. Rows of step k outside [y0 - (NS-k)B, y1 +
// (NS-k)B) feed no stored value: their arithmetic is skipped (wave-uniform).
// Intermediate cells outside the `ext` region keep their input value (fixed
// boundary cells), so the result equals NS single steps bit for bit.

template <typename T, int ORDER, int RB, int NS, bool FMA, bool CHECK, int PD = 1, bool NT = false>
struct StreamN {
    static constexpr int B = HeatOrder<ORDER>::B;
    static constexpr int NW = RB + 2 * B;
    static constexpr int P = NW / cgcd(NW, RB);  // phases until the window rings realign
    static constexpr int Q = P * PD / cgcd(P, PD);  // ... and the PD prefetch buffers

    V4<T> w[NS][NW];
    V4<T> nxt[PD][RB];  // input rows of the next PD phases, in flight
    const T* src;
    T* dst;
    int pitch, gy, xbase;
    bool out_lane, full_vec;
    int y0, y1, xb, xe, xb1, xe1, yb1, ye1;
    T xcfl, ycfl;
    int r0;

    __device__ __forceinline__ const T* row_ptr(int r) const {
        r = r < 0 ? 0 : (r >= gy ? gy - 1 : r);
        return src + (size_t)r * pitch;
    }

    template <bool MASK>
    __device__ __forceinline__ V4<T> upd(const V4<T> (&win)[NW], int s_lo, int row) const {
        const V4<T> c = win[(s_lo + B) % NW];
        const V4<T> L = wave_shr1(c);
        const V4<T> R = wave_shl1(c);
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
                ym[k] = win[(s_lo + B - (k + 1)) % NW][j];
                yp[k] = win[(s_lo + B + (k + 1)) % NW][j];
            }
            const T u = heat_update_sel<ORDER, FMA>(c[j], xm, xp, ym, yp, xcfl, ycfl);
            if constexpr (MASK) {
                const int x = xbase + j;
                o[j] = (row_in && x >= xb1 && x < xe1) ? u : c[j];
            } else {
                o[j] = u;
            }
        }
        return o;
    }

    // the RB rows of intermediate step K produced in this phase
    template <int K, int S>
    __device__ __forceinline__ void inter() {
        if constexpr (K < NS) {
#pragma unroll
            for (int i = 0; i < RB; ++i) {
                const int row = r0 - (K - 1) * B + i;
                if (row >= y0 - (NS - K) * B && row < y1 + (NS - K) * B)
                    w[K][(S + 2 * B + i) % NW] = upd<CHECK>(w[K - 1], (S + i) % NW, row);
            }
            inter<K + 1, S>();
        }
    }

    template <int PH>
    __device__ __forceinline__ bool phase() {
        if (r0 - (NS - 1) * B >= y1) return false;
        constexpr int S = (PH * RB) % NW;
        constexpr int F = PH % PD;
#pragma unroll
        for (int i = 0; i < RB; ++i) w[0][(S + 2 * B + i) % NW] = nxt[F][i];
#pragma unroll
        for (int i = 0; i < RB; ++i) nxt[F][i] = load4(row_ptr(r0 + PD * RB + B + i));  // unguarded, as above
        inter<1, S>();
#pragma unroll
        for (int i = 0; i < RB; ++i) {
            const int y = r0 - (NS - 1) * B + i;
            if (y >= y0 && y < y1) {
                const V4<T> o = upd<false>(w[NS - 1], (S + i) % NW, y);
                T* d = dst + (size_t)y * pitch;
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
        if constexpr (PH + 1 < Q)
            return phase<PH + 1>();
        else
            return true;
    }

    // NT: the output rows are streamed past the caches (non-temporal)
    __device__ __forceinline__ void store_out(T* d, const V4<T>& o) const {
        if constexpr (NT && sizeof(T) == 4) {
            typedef float f32x4 __attribute__((ext_vector_type(4)));
            const f32x4 ov = {o[0], o[1], o[2], o[3]};
            __builtin_nontemporal_store(ov, reinterpret_cast<f32x4*>(d));
        } else {
            store4(d, o);
        }
    }

    __device__ __forceinline__ void run() {
        r0 = y0 - (NS - 1) * B;
#pragma unroll
        for (int i = 0; i < 2 * B; ++i) w[0][i] = load4(row_ptr(r0 - B + i));
#pragma unroll
        for (int f = 0; f < PD; ++f)
#pragma unroll
            for (int i = 0; i < RB; ++i) nxt[f][i] = load4(row_ptr(r0 + f * RB + B + i));
        while (phase<0>()) {
        }
    }
};

template <typename T, int ORDER, int RB, int NS, bool FMA, bool CHECK, int PD, bool NT = false>
__device__ __forceinline__ void streamn_run(const T* src, T* dst, int pitch, int gy, int xbase, bool out_lane,
                                            bool full_vec, int y0, int y1, int xb, int xe, int xb1, int xe1, int yb1,
                                            int ye1, T xcfl, T ycfl) {
    StreamN<T, ORDER, RB, NS, FMA, CHECK, PD, NT> st;
    st.src = src;
    st.dst = dst;
    st.pitch = pitch;
    st.gy = gy;
    st.xbase = xbase;
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
    st.run();
}

template <typename T, int ORDER, int RB, int NS, bool FMA, int WPE = 1, int PD = 1, bool NT = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void heat_streamn_kernel(
    const T* __restrict__ prev, T* __restrict__ curr, int pitch, int gy, S2Regions R, int xb1, int xe1, int yb1,
    int ye1, T xcfl, T ycfl) {
    constexpr int B = HeatOrder<ORDER>::B;
    constexpr int OUT = StripN<NS>::kOut;
    const int lane = lane_id();
    int wave = (int)blockIdx.x * 4 + (int)(threadIdx.x / 64);
    if (wave >= R.wave_end[R.n - 1]) return;
    int r = 0;
    while (wave >= R.wave_end[r]) ++r;  // wave-uniform, <= 3 steps
    if (r > 0) wave -= R.wave_end[r - 1];
    const int xb = R.xb[r], xe = R.xe[r], yb = R.yb[r], ye = R.ye[r];
    const int strips = R.strips[r], chunk = R.chunk[r];
    const int strip = wave % strips;
    const int ck = wave / strips;
    const int y0 = yb + ck * chunk;
    const int y1 = min(ye, y0 + chunk);
    const int xs = (xb & ~3) + strip * OUT;
    const int xbase = xs - 4 * NS + 4 * lane;
    const int xl = min(max(xbase, 0), pitch - 4);
    const bool out_lane = (lane >= NS) && (lane <= 63 - NS) && (xbase < xe) && (xbase + 4 > xb);
    const bool full_vec = (xbase >= xb) && (xbase + 4 <= xe);
    // every intermediate cell that feeds a stored value lies inside ext, and
    // every output column inside [xb, xe): no per-cell selects
    constexpr int reach = 4 * (NS - 1);
    const bool inside = (xs - reach >= xb1) && (xs + OUT + reach <= xe1) && (y0 - (NS - 1) * B >= yb1) &&
                        (y1 + (NS - 1) * B <= ye1) && (xs >= xb) && (xs + OUT <= xe);
    if (inside)
        streamn_run<T, ORDER, RB, NS, FMA, false, PD, NT>(prev + xl, curr + xl, pitch, gy, xbase, out_lane, full_vec,
                                                          y0, y1, xb, xe, xb1, xe1, yb1, ye1, xcfl, ycfl);
    else
        streamn_run<T, ORDER, RB, NS, FMA, true, PD, NT>(prev + xl, curr + xl, pitch, gy, xbase, out_lane, full_vec,
                                                         y0, y1, xb, xe, xb1, xe1, yb1, ye1, xcfl, ycfl);
}

// ---------------------------------------------------------------- launchers

// Two-step pass: output region `g`; step-1 (intermediate) region `g1` must
// contain g and may extend at most B cells beyond it (into a 2B-deep halo,
// for the distributed loop); cells outside g1 keep their input value.
// Defaults from benchmarks/tune_heat2.py (16384^2, order 8; profiles/
// heat_stream2_tune.md): rows per block RB and a target wave count that sets
// the row chunk (more, shorter chunks win for the lighter FMA kernel).
template <typename T, bool FMA, int RB>
int stream2_chunk(int strips, int H, int chunk_hint) {
    const int env_chunk = (int)cme::tune_get(cme::kTuneStream2Chunk);  // tuning experiments only
    int chunk = chunk_hint > 0 ? chunk_hint : env_chunk;
    if (chunk <= 0) {
        const long target_waves = 256L * (sizeof(T) == 4 ? (FMA ? 128 : 48) : 24);
        long rows = ((long)strips * H + target_waves - 1) / target_waves;
        const long lo = 4 * RB > 16 ? 4 * RB : 16;
        if ((long)strips * cdiv(H, lo) < 1024) {
            // thin region (a distributed border strip, on the critical path
            // after each halo exchange): latency-bound, so trade redundant
            // halo rows for parallelism -- about 1024 waves, >= RB rows each
            rows = ((long)strips * H + 1023) / 1024;
            rows = rows < RB ? RB : rows;
        } else {
            rows = rows < lo ? lo : rows;
        }
        rows = rows > 512 ? 512 : rows;
        chunk = (int)rows;
    }
    return ((chunk + RB - 1) / RB) * RB;
}

// Two-step pass over `n` output regions `gs` (<= 4, one launch); step-1
// region `g1` must contain them and extend at most B cells beyond.
template <typename T, int ORDER, bool FMA, int RB = (sizeof(T) == 4 ? (FMA ? 2 : 4) : (FMA ? 4 : 2)), int WPE = 1>
int launch_stream2_multi(const T* prev, T* curr, int pitch, int gy, const Region* gs, int n, Region g1, T xcfl,
                         T ycfl, int chunk_hint, hipStream_t s) {
    if (n < 1 || n > kMaxS2Regions) return (int)hipErrorInvalidValue;
    if ((pitch & 63) != 0) return (int)hipErrorInvalidValue;
    S2Regions R{};
    int waves = 0;
    for (int i = 0; i < n; ++i) {
        const Region& g = gs[i];
        const int H = g.ye - g.yb;
        if (H <= 0 || g.xe <= g.xb) continue;  // empty region: no waves
        const int strips = (int)cdiv(g.xe - (g.xb & ~3), kStrip2Out);
        const int chunk = stream2_chunk<T, FMA, RB>(strips, H, chunk_hint);
        const int k = R.n++;
        R.xb[k] = g.xb, R.xe[k] = g.xe, R.yb[k] = g.yb, R.ye[k] = g.ye;
        R.strips[k] = strips;
        R.chunk[k] = chunk;
        waves += strips * (int)cdiv(H, chunk);
        R.wave_end[k] = waves;
    }
    if (R.n == 0) return 0;
    hipLaunchKernelGGL((heat_stream2_kernel<T, ORDER, RB, FMA, WPE>), dim3(cdiv(waves, 4)), dim3(256), 0, s, prev,
                       curr, pitch, gy, R, g1.xb, g1.xe, g1.yb, g1.ye, xcfl, ycfl);
    CME_LAUNCH_STATUS();
}

// NS-step pass (NS = 3, 4; fp32): rows per block and chunk heights from
// benchmarks/tune_heatn.py (profiles/heat_streamn_tune.md: at 16384^2 NS=3
// RB=4 ~190-row chunks 0.178 ms/step, NS=4 RB=2 0.195, stream2 0.237).
//
// Chunk rule, in units of the device's RESIDENT wave capacity `cap` (2 waves
// per SIMD for NS=3 RB=4): aim for 3 full rounds of waves (16384^2: 71 strips
// x 86 chunks of ~190 rows); when that makes chunks shorter than `min_chunk`
// rows -- a strong-scaled subdomain, where every chunk re-computes 2(NS-1)B
// warm-up rows and re-reads 2NS*B input rows -- use fewer whole rounds (2,
// then 1) with longer chunks instead of more, shorter ones. A whole number of
// rounds keeps the tail short. CME_STREAMN_CHUNK / _ROUNDS / _MINCHUNK
// override for experiments (benchmarks/tune_dist_rank.py). Thin regions
// (border strips: latency-bound, on the critical path after an exchange) use
// about 1024 waves.
template <int NS, int RB>
int streamn_chunk(int strips, int H, int chunk_hint, long cap) {
    const int env_chunk = (int)cme::tune_get(cme::kTuneStreamNChunk);
    const int env_rounds = (int)cme::tune_get(cme::kTuneStreamNRounds);
    const int env_min = (int)cme::tune_get(cme::kTuneStreamNMinChunk);
    const long thin_waves = cme::tune_get(cme::kTuneStreamNThinWaves) > 0 ? cme::tune_get(cme::kTuneStreamNThinWaves)
                                                                          : 1024L;
    // share of the resident waves a bulk region may take
    const int cap_pct = cme::tune_get(cme::kTuneStreamNCapPct) > 0 ? (int)cme::tune_get(cme::kTuneStreamNCapPct) : 100;
    cap = cap * cap_pct / 100;
    int chunk = chunk_hint > 0 ? chunk_hint : env_chunk;
    if (chunk <= 0) {
        const long lo = 8 * RB > 32 ? 8 * RB : 32;
        long rows;
        if ((long)strips * cdiv(H, lo) < 1024) {
            rows = ((long)strips * H + thin_waves - 1) / thin_waves;
            rows = rows < RB ? RB : rows;
        } else {
            const int max_rounds = env_rounds > 0 ? env_rounds : 3;
            const long min_chunk = env_min > 0 ? env_min : 64;
            rows = 0;
            for (int r = max_rounds; r >= 1; --r) {
                long per_strip = r * cap / strips;
                per_strip = per_strip < 1 ? 1 : per_strip;
                rows = (H + per_strip - 1) / per_strip;
                if (rows >= min_chunk) break;
            }
            rows = rows < lo ? lo : rows;
        }
        rows = rows > 1024 ? 1024 : rows;
        chunk = (int)rows;
    }
    return ((chunk + RB - 1) / RB) * RB;
}

// NT (non-temporal output stores) defaults to on for NS = 4: benchmarks/
// tune_heatn.py at 16384^2 (profiles/heat_streamn_nt_r2.log): NS=4 RB=2
// 0.1833 vs 0.1922 ms/step; NS=3 RB=4 loses with it (0.1827 vs 0.179).
template <typename T, int ORDER, int NS, bool FMA, int RB = (NS == 3 ? 4 : 2), int WPE = 1, int PD = 1,
          bool NT = (NS == 4)>
int launch_streamn_multi(const T* prev, T* curr, int pitch, int gy, const Region* gs, int n, Region g1, T xcfl,
                         T ycfl, int chunk_hint, hipStream_t s) {
    static_assert(NS >= 3 && NS <= 4, "streamN: 3 or 4 steps per pass");
    if (n < 1 || n > kMaxS2Regions) return (int)hipErrorInvalidValue;
    if ((pitch & 63) != 0) return (int)hipErrorInvalidValue;
    static const long cap = resident_waves(heat_streamn_kernel<T, ORDER, RB, NS, FMA, WPE, PD, NT>, 256);
    S2Regions R{};
    int waves = 0;
    for (int i = 0; i < n; ++i) {
        const Region& g = gs[i];
        const int H = g.ye - g.yb;
        if (H <= 0 || g.xe <= g.xb) continue;
        const int strips = (int)cdiv(g.xe - (g.xb & ~3), StripN<NS>::kOut);
        const int chunk = streamn_chunk<NS, RB>(strips, H, chunk_hint, cap);
        const int k = R.n++;
        R.xb[k] = g.xb, R.xe[k] = g.xe, R.yb[k] = g.yb, R.ye[k] = g.ye;
        R.strips[k] = strips;
        R.chunk[k] = chunk;
        waves += strips * (int)cdiv(H, chunk);
        R.wave_end[k] = waves;
    }
    if (R.n == 0) return 0;
    hipLaunchKernelGGL((heat_streamn_kernel<T, ORDER, RB, NS, FMA, WPE, PD, NT>), dim3(cdiv(waves, 4)), dim3(256), 0, s, prev,
                       curr, pitch, gy, R, g1.xb, g1.xe, g1.yb, g1.ye, xcfl, ycfl);
    CME_LAUNCH_STATUS();
}

template <typename T, int ORDER, bool FMA, int RB = (sizeof(T) == 4 ? (FMA ? 2 : 4) : (FMA ? 4 : 2)), int WPE = 1>
int launch_stream2(const T* prev, T* curr, int pitch, int gy, Region g, Region g1, T xcfl, T ycfl, int chunk_hint,
                   hipStream_t s) {
    return launch_stream2_multi<T, ORDER, FMA, RB, WPE>(prev, curr, pitch, gy, &g, 1, g1, xcfl, ycfl, chunk_hint, s);
}
