// LDS-resident tile pass (see heat_tile.hip for the design notes).
#pragma once

#include "cme213/common.h"
#include "cme213/heat_region.h"
#include "cme213/heat_stencil.h"

namespace cme_tile {

using namespace cme;

template <typename T>
struct alignas(2 * sizeof(T)) Pair {
    T v[2];
};

template <typename T, int ORDER, int NS, int TX, int TY>
struct TileGeom {
    static constexpr int B = HeatOrder<ORDER>::B;
    static constexpr int H = NS * B;
    static constexpr int LW = TX + 2 * H;  // LDS row: TX + 2H values (TX, H even for B >= 2)
    static constexpr int PW = LW + (LW & 1);
    static constexpr int LH = TY + 2 * H;
    static constexpr size_t kBytes = 2ull * LH * PW * sizeof(T);
    static_assert(TX % 2 == 0, "column pairs");
};

// One thread's share of a timestep: the column pair c0, c0 + 1 (w0 / w1:
// which of the two lies inside the step's region) over rows [rb, re) of the
// LDS tile, from src into dst.
template <typename T, int ORDER, bool FMA, int PW>
__device__ __forceinline__ void tile_band(const T* __restrict__ src, T* __restrict__ dst, int c0, int rb, int re,
                                          bool w0, bool w1, T xcfl, T ycfl) {
    constexpr int B = HeatOrder<ORDER>::B;
    constexpr int RING = 2 * B + 2;
    constexpr int NXP = (B + 1) / 2;  // x-neighbour pairs on each side
    const Pair<T>* s2 = reinterpret_cast<const Pair<T>*>(src);
    Pair<T>* d2 = reinterpret_cast<Pair<T>*>(dst);
    const int cp = c0 >> 1;  // pair column
    // Register ring of RING = 2B + 2 row pairs (one more than the
    // stencil's 2B + 1): row x sits in slot (x - (rb - B)) % RING, and
    // row r + 1 + B is loaded into the free slot while row r computes;
    // the x-neighbour pairs are double-buffered by row parity. The row
    // loop is unrolled by RING (even), so every slot index is a
    // compile-time constant: no register moves. LDS addresses are one
    // row pointer plus immediate offsets.
    constexpr int P = PW / 2;  // pairs per LDS row
    Pair<T> win[RING];
    Pair<T> xl[2][NXP], xr[2][NXP];
    {
        const Pair<T>* rp = s2 + (rb - B) * P + cp;
#pragma unroll
        for (int k = 0; k <= 2 * B; ++k) win[k] = rp[k * P];
        rp += B * P;  // row rb
#pragma unroll
        for (int q = 0; q < NXP; ++q) {
            xl[0][q] = rp[-1 - q];  // columns c0-2-2q, c0-1-2q
            xr[0][q] = rp[1 + q];   // columns c0+2+2q, c0+3+2q
        }
    }
    for (int r0 = rb; r0 < re; r0 += RING) {
        // one base address per RING rows: every load below is base +
        // a compile-time (non-negative) offset
        const Pair<T>* base = s2 + (r0 + 1) * P + cp - NXP;
        Pair<T>* dbase = d2 + r0 * P + cp;
        // row guards against one count (u < rem): row u's prefetch guard
        // is row u + 1's compute guard, one compare per row, no row index
        const int rem = re - r0;
#pragma unroll
        for (int u = 0; u < RING; ++u) {
            if (u < rem) {
                if (u + 1 < rem) {  // prefetch row r + 1: its x pairs, and row r + 1 + B into the free slot
                    const Pair<T>* rp = base + u * P;  // pair column c0 / 2 - NXP of row r + 1
                    win[(u + 1 + 2 * B) % RING] = rp[B * P + NXP];
#pragma unroll
                    for (int q = 0; q < NXP; ++q) {
                        xl[(u + 1) & 1][q] = rp[NXP - 1 - q];
                        xr[(u + 1) & 1][q] = rp[NXP + 1 + q];
                    }
                }
                const Pair<T>(&XL)[NXP] = xl[u & 1];
                const Pair<T>(&XR)[NXP] = xr[u & 1];
                const Pair<T> c = win[(u + B) % RING];
                T out[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    T xm[B], xp[B], ym[B], yp[B];
#pragma unroll
                    for (int k = 0; k < B; ++k) {
                        // x of column c0 + j - (k + 1) and c0 + j + (k + 1)
                        const int dm = j - (k + 1), dp = j + (k + 1);  // offsets from c0
                        xm[k] = dm >= 0 ? c.v[dm] : XL[(-dm - 1) / 2].v[1 - ((-dm - 1) & 1)];
                        xp[k] = dp <= 1 ? c.v[dp] : XR[(dp - 2) / 2].v[(dp - 2) & 1];
                        ym[k] = win[(u + B - (k + 1) + RING) % RING].v[j];
                        yp[k] = win[(u + B + (k + 1)) % RING].v[j];
                    }
                    out[j] = heat_update_sel<ORDER, FMA>(c.v[j], xm, xp, ym, yp, xcfl, ycfl);
                }
                if (w0 && w1) {
                    Pair<T> o;
                    o.v[0] = out[0];
                    o.v[1] = out[1];
                    dbase[u * P] = o;
                } else {
                    const int r = r0 + u;
                    if (w0) dst[r * PW + c0] = out[0];
                    if (w1) dst[r * PW + c0 + 1] = out[1];
                }
            }
        }
    }
}

// How a step's region is dealt to the threads: column pairs from ca,
// npairs of them, nb row bands of R rows (nb * npairs <= NT).
struct BandPlan {
    int ca, npairs, nb, R;
    float inv_np;  // ~1 / npairs (the band index, tile_step)
};

// The plan of region [c_lo, c_hi) x [r_lo, r_hi) (non-empty). With constant
// arguments (a whole interior tile, every step after unrolling) it folds to
// constants; the integer divisions then cost nothing -- they were ~60 of the
// ~100 VALU instructions of a wave's per-step setup (profiles/heat_tile_r5.md).
template <int NT>
__device__ __forceinline__ BandPlan band_plan(int c_lo, int c_hi, int r_lo, int r_hi) {
    BandPlan p;
    p.ca = c_lo & ~1;
    p.npairs = (c_hi - p.ca + 1) >> 1;
    p.nb = NT / p.npairs;
    p.nb = p.nb < 1 ? 1 : p.nb;
    p.R = (r_hi - r_lo + p.nb - 1) / p.nb;
    p.inv_np = __builtin_amdgcn_rcpf((float)p.npairs);
    return p;
}

// One timestep of the tile: rows [r_lo, r_hi) x columns [c_lo, c_hi) (LDS
// coordinates) from src into dst, dealt to the threads by plan `pl`.
template <typename T, int ORDER, bool FMA, int PW, int NT>
__device__ __forceinline__ void tile_step(const T* __restrict__ src, T* __restrict__ dst, int c_lo, int c_hi, int r_lo,
                                          int r_hi, const BandPlan& pl, T xcfl, T ycfl) {
    if (c_hi <= c_lo || r_hi <= r_lo) return;
    const int ca = pl.ca, npairs = pl.npairs, nb = pl.nb, R = pl.R;
    // band = task / npairs through a float reciprocal (3 VALU instead of a
    // ~20-instruction integer division per thread and step): task < NT and
    // npairs <= 64, so (task + 0.5) / npairs sits >= 1/128 from an integer and
    // the float error (rcp: 1 ulp; < 2^-12 here) cannot cross it
    static_assert(NT <= 4096, "tile_step: the reciprocal band index needs task < 4096");
    const float inv_np = pl.inv_np;
    for (int task = threadIdx.x; task < npairs * nb; task += NT) {
        const int band = (int)(((float)task + 0.5f) * inv_np);
        const int c0 = ca + 2 * (task - band * npairs);
        const int rb = r_lo + band * R;
        const int re = min(r_hi, rb + R);
        if (rb >= re) continue;
        tile_band<T, ORDER, FMA, PW>(src, dst, c0, rb, re, c0 >= c_lo, c0 + 1 < c_hi, xcfl, ycfl);
    }
}

// Tile + halo from global memory into both LDS buffers: LDS (0, 0) is grid
// cell (gx0, gy0); cells outside the grid buffer read as 0 (a point inside
// the region never reads them: the ghost layer stops every cone). Loads in
// batches of kLB per thread, all issued before their LDS stores, so the
// memory latency is paid once per batch, not once per element.
template <typename T, int LW, int LH, int PW, int NT>
__device__ __forceinline__ void tile_load(const T* __restrict__ prev, T* L0, T* L1, int gx0, int gy0, int pitch,
                                          int gy) {
    if constexpr (LW % 2 == 0) {
        // 16-B (fp64) / 8-B (fp32) column pairs where the tile's first column,
        // the pitch and the buffer are pair-aligned (every production shape):
        // half the loads, and the index math of one element per pair
        if (((gx0 | pitch) & 1) == 0 && ((uintptr_t)prev % (2 * sizeof(T))) == 0) {
            constexpr int LP = LW / 2, kP = LH * LP;
            constexpr int kLB = (kP + NT - 1) / NT < 16 ? (kP + NT - 1) / NT : 16;
            const Pair<T>* p2 = reinterpret_cast<const Pair<T>*>(prev);
            for (int i0 = 0; i0 < kP; i0 += NT * kLB) {
                Pair<T> v[kLB];
#pragma unroll
                for (int k = 0; k < kLB; ++k) {
                    const int i = i0 + k * NT + (int)threadIdx.x;
                    const int r = i / LP, cp = i - r * LP;
                    const int x = gx0 + 2 * cp, y = gy0 + r;  // x even: x < pitch covers x + 1
                    const bool in = i < kP && x >= 0 && x < pitch && y >= 0 && y < gy;
                    v[k] = in ? p2[((size_t)y * pitch + x) >> 1] : Pair<T>{{T(0), T(0)}};
                }
#pragma unroll
                for (int k = 0; k < kLB; ++k) {
                    const int i = i0 + k * NT + (int)threadIdx.x;
                    if (i < kP) {
                        const int r = i / LP, cp = i - r * LP;
                        reinterpret_cast<Pair<T>*>(L0 + r * PW)[cp] = v[k];
                        reinterpret_cast<Pair<T>*>(L1 + r * PW)[cp] = v[k];
                    }
                }
            }
            return;
        }
    }
    constexpr int kN = LH * LW;
    // every load of the tile in flight at once where it fits (9 per thread
    // for the production 64 x 64, NS = 4, 1024-thread shape: one memory
    // latency instead of two; the trace had the 8-per-batch load at 2.2 us)
    constexpr int kLB = (kN + NT - 1) / NT < 16 ? (kN + NT - 1) / NT : 16;
    for (int i0 = 0; i0 < kN; i0 += NT * kLB) {
        T v[kLB];
#pragma unroll
        for (int k = 0; k < kLB; ++k) {
            const int i = i0 + k * NT + (int)threadIdx.x;
            const int r = i / LW, c = i - r * LW;
            const int x = gx0 + c, y = gy0 + r;
            v[k] = (i < kN && x >= 0 && x < pitch && y >= 0 && y < gy) ? prev[(size_t)y * pitch + x] : T(0);
        }
#pragma unroll
        for (int k = 0; k < kLB; ++k) {
            const int i = i0 + k * NT + (int)threadIdx.x;
            if (i < kN) {
                const int r = i / LW, c = i - r * LW;
                L0[r * PW + c] = v[k];
                L1[r * PW + c] = v[k];
            }
        }
    }
}

// NTS: non-temporal output stores
template <typename T, int ORDER, int NS, bool FMA, int TX, int TY, int NT, bool NTS = false>
__global__ __launch_bounds__(NT) void heat_tile_kernel(const T* __restrict__ prev, T* __restrict__ curr, int pitch,
                                                       int gy, Region g, int tiles_x, T xcfl, T ycfl,
                                                       unsigned long long* __restrict__ trace) {
    // trace (profiling only, benchmarks/trace_tile.py): thread 0 of each
    // workgroup records the wall clock at entry, after the load, after each
    // step and after its stores -- trace[8 * block + 0 .. NS + 2]
    unsigned long long tr[8];
    if (trace && threadIdx.x == 0) tr[0] = wall_clock64();
    using G = TileGeom<T, ORDER, NS, TX, TY>;
    constexpr int B = G::B, H = G::H, PW = G::PW, LW = G::LW, LH = G::LH;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* L0 = reinterpret_cast<T*>(smem);
    // the second buffer's element offset goes through an opaque SGPR: folded
    // as a constant, its byte offset (72 KB for fp64 order 8) overflows the
    // 16-bit ds_read offset field and every LDS read of the unrolled step
    // loop paid its own v_add_u32 (5 per row pair)
    // (only where it overflows: a fitting constant offset costs nothing)
    int l1_off = LH * PW;
    if constexpr ((size_t)(LH + 3 * B + 3) * PW * sizeof(T) > 65535) asm volatile("" : "+s"(l1_off));
    T* L1 = L0 + l1_off;
    const int tyi = (int)blockIdx.x / tiles_x;
    const int txi = (int)blockIdx.x - tyi * tiles_x;
    const int ox = g.xb + txi * TX, oy = g.yb + tyi * TY;  // output origin (grid)
    const int gx0 = ox - H, gy0 = oy - H;                  // LDS (0, 0) in grid coordinates
    tile_load<T, LW, LH, PW, NT>(prev, L0, L1, gx0, gy0, pitch, gy);
    __syncthreads();
    if (trace && threadIdx.x == 0) tr[1] = wall_clock64();
    // region g in LDS coordinates
    const int gxl = g.xb - gx0, gxh = g.xe - gx0, gyl = g.yb - gy0, gyh = g.ye - gy0;
    // a tile whose every step region is unclipped by g (all but the edge
    // tiles) takes each step's band plan as compile-time constants
    const bool inner = gxl <= B && gxh >= H + TX + (NS - 1) * B && gyl <= B && gyh >= H + TY + (NS - 1) * B;
#pragma unroll
    for (int s = 1; s <= NS; ++s) {
        const int e = (NS - s) * B;  // this step's reach beyond the output tile
        const int c_lo = max(H - e, gxl), c_hi = min(H + TX + e, gxh);
        const int r_lo = max(H - e, gyl), r_hi = min(H + TY + e, gyh);
        BandPlan pl{0, 1, 1, 1, 1.0f};
        if (inner)
            pl = band_plan<NT>(H - e, H + TX + e, H - e, H + TY + e);
        else if (c_hi > c_lo && r_hi > r_lo)
            pl = band_plan<NT>(c_lo, c_hi, r_lo, r_hi);
        tile_step<T, ORDER, FMA, PW, NT>((s & 1) ? L0 : L1, (s & 1) ? L1 : L0, c_lo, c_hi, r_lo, r_hi, pl, xcfl,
                                         ycfl);
        __syncthreads();
        if (trace && threadIdx.x == 0) tr[1 + s] = wall_clock64();
    }
    const T* fin = (NS & 1) ? L1 : L0;
    const int c_lo = max(H, gxl), c_hi = min(H + TX, gxh);
    const int r_lo = max(H, gyl), r_hi = min(H + TY, gyh);
    const int w = c_hi - c_lo;
    // a whole tile (every tile but the ragged right / bottom ones) goes out as
    // column pairs with a compile-time row length
    bool whole = w == TX && r_hi - r_lo == TY && ((gx0 | pitch) & 1) == 0 &&
                 ((uintptr_t)curr % (2 * sizeof(T))) == 0;
    if constexpr (H % 2 != 0) whole = false;
    if (whole) {
        if constexpr (H % 2 == 0) {
            typedef T T2 __attribute__((ext_vector_type(2)));
            constexpr int TP = TX / 2;
            for (int i = threadIdx.x; i < TP * TY; i += NT) {
                const int r = H + i / TP, cp = H / 2 + i % TP;
                const T2 v = reinterpret_cast<const T2*>(fin + r * PW)[cp];
                T2* d = reinterpret_cast<T2*>(curr + (size_t)(gy0 + r) * pitch + gx0) + cp;
                if constexpr (NTS)
                    __builtin_nontemporal_store(v, d);
                else
                    *d = v;
            }
        }
    } else if (w > 0 && r_hi > r_lo) {
        for (int i = threadIdx.x; i < w * (r_hi - r_lo); i += NT) {
            const int r = r_lo + i / w, c = c_lo + i % w;
            T* d = curr + (size_t)(gy0 + r) * pitch + gx0 + c;
            if constexpr (NTS)
                __builtin_nontemporal_store(fin[r * PW + c], d);
            else
                *d = fin[r * PW + c];
        }
    }
    if (trace && threadIdx.x == 0) {  // vector stores (lane 0)
        tr[NS + 2] = wall_clock64();
        for (int i = 0; i < NS + 3; ++i) trace[8ull * blockIdx.x + i] = tr[i];
    }
}

template <typename T, int ORDER, int NS, bool FMA, int TX, int TY, int NT, bool NTS = false>
int launch_tile(const T* prev, T* curr, int pitch, int gy, Region g, T xcfl, T ycfl, hipStream_t s,
                unsigned long long* trace = nullptr) {
    using G = TileGeom<T, ORDER, NS, TX, TY>;
    auto k = heat_tile_kernel<T, ORDER, NS, FMA, TX, TY, NT, NTS>;
    static const hipError_t attr =
        hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::kBytes);
    if (attr != hipSuccess) return (int)attr;
    const int W = g.xe - g.xb, Hh = g.ye - g.yb;
    if (W <= 0 || Hh <= 0) return 0;
    const int tx = (W + TX - 1) / TX, ty = (Hh + TY - 1) / TY;
    hipLaunchKernelGGL(k, dim3(tx * ty), dim3(NT), G::kBytes, s, prev, curr, pitch, gy, g, tx, xcfl, ycfl, trace);
    return (int)hipGetLastError();
}

}  // namespace cme_tile
