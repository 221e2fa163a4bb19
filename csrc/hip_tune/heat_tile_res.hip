// Resident LDS tiles for SMALL heat grids across a whole run (the hw5 shapes,
// hw/hw5/2dHeat_solution.cpp:501-535 and its time loop :537-628: 1000^2,
// order 8, fp64, 1000 steps).
//
// The tile pass (heat_tile.hip) loads a 64 x 64 tile plus an NS*B halo into
// LDS, runs NS steps over the shrinking dependency cone and writes the tile
// back: per 4-step pass at 1000^2 ~2.2 us of load, 12.2 us of steps and a
// ~4 us kernel boundary (profiles/heat_tile_r4.md). Here ONE cooperative
// launch holds every tile in LDS for the whole run (1000^2 fp64: 256 tiles,
// one workgroup per CU) and only the halo moves:
//
//  * per exchange (every NS = 2 steps by default: the cone recomputes 13 %
//    instead of 43 % at NS = 4) a tile writes the NS*B-deep ring of its own
//    cells that its neighbours read, and reads the ring around it that they
//    wrote -- 1.8 K + 2.3 K values instead of 4 K + 9 K;
//  * the exchange is hidden behind the INNER cone: cells at least s*B inside
//    the tile after step s depend on the tile's own cells only, so each
//    pass first runs steps 1..NS over those shrinking inner rectangles, then
//    waits for its 8 neighbours' completion words, loads the halo, and runs
//    steps 1..NS over the OUTER ring (region_s minus inner_s, up to four
//    rectangles). The two ping-pong LDS buffers stay consistent: inner step
//    s + 2 overwrites buffer (s & 1) only where outer step s + 1 does not
//    read (inner_{s+2} lies (s+2)B inside the tile edge, outer_{s+1} plus the
//    stencil reach ends at (s+2)B - 1);
//  * tiles are placed XCD-contiguous (workgroup i runs on XCD i % 8, so tile
//    rows are dealt to the XCDs in bands) and the ring is stored write-
//    through (sc1) with no L2 write-back: its readers on another XCD find it
//    in memory when the completion word is there, its readers on this XCD
//    in the shared L2 (cdna_hip_programming.md Guideline 16, R1). Each
//    consumer does one agent-scope acquire after its 8 flags.
//
// Every step evaluates the shared expression of heat_stencil.h, so the run
// is bitwise equal to single steps (tests/test_heat_tile_res.py). The last
// pass writes the whole tile; the other buffer's interior is left stale (the
// ghost cells of both stay the boundary values).
//
// Measured (profiles/heat_tile_res_r5.md): 10.4-12 us per 2 steps at 1000^2
// fp64 against 8.9 for the per-pass 4-step tile launches -- the split
// doubles the step calls, whose register-window fill dominates on these small
// rectangles, and the halo hand-off (1.6-2.5 us) outlasts the inner cone.
// So heat_run uses it only with CME_TILE_RES=1; the schedule stays for study.
//
// Bounded waits (the same protocol as heat_flow.hip): a completion word not
// reached within `spins` polls sets the per-call abort word -- every
// workgroup leaves at its next wait -- and the sticky pinned timeout word of
// cme_heat_tile_res_status. The launch is cooperative, so a grid that cannot
// be co-resident is refused at launch instead of deadlocking.
#include "../hip/heat_tile.h"
#include "cme213/persist_ws.h"
#include "cme213/tuning.h"

using namespace cme;
using namespace cme_tile;

namespace {

struct Rect {
    int c_lo, c_hi, r_lo, r_hi;  // LDS coordinates, half-open
};

// One timestep over NR disjoint rectangles from src into dst. The
// rectangles' row bands (a column pair each) are dealt to the NT threads
// together: R rows per band, the smallest R whose bands fit in one round.
template <typename T, int ORDER, bool FMA, int PW, int NT, int NR>
__device__ __forceinline__ void rects_step(const T* __restrict__ src, T* __restrict__ dst, const Rect (&q)[NR],
                                           T xcfl, T ycfl, int minr) {
    int np[NR], nr[NR];
    int work = 0;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        const bool empty = q[i].c_hi <= q[i].c_lo || q[i].r_hi <= q[i].r_lo;
        np[i] = empty ? 0 : (q[i].c_hi - (q[i].c_lo & ~1) + 1) >> 1;
        nr[i] = empty ? 0 : q[i].r_hi - q[i].r_lo;
        work += np[i] * nr[i];
    }
    if (work == 0) return;
    int R = max(minr, (work + NT - 1) / NT);
    for (;; ++R) {  // ends: at R = the tallest rectangle, one band per column pair (<= NR * 41 <= NT)
        int tasks = 0;
#pragma unroll
        for (int i = 0; i < NR; ++i) tasks += np[i] * ((nr[i] + R - 1) / R);
        if (tasks <= NT) break;
    }
    int t = (int)threadIdx.x;
    int c0 = 0, rb = 0, re = 0;
    bool w0 = false, w1 = false, mine = false;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        const int n = np[i] * ((nr[i] + R - 1) / R);
        if (!mine && t < n) {
            const int band = (int)(((float)t + 0.5f) / (float)np[i]);  // t < NT, np <= 64: exact (tile_step)
            c0 = (q[i].c_lo & ~1) + 2 * (t - band * np[i]);
            rb = q[i].r_lo + band * R;
            re = min(q[i].r_hi, rb + R);
            w0 = c0 >= q[i].c_lo;
            w1 = c0 + 1 < q[i].c_hi;
            mine = true;
        }
        if (!mine) t -= n;
    }
    // one call site: the band body is inlined once, whatever rectangle a lane drew
    if (mine && rb < re) tile_band<T, ORDER, FMA, PW>(src, dst, c0, rb, re, w0, w1, xcfl, ycfl);
}

// write-through (sc1) store of one element at element index `idx` of `base`
// (byte offsets fit 32 bits: the launcher checks the buffer size)
template <typename T>
__device__ __forceinline__ void store_wt(T* base, int idx, T v) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
    if constexpr (sizeof(T) == 8) {
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rs, idx * 8, 0, 16);
    } else {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rs, idx * 4, 0, 16);
    }
}

struct ResArgs {
    unsigned* ctl;       // [0] abort
    unsigned* done;      // [ntiles]: 1 + the last pass whose ring that tile published (zeroed per call)
    unsigned* timeout;   // pinned host word: set when a wait gives up (sticky)
    unsigned spins;      // polls per wait before giving up
    int npass;
    int fail_tile;       // diagnostics (tests): this tile never publishes (-1: none)
    int minr;            // rows per band at least (CME_TILE_RES_MINR)
    // profiling: 8 words per (pass, tile): pass start, inner steps done, halo
    // in, outer steps done (ring stores issued), ring published (stamped
    // during the next pass)
    unsigned long long* trace;
};

template <typename T, int ORDER, int NS, bool FMA, int TX, int TY, int NT>
__global__ __launch_bounds__(NT) void heat_tile_res_kernel(T* a, T* b, int pitch, int gy, Region g, int tiles_x,
                                                           int ntiles, T xcfl, T ycfl, ResArgs f) {
    using G = TileGeom<T, ORDER, NS, TX, TY>;
    static_assert(NS % 2 == 0, "a pass must end in the LDS buffer the next one starts from");
    constexpr int B = G::B, H = G::H, PW = G::PW, LW = G::LW, LH = G::LH;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int s_stop;
    T* L0 = reinterpret_cast<T*>(smem);
    int l1_off = LH * PW;  // opaque where the folded offset would overflow ds_read's field (heat_tile.h)
    if constexpr ((size_t)(LH + 3 * B + 3) * PW * sizeof(T) > 65535) asm volatile("" : "+s"(l1_off));
    T* L1 = L0 + l1_off;
    const int lane = lane_id();
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
    // XCD-contiguous tiles: the workgroups of XCD j (blockIdx % 8 == j) take
    // the j-th run of ntiles / 8 (+1) tiles in row-major order
    const int blk = (int)blockIdx.x;
    const int xcd = blk & 7, q8 = ntiles >> 3, r8 = ntiles & 7;
    const int tile = xcd * q8 + min(xcd, r8) + (blk >> 3);
    const int tiles_y = ntiles / tiles_x;
    const int tyi = tile / tiles_x, txi = tile - tyi * tiles_x;
    const int gx0 = g.xb + txi * TX - H, gy0 = g.yb + tyi * TY - H;  // LDS (0, 0) in grid coordinates
    // region g in LDS coordinates; the tile is [H, H + TX) x [H, H + TY) clipped to it
    const int gxl = g.xb - gx0, gxh = g.xe - gx0, gyl = g.yb - gy0, gyh = g.ye - gy0;
    const int tcx = min(H + TX, gxh), tcy = min(H + TY, gyh);
    const bool left_g = txi == 0, right_g = H + TX >= gxh, top_g = tyi == 0, bottom_g = H + TY >= gyh;
    if (threadIdx.x == 0) s_stop = 0;
    tile_load<T, LW, LH, PW, NT>(a, L0, L1, gx0, gy0, pitch, gy);
    __syncthreads();
    // wave 0, lanes 0..8: the completion word of one neighbour each (lane = 3 dy + dx)
    const unsigned* watch = nullptr;
    if (wv == 0 && lane < 9 && lane != 4) {
        const int nx = txi + lane % 3 - 1, ny = tyi + lane / 3 - 1;
        if (nx >= 0 && nx < tiles_x && ny >= 0 && ny < tiles_y) watch = f.done + ny * tiles_x + nx;
    }
    for (int p = 0; p < f.npass; ++p) {
        T* src = (p & 1) ? b : a;
        T* dst = (p & 1) ? a : b;
        // profiling stamps go straight out (vector stores of lane 0): no
        // registers held across the pass
        unsigned long long* tr = f.trace ? f.trace + 8ull * ((size_t)p * ntiles + tile) : nullptr;
        if (tr && threadIdx.x == 0) tr[0] = wall_clock64();
        // ---- inner cone: needs no halo
#pragma unroll
        for (int s = 1; s <= NS; ++s) {
            const Rect in[1] = {{left_g ? gxl : H + s * B, right_g ? gxh : H + TX - s * B, top_g ? gyl : H + s * B,
                                 bottom_g ? gyh : H + TY - s * B}};
            rects_step<T, ORDER, FMA, PW, NT, 1>((s & 1) ? L0 : L1, (s & 1) ? L1 : L0, in, xcfl, ycfl, f.minr);
            // the previous pass's ring stores (write-through) landed behind
            // the first inner step: every wave drains them before the
            // barrier, then one lane publishes the ring
            if (s == 1 && p > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (s == 1 && p > 0 && threadIdx.x == 0) {
                if (tr) tr[4 - 8ll * ntiles] = wall_clock64();  // the previous pass's slot, before the flag
                if (tile != f.fail_tile)
                    __hip_atomic_store(f.done + tile, (unsigned)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (tr && threadIdx.x == 0) tr[1] = wall_clock64();
        // ---- halo: the neighbours' pass p - 1 rings (pass 0 has the loaded one)
        if (p > 0) {
            if (wv == 0) {
                bool give_up = false;
                for (unsigned spins = 0;; ++spins) {
                    const bool ok = watch == nullptr ||
                                    (int)(__hip_atomic_load(watch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) -
                                          (unsigned)p) >= 0;
                    if (__all(ok)) break;
                    if (spins >= f.spins) {
                        if (lane == 0) {
                            __hip_atomic_store(f.ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            __hip_atomic_store(f.timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        }
                        give_up = true;
                        break;
                    }
                    if ((spins & 255u) == 255u &&
                        __builtin_amdgcn_readfirstlane(
                            __hip_atomic_load(f.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0u) {
                        give_up = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                // ONE acquire after the match; its wait holds the barrier below
                // until the invalidate has completed
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (give_up && lane == 0) s_stop = 1;
                // lane 0's LDS write is complete before the barrier the other
                // waves read it behind (heat_flow.hip header)
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
            __syncthreads();
            if (__builtin_amdgcn_readfirstlane(s_stop)) break;
            // the NS*B ring around the tile (cells inside g) into L0: top and
            // bottom bands of whole LDS rows, then the left / right columns
            constexpr int kTB = 2 * H * LW, kRing = kTB + 2 * H * TY;
            constexpr int kPer = (kRing + NT - 1) / NT;
            T v[kPer];
            int at[kPer];
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const int i = k * NT + (int)threadIdx.x;
                int r, c;
                if (i < kTB) {
                    r = i / LW;
                    c = i - r * LW;
                    if (r >= H) r += TY;
                } else {
                    const int j = i - kTB;
                    r = H + j / (2 * H);
                    c = j - (r - H) * (2 * H);
                    if (c >= H) c += TX;
                }
                const bool in = i < kRing && c >= gxl && c < gxh && r >= gyl && r < gyh;
                at[k] = in ? r * PW + c : -1;
                v[k] = in ? src[(size_t)(gy0 + r) * pitch + gx0 + c] : T(0);
            }
#pragma unroll
            for (int k = 0; k < kPer; ++k)
                if (at[k] >= 0) L0[at[k]] = v[k];
            __syncthreads();
        }
        if (tr && threadIdx.x == 0) tr[2] = wall_clock64();
        // ---- outer ring: region_s minus inner_s, up to four rectangles
#pragma unroll
        for (int s = 1; s <= NS; ++s) {
            const int e = (NS - s) * B;
            const int C0 = max(H - e, gxl), C1 = min(H + TX + e, gxh);
            const int R0 = max(H - e, gyl), R1 = min(H + TY + e, gyh);
            int ic0 = left_g ? gxl : H + s * B, ic1 = right_g ? gxh : H + TX - s * B;
            int ir0 = top_g ? gyl : H + s * B, ir1 = bottom_g ? gyh : H + TY - s * B;
            if (ic0 >= ic1 || ir0 >= ir1) {  // no inner part: the top rectangle is the whole region
                ic0 = ic1 = C0;
                ir0 = ir1 = R1;
            }
            const Rect out[4] = {{C0, C1, R0, ir0}, {C0, C1, ir1, R1}, {C0, ic0, ir0, ir1}, {ic1, C1, ir0, ir1}};
            rects_step<T, ORDER, FMA, PW, NT, 4>((s & 1) ? L0 : L1, (s & 1) ? L1 : L0, out, xcfl, ycfl, f.minr);
            __syncthreads();
        }
        // ---- publish: the ring the neighbours read (write-through), or on the
        // last pass the whole tile
        if (p + 1 < f.npass) {
            // tile cells within H of its edge: top / bottom bands, then the
            // left / right columns of the rows between
            constexpr int kTB = 2 * H * TX, kRing = kTB + 2 * H * (TY - 2 * H);
            for (int i = (int)threadIdx.x; i < kRing; i += NT) {
                int r, c;
                if (i < kTB) {
                    r = i / TX;
                    c = H + i - r * TX;
                    r = r < H ? H + r : TY + (r - H);
                } else {
                    const int j = i - kTB;
                    r = 2 * H + j / (2 * H);
                    c = j - (r - 2 * H) * (2 * H);
                    c = c < H ? H + c : TX + (c - H);
                }
                if (c < tcx && r < tcy) store_wt(dst, (gy0 + r) * pitch + gx0 + c, L0[r * PW + c]);
            }
        } else {
            const int w = tcx - H;
            for (int i = (int)threadIdx.x; i < w * (tcy - H); i += NT) {
                const int r = H + i / w, c = H + i % w;
                dst[(size_t)(gy0 + r) * pitch + gx0 + c] = L0[r * PW + c];
            }
        }
        if (tr && threadIdx.x == 0) tr[3] = tr[4] = wall_clock64();  // [4]: the next pass re-stamps it
    }
}

PersistWs& res_ws() {  // abort word + completion words (cme213/persist_ws.h), per device
    return persist_ws_for<1>();
}

constexpr int kCtlWords = 64;

template <typename T, int ORDER, int NS, bool FMA>
int launch_res(T* a, T* b, int pitch, int gy, Region g, T xcfl, T ycfl, int npass, hipStream_t s,
               unsigned long long* trace, int* ntiles_out) {
    constexpr int TX = 64, TY = 64, NT = 1024;
    using G = TileGeom<T, ORDER, NS, TX, TY>;
    static_assert(4 * (G::LW / 2 + 1) <= NT, "rects_step: one band per column pair must fit one round");
    auto k = heat_tile_res_kernel<T, ORDER, NS, FMA, TX, TY, NT>;
    static const hipError_t attr =
        hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::kBytes);
    if (attr != hipSuccess) return (int)attr;
    if (npass < 1) return 0;
    const int W = g.xe - g.xb, Hh = g.ye - g.yb;
    if (W <= 0 || Hh <= 0) return 0;
    if ((size_t)gy * pitch * sizeof(T) >= (1ull << 31)) return (int)hipErrorInvalidValue;  // 32-bit store offsets
    const int tiles_x = (W + TX - 1) / TX, tiles_y = (Hh + TY - 1) / TY;
    const int ntiles = tiles_x * tiles_y;
    if (ntiles_out) *ntiles_out = ntiles;
    static const long resident = [&] {
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, NT, G::kBytes) != hipSuccess || per_cu < 1)
            per_cu = 0;
        return (long)per_cu * device_cu_count();
    }();
    if (ntiles > resident) return (int)hipErrorCooperativeLaunchTooLarge;  // the caller runs tile passes
    PersistWs& w = res_ws();
    const size_t need = kCtlWords + (size_t)ntiles;
    {
        const int rc = w.reserve(need);
        if (rc) return rc;
    }
    CME_TRY(hipMemsetAsync(w.dev, 0, need * 4, s));
    ResArgs f;
    f.ctl = w.dev;
    f.done = w.dev + kCtlWords;
    f.timeout = w.timeout;
    const long sp = cme::tune_get(cme::kTuneFlowSpins);
    f.spins = sp > 0 ? (unsigned)sp : (1u << 22);
    f.npass = npass;
    // diagnostics: CME_FLOW_MODE 2048 -> tile 0 never publishes (the timeout test)
    f.fail_tile = (cme::tune_get(cme::kTuneFlowMode) & 2048) ? 0 : -1;
    f.minr = (int)cme::tune_get(cme::kTuneTileResMinR);
    if (f.minr < 1) f.minr = 1;
    f.trace = trace;
    void* args[] = {&a, &b, &pitch, &gy, &g, (void*)&tiles_x, (void*)&ntiles, &xcfl, &ycfl, &f};
    CME_TRY(hipLaunchCooperativeKernel((const void*)k, dim3((unsigned)ntiles), dim3(NT), args, (unsigned)G::kBytes,
                                       s));
    return 0;
}

template <typename T, int ORDER, bool FMA>
int res_ns(T* a, T* b, int pitch, int gy, Region g, int ns, T xc, T yc, int npass, hipStream_t s,
           unsigned long long* trace, int* nt) {
    if (ns == 2) return launch_res<T, ORDER, 2, FMA>(a, b, pitch, gy, g, xc, yc, npass, s, trace, nt);
    if constexpr (ORDER == 8)
        if (ns == 4) return launch_res<T, ORDER, 4, FMA>(a, b, pitch, gy, g, xc, yc, npass, s, trace, nt);
    return (int)hipErrorInvalidValue;
}

template <typename T>
int res_run(T* a, T* b, int pitch, int gy, Region g, int order, int ns, int fma, T xc, T yc, int npass,
            hipStream_t s, unsigned long long* trace, int* nt) {
    if (fma) {
        switch (order) {
            case 2: return res_ns<T, 2, true>(a, b, pitch, gy, g, ns, xc, yc, npass, s, trace, nt);
            case 4: return res_ns<T, 4, true>(a, b, pitch, gy, g, ns, xc, yc, npass, s, trace, nt);
            case 8: return res_ns<T, 8, true>(a, b, pitch, gy, g, ns, xc, yc, npass, s, trace, nt);
        }
    } else {
        switch (order) {
            case 2: return res_ns<T, 2, false>(a, b, pitch, gy, g, ns, xc, yc, npass, s, trace, nt);
            case 4: return res_ns<T, 4, false>(a, b, pitch, gy, g, ns, xc, yc, npass, s, trace, nt);
            case 8: return res_ns<T, 8, false>(a, b, pitch, gy, g, ns, xc, yc, npass, s, trace, nt);
        }
    }
    return (int)hipErrorInvalidValue;
}

}  // namespace

// npass passes of ns (2, or 4 at order 8) steps of the whole region
// [xb, xe) x [yb, ye) with every tile resident in LDS, in ONE cooperative
// launch; the result lands in (npass & 1 ? b : a). Every cell outside the
// region holds the same fixed value in a and b. Returns
// hipErrorCooperativeLaunchTooLarge when the tiles cannot all be resident
// (heat_run then runs tile passes). trace (may be null): 4 wall-clock stamps
// per (pass, tile), index pass * ntiles + tile; *ntiles (may be null) = tiles.
CME_EXPORT int cme_heat_tile_res_f64(double* a, double* b, int pitch, int gy, int xb, int xe, int yb, int ye, int order,
                                     int ns, int fma, double xcfl, double ycfl, int npass, unsigned long long* trace,
                                     int* ntiles, void* stream) {
    return res_run<double>(a, b, pitch, gy, Region{xb, xe, yb, ye}, order, ns, fma, xcfl, ycfl, npass,
                           as_stream(stream), trace, ntiles);
}

CME_EXPORT int cme_heat_tile_res_f32(float* a, float* b, int pitch, int gy, int xb, int xe, int yb, int ye, int order,
                                     int ns, int fma, float xcfl, float ycfl, int npass, unsigned long long* trace,
                                     int* ntiles, void* stream) {
    return res_run<float>(a, b, pitch, gy, Region{xb, xe, yb, ye}, order, ns, fma, xcfl, ycfl, npass,
                          as_stream(stream), trace, ntiles);
}

// Sticky give-up flag of the resident launches (pinned host word; read after
// the stream is synchronised). reset != 0 clears it.
CME_EXPORT int cme_heat_tile_res_status(unsigned* timed_out, int reset) {
    *timed_out = res_ws().take_timeout(reset != 0);
    return 0;
}

CME_REGISTER_KERNEL(heat_tile_res2_f64_o8, 1024, heat_tile_res_kernel<double, 8, 2, false, 64, 64, 1024>);
CME_REGISTER_KERNEL(heat_tile_res2_fma_f64_o8, 1024, heat_tile_res_kernel<double, 8, 2, true, 64, 64, 1024>);
