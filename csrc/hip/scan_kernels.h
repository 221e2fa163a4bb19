// Kernel templates and launchers of the scan / reduction family (entry
// points: scan.hip production, hip_tune/scan_tune.hip tuning arms).
#pragma once
#include "cme213/common.h"
#include "cme213/tuning.h"
#include "cme213/lookback.h"
#include "cme213/wave.h"

using namespace cme;

namespace {

constexpr int kScanThreads = 256;
constexpr int kScanWaves = kScanThreads / kWave;
constexpr int kScanItemsPerLane = 16;  // 4 x 16-B vectors
constexpr int kScanTile = kScanThreads * kScanItemsPerLane;  // 4096
// Production look-back scan: 16 rows of 16-B vectors per lane (16384-element
// tiles), the two-level look-back (lookback.h lb2_lookback), two tiles of
// loads in flight behind it and non-temporal output stores.
// benchmarks/tune_scan.py at 2^26 fp32 (profiles/scan_tune_r2*.log): 0.0957
// ms (5.61 TB/s) vs 0.138 for round 1's one-level / 8-row / 1-deep arm; 0.085
// with the look-back switched off.
constexpr int kLbRows = 16;
constexpr int kLbMode = 200;  // two-level look-back
constexpr int kLbPf = 2;
// Non-temporal output stores (the scan output is written once): 0.0957 ms
// (5.61 TB/s, 86 % of the one-shot copy) vs 0.115 with plain stores.
constexpr bool kLbNt = true;

template <typename T>
struct Vec4 {
    T x, y, z, w;
};

template <typename T>
__device__ __forceinline__ Vec4<T> load_v4(const T* p, long long i, long long n, T id) {
    Vec4<T> r;
    if (i + 3 < n) {
        typedef T v4 __attribute__((ext_vector_type(4)));
        v4 v = *reinterpret_cast<const v4*>(p + i);
        r.x = v.x;
        r.y = v.y;
        r.z = v.z;
        r.w = v.w;
    } else {
        r.x = i < n ? p[i] : id;
        r.y = i + 1 < n ? p[i + 1] : id;
        r.z = i + 2 < n ? p[i + 2] : id;
        r.w = i + 3 < n ? p[i + 3] : id;
    }
    return r;
}

template <typename T>
__device__ __forceinline__ void store_v4(T* p, long long i, long long n, const Vec4<T>& r) {
    if (i + 3 < n) {
        typedef T v4 __attribute__((ext_vector_type(4)));
        v4 v = {r.x, r.y, r.z, r.w};
        *reinterpret_cast<v4*>(p + i) = v;
    } else {
        if (i < n) p[i] = r.x;
        if (i + 1 < n) p[i + 1] = r.y;
        if (i + 2 < n) p[i + 2] = r.z;
        if (i + 3 < n) p[i + 3] = r.w;
    }
}

// ------------------------------------------------------------ look-back scan
// ROWS 16-B vectors per lane (tile = 256 * 4 * ROWS elements). LOOKBACK=false
// is a timing-only diagnostic arm (tiles scanned independently: wrong result).
template <typename T, bool EXCLUSIVE, int ROWS = 4, bool LOOKBACK = true, int LBD = 1, bool LATE_PF0 = false,
          int PF = 1, bool NTS = false>
__global__ __launch_bounds__(kScanThreads) void scan_lookback_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                                     long long n, uint64_t* desc, int tiles,
                                                                     unsigned* timeout, uint32_t epoch = 0) {
    constexpr int TILE = kScanThreads * 4 * ROWS;
    constexpr int WAVE_ELEMS = kWave * 4 * ROWS;
    __shared__ T s_wtot[2][kScanWaves];
    __shared__ T s_prefix[2];
    const int lane = lane_id();
    int parity = 0;
    // Persistent: block b scans tiles b, b+G, b+2G, ... in order (G = grid size,
    // at most 4 blocks of 256 per CU: co-resident), so every tile's
    // predecessors are owned by running blocks -- no ordering ticket (a single
    // atomic word saturates at ~88 ops/us) and no dispatch-order assumption.
    // The next tile's loads are issued before this tile's look-back wait, so
    // two tiles of loads are in flight per block (the scan is latency-bound
    // on the look-back hand-off, not on bandwidth).
    const int wid = threadIdx.x / kWave;
    Vec4<T> v[ROWS];
    Vec4<T> vn[ROWS];  // PF = 2: tile + G, loaded one iteration ahead
    if (blockIdx.x < tiles) {
        const long long b0 = (long long)blockIdx.x * TILE + wid * WAVE_ELEMS;
#pragma unroll
        for (int k = 0; k < ROWS; ++k) v[k] = load_v4(in, b0 + k * 256 + lane * 4, n, T(0));
        if constexpr (PF == 2) {
            const long long b1 = (long long)(blockIdx.x + gridDim.x) * TILE + wid * WAVE_ELEMS;
            if (blockIdx.x + gridDim.x < tiles) {
#pragma unroll
                for (int k = 0; k < ROWS; ++k) vn[k] = load_v4(in, b1 + k * 256 + lane * 4, n, T(0));
            }
        }
    }
    for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x, parity ^= 1) {
    const long long base = (long long)tile * TILE + wid * WAVE_ELEMS;

    // in-lane inclusive scan of each 4-vector, wave scans of the lane totals,
    // serial carry across the wave-rows
    T run = T(0);
    T ex[ROWS];
#pragma unroll
    for (int k = 0; k < ROWS; ++k) {
        T a = v[k].x, b = a + v[k].y, c = b + v[k].z, d = c + v[k].w;
        T wt;
        T e = wave_exclusive_scan<OpAdd>(d, &wt);
        ex[k] = run + e;
        run = run + wt;
        if (EXCLUSIVE) {
            v[k].w = c;
            v[k].z = b;
            v[k].y = a;
            v[k].x = T(0);
        } else {
            v[k].y = b;
            v[k].z = c;
            v[k].w = d;
        }
    }
    if (lane == 0) s_wtot[parity][wid] = run;
    lds_bcast_sync();
    T wpre = T(0), tot = T(0);
#pragma unroll
    for (int w = 0; w < kScanWaves; ++w) {
        T t = s_wtot[parity][w];
        if (w < wid) wpre = wpre + t;
        tot = tot + t;
    }
    constexpr bool kTwoLevel = LBD == 200;
    if constexpr (kTwoLevel) {
        if (wid == 0 && lane == 0) lb2_put(desc + tile, tot, 0u, epoch);  // agg[tile]
    } else if (LOOKBACK && wid == 0 && lane == 0 && tile > 0) {
        lb_publish(desc + tile, kStAggregate, lb_bits(tot), epoch);
    }
    // prefetch the next tile of this block while the look-back resolves
    // (LATE_PF0: the look-back wave issues its share after the look-back, so
    // its polls do not queue behind its own prefetch in the vmcnt order)
    // PF = 2 keeps two tiles of loads in flight behind the look-back: tile
    // + G is already in vn, tile + 2G goes to vn2
    Vec4<T> vn2[ROWS];
    const int next = tile + gridDim.x;
    const int pf_tile = PF == 2 ? next + gridDim.x : next;
    const long long nb = (long long)pf_tile * TILE + wid * WAVE_ELEMS;
    if (pf_tile < tiles && !(LATE_PF0 && LOOKBACK && wid == 0)) {
#pragma unroll
        for (int k = 0; k < ROWS; ++k) {
            if constexpr (PF == 2)
                vn2[k] = load_v4(in, nb + k * 256 + lane * 4, n, T(0));
            else
                vn[k] = load_v4(in, nb + k * 256 + lane * 4, n, T(0));
        }
    }
    if (!LOOKBACK) {
        if (threadIdx.x == 0) s_prefix[parity] = T(0);
    } else if (kTwoLevel && wid == 0) {
        const T pre = lb2_lookback<T>(lb2_views(desc, tiles), tile, tiles, tot, 0u, timeout, epoch);
        if (lane == 0) s_prefix[parity] = pre;
    } else if (wid == 0) {
        if (tile == 0) {
            if (lane == 0) {
                lb_publish(desc, kStInclusive, lb_bits(tot), epoch);
                s_prefix[parity] = T(0);
            }
        } else {
            T pre;
            if constexpr (LBD < 0)
                pre = lb_lookback_probe<T, false, -LBD>(desc, tile, timeout, epoch);
            else if constexpr (LBD >= 100 && LBD < 200)  // tuning: window 1, s_sleep(LBD - 100) back-off
                pre = lb_lookback<T, false, 1, LBD - 100>(desc, tile, timeout, epoch);
            else
                pre = lb_lookback<T, false, LBD>(desc, tile, timeout, epoch);
            if (lane == 0) {
                lb_publish(desc + tile, kStInclusive, lb_bits(pre + tot), epoch);
                s_prefix[parity] = pre;
            }
        }
        if (LATE_PF0 && next < tiles) {
#pragma unroll
            for (int k = 0; k < ROWS; ++k) vn[k] = load_v4(in, nb + k * 256 + lane * 4, n, T(0));
        }
    }
    lds_bcast_sync();
    const T p = s_prefix[parity] + wpre;
#pragma unroll
    for (int k = 0; k < ROWS; ++k) {
        const T q = p + ex[k];
        Vec4<T> r{q + v[k].x, q + v[k].y, q + v[k].z, q + v[k].w};
        const long long oi = base + k * 256 + lane * 4;
        if (NTS && oi + 3 < n) {  // write-once output: stream it past the caches
            typedef T v4 __attribute__((ext_vector_type(4)));
            const v4 o = {r.x, r.y, r.z, r.w};
            __builtin_nontemporal_store(o, reinterpret_cast<v4*>(out + oi));
        } else {
            store_v4(out, oi, n, r);
        }
    }
#pragma unroll
    for (int k = 0; k < ROWS; ++k) v[k] = vn[k];
    if constexpr (PF == 2) {
#pragma unroll
        for (int k = 0; k < ROWS; ++k) vn[k] = vn2[k];
    }
    }  // tile loop
}

// ------------------------------------------------------------ reduce-then-scan
// Deterministic three-kernel scan (no inter-workgroup hand-off inside a
// launch): K1 reduces contiguous chunks, K2 scans the chunk totals in one
// block, K3 rescans each chunk tile by tile with the carry in LDS, prefetching
// the next tile while the current one is scanned. 12 B/element of traffic,
// bitwise reproducible (fixed summation tree).
constexpr int kRtsBlocks = 1024;

template <typename T>
__global__ __launch_bounds__(256) void rts_reduce_kernel(const T* __restrict__ in, long long n, long long chunk,
                                                         T* __restrict__ part) {
    __shared__ T lds[4];
    const long long b0 = (long long)blockIdx.x * chunk;
    const long long b1 = b0 + chunk < n ? b0 + chunk : n;
    T acc = T(0);
    for (long long i = b0 + threadIdx.x * 4; i < b1; i += 1024) {
        Vec4<T> v = load_v4(in, i, b1, T(0));
        acc = acc + ((v.x + v.y) + (v.z + v.w));
    }
    T r = block_reduce<4>(acc, lds, OpAdd());
    if (threadIdx.x == 0) part[blockIdx.x] = r;
}

// exclusive scan of m partials in place, one block of 1024 threads: 8192
// values per round staged through LDS with coalesced 16-B loads and stores,
// 8 consecutive values per thread scanned serially, the 1024 thread totals by
// the block scan (m = 16384 tile sums of a 2^26 tree scan: 2 rounds; direct
// thread-contiguous global loads touched 16x the lines and took 17 us)
template <typename T>
__global__ __launch_bounds__(1024) void rts_partials_kernel(T* part, int m) {
    constexpr int kPer = 8, kRound = 1024 * kPer;
    __shared__ T lds[16];
    __shared__ T stage[kRound + kRound / 16];  // one pad word per 16 (thread runs of 8: conflict-free halves)
    auto sp = [](int i) { return i + (i >> 4); };
    const int t = threadIdx.x;
    T carry = T(0);
    for (int base = 0; base < m; base += kRound) {
#pragma unroll
        for (int k = 0; k < kPer / 4; ++k) {
            const int e = (k * 1024 + t) * 4;
            const Vec4<T> q = load_v4(part, (long long)base + e, m, T(0));
            stage[sp(e)] = q.x;
            stage[sp(e + 1)] = q.y;
            stage[sp(e + 2)] = q.z;
            stage[sp(e + 3)] = q.w;
        }
        __syncthreads();
        T v[kPer];
        T acc = T(0);
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            v[k] = stage[sp(t * kPer + k)];
            acc = acc + v[k];
        }
        T tot;
        T run = carry + block_exclusive_scan<16>(acc, lds, tot, OpAdd());  // (its barriers order the reads)
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            stage[sp(t * kPer + k)] = run;
            run = run + v[k];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kPer / 4; ++k) {
            const int e = (k * 1024 + t) * 4;
            store_v4(part, (long long)base + e, m, Vec4<T>{stage[sp(e)], stage[sp(e + 1)], stage[sp(e + 2)], stage[sp(e + 3)]});
        }
        __syncthreads();  // the next round's staging writes
        carry = carry + tot;
    }
}

template <typename T, bool EXCLUSIVE>
__global__ __launch_bounds__(256) void rts_scan_kernel(const T* __restrict__ in, T* __restrict__ out, long long n,
                                                       long long chunk, const T* __restrict__ part) {
    __shared__ T s_wtot[2][kScanWaves];
    const int lane = lane_id();
    const int wid = threadIdx.x / kWave;
    const long long b0 = (long long)blockIdx.x * chunk;
    const long long b1 = b0 + chunk < n ? b0 + chunk : n;
    T carry = part[blockIdx.x];
    Vec4<T> v[4], nv[4];
    auto load_tile = [&](long long t0, Vec4<T>* dst) {
#pragma unroll
        for (int k = 0; k < 4; ++k) dst[k] = load_v4(in, t0 + wid * 1024 + k * 256 + lane * 4, b1, T(0));
    };
    if (b0 < b1) load_tile(b0, v);
    int parity = 0;
    for (long long t0 = b0; t0 < b1; t0 += kScanTile, parity ^= 1) {
        if (t0 + kScanTile < b1) load_tile(t0 + kScanTile, nv);
        T run = T(0);
        T ex[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            T a = v[k].x, b = a + v[k].y, c = b + v[k].z, d = c + v[k].w;
            T wt;
            T e = wave_exclusive_scan<OpAdd>(d, &wt);
            ex[k] = run + e;
            run = run + wt;
            if (EXCLUSIVE) {
                v[k].w = c;
                v[k].z = b;
                v[k].y = a;
                v[k].x = T(0);
            } else {
                v[k].y = b;
                v[k].z = c;
                v[k].w = d;
            }
        }
        if (lane == 0) s_wtot[parity][wid] = run;
        lds_bcast_sync();
        T wpre = T(0), tot = T(0);
#pragma unroll
        for (int w = 0; w < kScanWaves; ++w) {
            T t = s_wtot[parity][w];
            if (w < wid) wpre = wpre + t;
            tot = tot + t;
        }
        const T p = carry + wpre;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const T q = p + ex[k];
            Vec4<T> r{q + v[k].x, q + v[k].y, q + v[k].z, q + v[k].w};
            store_v4(out, t0 + wid * 1024 + k * 256 + lane * 4, b1, r);
        }
        carry = carry + tot;
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = nv[k];
    }
}

template <typename T>
int launch_rts(const T* in, T* out, long long n, int exclusive, void* ws, hipStream_t s) {
    if (n <= 0) return 0;
    long long tiles = (n + kScanTile - 1) / kScanTile;
    int blocks = tiles < kRtsBlocks ? (int)tiles : kRtsBlocks;
    long long chunk = ((tiles + blocks - 1) / blocks) * kScanTile;
    blocks = (int)((n + chunk - 1) / chunk);
    T* part = (T*)ws;
    hipLaunchKernelGGL(rts_reduce_kernel<T>, dim3(blocks), dim3(256), 0, s, in, n, chunk, part);
    hipLaunchKernelGGL(rts_partials_kernel<T>, dim3(1), dim3(1024), 0, s, part, blocks);
    if (exclusive)
        hipLaunchKernelGGL((rts_scan_kernel<T, true>), dim3(blocks), dim3(256), 0, s, in, out, n, chunk, part);
    else
        hipLaunchKernelGGL((rts_scan_kernel<T, false>), dim3(blocks), dim3(256), 0, s, in, out, n, chunk, part);
    CME_LAUNCH_STATUS();
}

// ------------------------------------------------------------ multi-level
// Block algorithms operate on 2*kMLThreads elements in LDS.
constexpr int kMLThreads = 256;
constexpr int kMLElems = 2 * kMLThreads;
// ds_read/write_b32 bank of byte address a is (a/4) % 32 on gfx950: pad one
// word every 32 (Harris' CONFLICT_FREE_OFFSET with LOG_NUM_BANKS = 5).
__host__ __device__ constexpr int cf(int i) { return i + (i >> 5); }

template <typename T>
__device__ void blelloch_block(T* s, T& total) {
    const int t = threadIdx.x;
    int offset = 1;
    for (int d = kMLElems >> 1; d > 0; d >>= 1) {  // up-sweep (reduce)
        __syncthreads();
        if (t < d) {
            int ai = offset * (2 * t + 1) - 1, bi = offset * (2 * t + 2) - 1;
            s[cf(bi)] += s[cf(ai)];
        }
        offset <<= 1;
    }
    __syncthreads();
    total = s[cf(kMLElems - 1)];
    __syncthreads();
    if (t == 0) s[cf(kMLElems - 1)] = T(0);
    for (int d = 1; d < kMLElems; d <<= 1) {  // down-sweep
        offset >>= 1;
        __syncthreads();
        if (t < d) {
            int ai = offset * (2 * t + 1) - 1, bi = offset * (2 * t + 2) - 1;
            T x = s[cf(ai)];
            s[cf(ai)] = s[cf(bi)];
            s[cf(bi)] += x;
        }
    }
    __syncthreads();
}

// Hillis-Steele inclusive scan (double-buffered), then shift to exclusive.
template <typename T>
__device__ void hillis_block(T* s, T* s2, T& total) {
    const int t = threadIdx.x;
    T* src = s;
    T* dst = s2;
    for (int off = 1; off < kMLElems; off <<= 1) {
        __syncthreads();
        for (int i = t; i < kMLElems; i += kMLThreads) dst[cf(i)] = i >= off ? src[cf(i)] + src[cf(i - off)] : src[cf(i)];
        T* tmp = src;
        src = dst;
        dst = tmp;
    }
    __syncthreads();
    total = src[cf(kMLElems - 1)];
    for (int i = t; i < kMLElems; i += kMLThreads) dst[cf(i)] = i ? src[cf(i - 1)] : T(0);
    __syncthreads();
    if (dst != s)
        for (int i = t; i < kMLElems; i += kMLThreads) s[cf(i)] = dst[cf(i)];
    __syncthreads();
}

template <typename T, int ALGO>
__global__ __launch_bounds__(kMLThreads) void scan_block_kernel(const T* in, T* out, T* sums, long long n) {
    __shared__ T s[cf(kMLElems) + 1];
    __shared__ T s2[ALGO == 1 ? cf(kMLElems) + 1 : 1];
    const long long b = (long long)blockIdx.x * kMLElems;
    for (int i = threadIdx.x; i < kMLElems; i += kMLThreads) s[cf(i)] = b + i < n ? in[b + i] : T(0);
    T total;
    if constexpr (ALGO == 0) blelloch_block(s, total);
    else hillis_block(s, s2, total);
    for (int i = threadIdx.x; i < kMLElems; i += kMLThreads)
        if (b + i < n) out[b + i] = s[cf(i)];
    if (threadIdx.x == 0 && sums) sums[blockIdx.x] = total;
}

template <typename T>
__global__ __launch_bounds__(256) void add_offsets_kernel(T* __restrict__ out, const T* __restrict__ offs, long long n) {
    const long long b = (long long)blockIdx.x * kMLElems;
    const T o = offs[blockIdx.x];
    for (int i = threadIdx.x; i < kMLElems; i += 256)
        if (b + i < n) out[b + i] += o;
}

template <typename T>
__global__ void to_inclusive_kernel(const T* __restrict__ in, T* __restrict__ out, long long n) {
    long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i < n) out[i] += in[i];
}

// ------------------------------------------------------------ tree scans, rts
// The lecture's block algorithms (Blelloch work-efficient up/down-sweep,
// Hillis-Steele) as the block level of a reduce-then-scan (K1/K2 shared with
// the DPP version above): each thread scans 16 consecutive elements in
// registers, the 256 thread totals are scanned in LDS by the tree algorithm
// (conflict-free padding cf()), the chunk carry rides in a register. 12 B per
// element like rts, instead of the multi-level scheme's 16.
constexpr int kTreeItems = 16;
constexpr int kTreeTile = 256 * kTreeItems;

template <typename T, int ALGO>
__device__ __forceinline__ T tree_block_exclusive(T v, T* s, T* s2, T& total) {
    const int t = threadIdx.x;
    if constexpr (ALGO == 0) {
        // Blelloch's up-sweep / down-sweep tree over each wave's 64 values in
        // LDS, then the 4 wave totals. A wave's LDS operations execute in
        // order, so the tree levels inside a wave need no workgroup barrier
        // (only the compiler's wave barrier between levels): 2 barriers per
        // 256 values instead of the 256-wide tree's 17, which held the pass
        // at 117 us for 2^26 floats against 83 for the DPP block scan
        const int lane = t & (kWave - 1), w = t / kWave;
        T* sw = s + w * (kWave + kWave / 32);  // this wave's padded 64-value segment: cf(j) = j + j / 32
        sw[cf(lane)] = v;
        int offset = 1;
#pragma unroll
        for (int d = kWave / 2; d > 0; d >>= 1) {  // up-sweep (reduce)
            wave_lds_sync();
            if (lane < d) {
                const int ai = offset * (2 * lane + 1) - 1, bi = offset * (2 * lane + 2) - 1;
                sw[cf(bi)] += sw[cf(ai)];
            }
            offset <<= 1;
        }
        wave_lds_sync();
        const T wtot = sw[cf(kWave - 1)];
        wave_lds_sync();
        if (lane == 0) sw[cf(kWave - 1)] = T(0);
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {  // down-sweep
            offset >>= 1;
            wave_lds_sync();
            if (lane < d) {
                const int ai = offset * (2 * lane + 1) - 1, bi = offset * (2 * lane + 2) - 1;
                const T x = sw[cf(ai)];
                sw[cf(ai)] = sw[cf(bi)];
                sw[cf(bi)] += x;
            }
        }
        wave_lds_sync();
        T r = sw[cf(lane)];
        // the wave totals (stored past the 4 segments), one barrier
        T* st = s + 4 * (kWave + kWave / 32);
        if (lane == 0) st[w] = wtot;
        __syncthreads();
        T off = T(0);
        total = T(0);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const T x = st[k];
            if (k < w) off = off + x;
            total = total + x;
        }
        __syncthreads();  // the next tile rewrites the segments and totals
        return r + off;
    } else {  // Hillis-Steele (double-buffered) over 256 values
        T* src = s;
        T* dst = s2;
        src[t] = v;
        for (int off = 1; off < 256; off <<= 1) {
            __syncthreads();
            dst[t] = t >= off ? src[t] + src[t - off] : src[t];
            T* tmp = src;
            src = dst;
            dst = tmp;
        }
        __syncthreads();
        total = src[255];
        const T r = t ? src[t - 1] : T(0);
        __syncthreads();
        return r;
    }
}

// LDS index of the tile staging buffer: one pad word per 16, so a thread's
// run of 16 consecutive values starts 17 words after its neighbour's (no bank
// conflicts in the thread-contiguous reads / writes)
__host__ __device__ constexpr int tpad(int i) { return i + (i >> 4); }

// Tile-parallel reduce-then-scan with the lecture's tree at the block level.
//  K1 tile_reduce_kernel: one sum per 4096-element tile (16 B loads, the next
//     tile prefetched), tiles visited in ascending order (iteration j of the
//     grid-stride loop covers tiles [jG, (j+1)G));
//  K2 rts_partials_kernel: exclusive scan of the tile sums (one block);
//  K3 tile_tree_scan_kernel: each tile independently -- coalesced 16-B loads
//     staged through LDS, 16 consecutive values per thread scanned in
//     registers, the 256 thread totals by the block tree (Blelloch / Hillis),
//     plus the tile's prefix from K2 -- visiting the tiles in DESCENDING
//     order, so the first tiles K3 reads are the last K1 read, still in the
//     256 MB Infinity Cache (every 2^26 fp32 tile but the first ~13 MB of K1's
//     sweep), and storing non-temporally (the output is written once).
// 12 B per element from HBM at most (my-refs/scan.pdf: reduce, scan of block
// sums, scan + add), bitwise reproducible (fixed trees, no hand-off).
template <typename T>
__device__ __forceinline__ void tile_load4(const T* __restrict__ in, long long t0, long long n, Vec4<T> (&q)[4]) {
#pragma unroll
    for (int k = 0; k < kTreeTile / 1024; ++k) q[k] = load_v4(in, t0 + k * 1024 + (int)threadIdx.x * 4, n, T(0));
}

template <typename T>
__global__ __launch_bounds__(256) void tile_reduce_kernel(const T* __restrict__ in, long long n, int ntiles,
                                                          T* __restrict__ tsum) {
    __shared__ T lds[4];
    Vec4<T> q[4], qn[4];
    int tile = blockIdx.x;
    if (tile < ntiles) tile_load4(in, (long long)tile * kTreeTile, n, q);
    for (; tile < ntiles; tile += gridDim.x) {
        if (tile + (int)gridDim.x < ntiles) tile_load4(in, (long long)(tile + gridDim.x) * kTreeTile, n, qn);
        T acc = T(0);
#pragma unroll
        for (int k = 0; k < 4; ++k) acc = acc + ((q[k].x + q[k].y) + (q[k].z + q[k].w));
        const T r = block_reduce<4>(acc, lds, OpAdd());
        if (threadIdx.x == 0) tsum[tile] = r;
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = qn[k];
    }
}

template <typename T, bool EXCLUSIVE, int ALGO>
__global__ __launch_bounds__(256) void tile_tree_scan_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                             long long n, int ntiles, const T* __restrict__ tpre) {
    __shared__ T s[4 * (kWave + kWave / 32) + 4];  // Blelloch: 4 padded wave segments + the wave totals
    __shared__ T s2[ALGO == 1 ? 256 : 1];
    __shared__ T tile[tpad(kTreeTile)];
    const int t = threadIdx.x;
    Vec4<T> q[4], qn[4];
    int j = blockIdx.x;  // tile ntiles - 1 - j
    if (j < ntiles) tile_load4(in, (long long)(ntiles - 1 - j) * kTreeTile, n, q);
    for (; j < ntiles; j += gridDim.x) {
        const int id = ntiles - 1 - j;
        const long long t0 = (long long)id * kTreeTile;
        const T tile_pre = tpre[id];
        if (j + (int)gridDim.x < ntiles) tile_load4(in, (long long)(id - (int)gridDim.x) * kTreeTile, n, qn);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int e = k * 1024 + t * 4;
            tile[tpad(e)] = q[k].x;
            tile[tpad(e + 1)] = q[k].y;
            tile[tpad(e + 2)] = q[k].z;
            tile[tpad(e + 3)] = q[k].w;
        }
        __syncthreads();
        T v[kTreeItems];
#pragma unroll
        for (int k = 0; k < kTreeItems; ++k) v[k] = tile[tpad(t * kTreeItems + k)];
        T acc = T(0);
#pragma unroll
        for (int k = 0; k < kTreeItems; ++k) {  // serial in-thread scan
            const T x = v[k];
            v[k] = EXCLUSIVE ? acc : acc + x;
            acc = acc + x;
        }
        T tot;
        // (its barriers also order every thread's reads above before the
        // writes below)
        const T pre = tile_pre + tree_block_exclusive<T, ALGO>(acc, s, s2, tot);
#pragma unroll
        for (int k = 0; k < kTreeItems; ++k) tile[tpad(t * kTreeItems + k)] = pre + v[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int e = k * 1024 + t * 4;
            const long long oi = t0 + e;
            const Vec4<T> r{tile[tpad(e)], tile[tpad(e + 1)], tile[tpad(e + 2)], tile[tpad(e + 3)]};
            if (oi + 4 <= n) {
                typedef T v4 __attribute__((ext_vector_type(4)));
                const v4 o = {r.x, r.y, r.z, r.w};
                __builtin_nontemporal_store(o, reinterpret_cast<v4*>(out + oi));
            } else {
                store_v4(out, oi, n, r);
            }
        }
        __syncthreads();  // the next tile's staging writes
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = qn[k];
    }
}

// ws: 4-B tile sums / prefixes, cdiv(n, 4096) of them
template <typename T>
int launch_tree_rts(const T* in, T* out, long long n, int algo, int exclusive, void* ws, hipStream_t s) {
    if (n <= 0) return 0;
    const long long tiles = (n + kTreeTile - 1) / kTreeTile;
    if (tiles >= (1ll << 31)) return (int)hipErrorInvalidValue;
    const int nt = (int)tiles;
    const int blocks = nt < kRtsBlocks ? nt : kRtsBlocks;
    T* part = (T*)ws;
    hipLaunchKernelGGL(tile_reduce_kernel<T>, dim3(blocks), dim3(256), 0, s, in, n, nt, part);
    hipLaunchKernelGGL(rts_partials_kernel<T>, dim3(1), dim3(1024), 0, s, part, nt);
#define TREE(E, A) \
    hipLaunchKernelGGL((tile_tree_scan_kernel<T, E, A>), dim3(blocks), dim3(256), 0, s, in, out, n, nt, part)
    if (algo == 0) {
        if (exclusive) TREE(true, 0); else TREE(false, 0);
    } else {
        if (exclusive) TREE(true, 1); else TREE(false, 1);
    }
#undef TREE
    CME_LAUNCH_STATUS();
}

// ------------------------------------------------------------ reduction
template <typename T, typename Op>
__global__ __launch_bounds__(256) void reduce_partial_kernel(const T* __restrict__ in, long long n, T* __restrict__ part,
                                                             Op op) {
    __shared__ T lds[4];
    T acc = Op::template identity<T>();
    const long long stride = (long long)gridDim.x * 256 * 4;
    long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
    // four 16-B loads in flight per lane: 2^26 f32 cold 0.0497 -> 0.0452 ms
    // (hip_tune/scan_tune.hip cme_reduce_tune, profiles/scan_r5.md round 6)
    constexpr int U = 4;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        Vec4<T> v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = load_v4(in, i + u * stride, n, Op::template identity<T>());
#pragma unroll
        for (int u = 0; u < U; ++u) acc = op(acc, op(op(v[u].x, v[u].y), op(v[u].z, v[u].w)));
    }
    for (; i < n; i += stride) {
        Vec4<T> v = load_v4(in, i, n, Op::template identity<T>());
        acc = op(acc, op(op(v.x, v.y), op(v.z, v.w)));
    }
    T r = block_reduce<4>(acc, lds, op);
    if (threadIdx.x == 0) part[blockIdx.x] = r;
}

template <typename T, typename Op>
__global__ __launch_bounds__(1024) void reduce_final_kernel(const T* __restrict__ part, int m, T* __restrict__ out,
                                                            Op op) {
    __shared__ T lds[16];
    T acc = Op::template identity<T>();
    for (int i = threadIdx.x; i < m; i += 1024) acc = op(acc, part[i]);
    T r = block_reduce<16>(acc, lds, op);
    if (threadIdx.x == 0) *out = r;
}

// The lecture's shared-memory tree (Lecture05 slides 15-16), one element per
// thread per step; kept for the optimisation ladder.
template <typename T>
__global__ __launch_bounds__(256) void reduce_tree_kernel(const T* __restrict__ in, long long n, T* __restrict__ part) {
    __shared__ T s[256];
    T acc = T(0);
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) acc += in[i];
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) s[threadIdx.x] += s[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = s[0];
}

// ------------------------------------------------------------ segmented scan
// Pair operator for (flag, value): (f1,v1) . (f2,v2) = (f1|f2, f2 ? v2 : v1+v2)
__device__ __forceinline__ void seg_combine(uint32_t& f, float& v, uint32_t fs, float vs) {
    v = f ? v : vs + v;
    f = f | fs;
}

// Wave inclusive segmented scan via DPP (flags 0/1 per lane).
__device__ __forceinline__ float wave_segscan(float v, uint32_t f, uint32_t* f_out) {
#define SEG_STEP(CTRL, RM)                                           \
    {                                                                \
        float vs = dpp_move<CTRL, RM>(0.0f, v);                      \
        uint32_t fs = dpp_move<CTRL, RM>(0u, f);                     \
        seg_combine(f, v, fs, vs);                                   \
    }
    SEG_STEP(kDppRowShr1, 0xf)
    SEG_STEP(kDppRowShr2, 0xf)
    SEG_STEP(kDppRowShr4, 0xf)
    SEG_STEP(kDppRowShr8, 0xf)
    SEG_STEP(kDppRowBcast15, 0xa)
    SEG_STEP(kDppRowBcast31, 0xc)
#undef SEG_STEP
    *f_out = f;
    return v;
}

// flags source: MODE 0 = uint8 per element, MODE 1 = bitmask words (bit i%32
// of word i/32). FUSED_MUL: v = a[i]*x[i] before scanning (final project).
// Raw per-row inputs of one lane (loads only; decoding and the fused
// multiply happen at use, so a prefetch never waits on memory).
struct SegRaw {
    Vec4<float> a, x;
    uint32_t fw;  // MODE 0: 4 flag bytes; MODE 1: the bitmask word
};

template <int MODE, bool FUSED_MUL>
__device__ __forceinline__ SegRaw seg_load(const float* __restrict__ in, const float* __restrict__ xmul,
                                           const void* __restrict__ flags, long long i, long long n) {
    SegRaw r;
    r.a = load_v4(in, i, n, 0.f);
    if constexpr (FUSED_MUL) r.x = load_v4(xmul, i, n, 0.f);
    if constexpr (MODE == 0) {
        const uint8_t* fp = (const uint8_t*)flags;
        if (i + 3 < n) {
            r.fw = *reinterpret_cast<const uint32_t*>(fp + i);
        } else {
            r.fw = 0;
            for (int j = 0; j < 4; ++j)
                if (i + j < n && fp[i + j]) r.fw |= 1u << (8 * j);
        }
    } else {
        const uint32_t* fw = (const uint32_t*)flags;
        r.fw = i < n ? fw[i >> 5] : 0u;
    }
    return r;
}

// ROWS 16-B vectors per lane per tile; PREFETCH issues the next tile's loads
// before the look-back wait (two tiles of loads in flight per block).
// Production: ROWS 4, no prefetch (benchmarks/tune_scan.py --spmv: prefetch
// and 8 rows both lose to register pressure -- profiles/spmv_scan_tune.jsonl).
//
// MULTI: `iters` in-place steps a <- segscan(a * xmul) in ONE launch (in ==
// out). Block b owns tiles b, b+G, ... in every step and each lane re-reads
// exactly the elements it wrote, so a step's input needs no cross-block
// synchronisation -- only the look-back does. Step i has its OWN descriptor
// set (`desc + i * desc_stride`, epoch `epoch + i`): blocks that own only
// early tiles depend on nothing later and may run several steps ahead, so a
// set may not be reused within a launch. Every wait depends only on earlier
// (step, tile) pairs of a co-resident grid (processed in that order by every
// block), so the smallest unfinished pair can always proceed.
template <int MODE, bool FUSED_MUL, int ROWS = 4, bool PREFETCH = false, bool LB2 = false, bool MULTI = false>
__global__ __launch_bounds__(kScanThreads) void segscan_kernel(const float* __restrict__ in, const float* __restrict__ xmul,
                                                               float* __restrict__ out, const void* __restrict__ flags,
                                                               long long n, uint64_t* desc0, int tiles,
                                                               unsigned* timeout, uint32_t epoch0, int iters = 1,
                                                               long long desc_stride = 0) {
    constexpr int TILE = kScanThreads * 4 * ROWS;
    constexpr int WAVE_ELEMS = kWave * 4 * ROWS;
    __shared__ float s_wv_[2][kScanWaves];
    __shared__ uint32_t s_wf_[2][kScanWaves];
    __shared__ float s_prefix_[2];
    const int lane = lane_id();
    const int wid = threadIdx.x / kWave;
    int parity = 0;
    // MULTI runs in place: every load goes through `out` (a restrict pointer
    // must be the only path to the data it modifies)
    const float* src = MULTI ? (const float*)out : in;
    SegRaw raw[ROWS];
    if (blockIdx.x < tiles) {
        const long long b0 = (long long)blockIdx.x * TILE + wid * WAVE_ELEMS;
#pragma unroll
        for (int k = 0; k < ROWS; ++k) raw[k] = seg_load<MODE, FUSED_MUL>(src, xmul, flags, b0 + k * 256 + lane * 4, n);
    }
    const int nit = MULTI ? iters : 1;
    for (int it = 0; it < nit; ++it) {
    uint64_t* desc = desc0 + (MULTI ? it * desc_stride : 0);
    const uint32_t epoch = epoch0 + (uint32_t)it;
    // persistent, co-resident grid (see scan_lookback_kernel)
    for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x, parity ^= 1) {
    float* s_wv = s_wv_[parity];
    uint32_t* s_wf = s_wf_[parity];
    float& s_prefix = s_prefix_[parity];
    const long long base = (long long)tile * TILE + wid * WAVE_ELEMS;

    float val[ROWS][4];
    uint32_t flm[ROWS];  // bit j: a head at or before element j of the lane's 4
    float run_v = 0.f;   // running (segment-aware) value across the rows
    uint32_t run_f = 0;  // any head seen so far in this wave
    float ex_v[ROWS];
    uint32_t ex_f[ROWS];
#pragma unroll
    for (int k = 0; k < ROWS; ++k) {
        const long long i = base + k * 256 + lane * 4;
        Vec4<float> a = raw[k].a;
        if constexpr (FUSED_MUL) {
            a.x *= raw[k].x.x;
            a.y *= raw[k].x.y;
            a.z *= raw[k].x.z;
            a.w *= raw[k].x.w;
        }
        uint32_t f4;
        if constexpr (MODE == 0) {
            const uint32_t w = raw[k].fw;
            f4 = (w & 1u) | ((w >> 7) & 2u) | ((w >> 14) & 4u) | ((w >> 21) & 8u);
        } else {
            f4 = (raw[k].fw >> (i & 31)) & 0xfu;
        }
        // in-lane inclusive segmented scan of 4 values
        float v0 = a.x, v1 = a.y, v2 = a.z, v3 = a.w;
        const uint32_t g0 = f4 & 1, g1 = (f4 >> 1) & 1, g2 = (f4 >> 2) & 1, g3 = (f4 >> 3) & 1;
        v1 = g1 ? v1 : v0 + v1;
        v2 = g2 ? v2 : v1 + v2;
        v3 = g3 ? v3 : v2 + v3;
        val[k][0] = v0;
        val[k][1] = v1;
        val[k][2] = v2;
        val[k][3] = v3;
        const uint32_t c1 = g0 | g1, c2 = c1 | g2, c3 = c2 | g3;
        flm[k] = g0 | (c1 << 1) | (c2 << 2) | (c3 << 3);
        // wave scan of lane totals (value v3, flag = any head in lane)
        uint32_t lf;
        float inc = wave_segscan(v3, c3, &lf);
        // exclusive (shift by one lane); lane 0 gets the carry from earlier rows
        float e_v = dpp_move<kDppWaveShr1>(0.f, inc);
        uint32_t e_f = dpp_move<kDppWaveShr1>(0u, lf);
        float row_tot_v = wave_readlane(inc, kWave - 1);
        uint32_t row_tot_f = (uint32_t)__builtin_amdgcn_readlane((int)lf, kWave - 1);
        // combine carry (run) with the exclusive lane prefix: carry applies
        // unless a head occurred in earlier lanes of this row
        ex_v[k] = e_f ? e_v : run_v + e_v;
        ex_f[k] = e_f | run_f;
        run_v = row_tot_f ? row_tot_v : run_v + row_tot_v;
        run_f = run_f | row_tot_f;
    }
    if (lane == 0) {
        s_wv[wid] = run_v;
        s_wf[wid] = run_f;
    }
    __syncthreads();
    // wave prefix (segment-aware) and tile aggregate
    float wpre_v = 0.f;
    uint32_t wpre_f = 0;
    float tot_v = 0.f;
    uint32_t tot_f = 0;
#pragma unroll
    for (int w = 0; w < kScanWaves; ++w) {
        const float tv = s_wv[w];
        const uint32_t tf = s_wf[w];
        if (w < wid) {
            wpre_v = tf ? tv : wpre_v + tv;
            wpre_f |= tf;
        }
        tot_v = tf ? tv : tot_v + tv;
        tot_f |= tf;
    }
    const uint32_t hf = tot_f ? kStFlag : 0u;
    if constexpr (LB2) {
        if (wid == 0 && lane == 0) lb2_put(desc + tile, tot_v, hf, epoch);  // agg[tile]
    } else if (wid == 0 && lane == 0 && tile > 0) {
        lb_publish(desc + tile, kStAggregate | hf, __builtin_bit_cast(uint32_t, tot_v), epoch);
    }
    const int next = tile + gridDim.x;
    if (PREFETCH && next < tiles) {
        const long long nb = (long long)next * TILE + wid * WAVE_ELEMS;
#pragma unroll
        for (int k = 0; k < ROWS; ++k) raw[k] = seg_load<MODE, FUSED_MUL>(src, xmul, flags, nb + k * 256 + lane * 4, n);
    }
    if (LB2 && wid == 0) {
        const float pre = lb2_lookback<float, true>(lb2_views(desc, tiles), tile, tiles, tot_v, hf, timeout, epoch);
        if (lane == 0) s_prefix = pre;
    } else if (wid == 0) {
        if (tile == 0) {
            if (lane == 0) {
                lb_publish(desc, kStInclusive | hf, __builtin_bit_cast(uint32_t, tot_v), epoch);
                s_prefix = 0.f;
            }
        } else {
            float pre = lb_lookback<float, true>(desc, tile, timeout, epoch);
            if (lane == 0) {
                float incl = tot_f ? tot_v : pre + tot_v;
                lb_publish(desc + tile, kStInclusive | hf, __builtin_bit_cast(uint32_t, incl), epoch);
                s_prefix = pre;
            }
        }
    }
    lds_bcast_sync();
    // carry into this wave: tile prefix unless a head precedes in the tile
    const float tile_pre = s_prefix;
    const float wcarry = wpre_f ? wpre_v : tile_pre + wpre_v;
#pragma unroll
    for (int k = 0; k < ROWS; ++k) {
        const float c = ex_f[k] ? ex_v[k] : wcarry + ex_v[k];
        Vec4<float> r;
        r.x = (flm[k] & 1u) ? val[k][0] : c + val[k][0];
        r.y = (flm[k] & 2u) ? val[k][1] : c + val[k][1];
        r.z = (flm[k] & 4u) ? val[k][2] : c + val[k][2];
        r.w = (flm[k] & 8u) ? val[k][3] : c + val[k][3];
        store_v4(out, base + k * 256 + lane * 4, n, r);
    }
    if (!PREFETCH && next < tiles) {
        const long long nb = (long long)next * TILE + wid * WAVE_ELEMS;
#pragma unroll
        for (int k = 0; k < ROWS; ++k) raw[k] = seg_load<MODE, FUSED_MUL>(src, xmul, flags, nb + k * 256 + lane * 4, n);
    } else if (MULTI && next >= tiles && it + 1 < nit) {
        // the next step starts at this block's first tile, which this lane
        // stored earlier (the tile just stored, if the block owns only one)
        const long long nb = (long long)blockIdx.x * TILE + wid * WAVE_ELEMS;
#pragma unroll
        for (int k = 0; k < ROWS; ++k) raw[k] = seg_load<MODE, FUSED_MUL>(src, xmul, flags, nb + k * 256 + lane * 4, n);
    }
    }  // tile loop
    }  // step loop
}

// epoch 0: zero the descriptors first (one memset); epoch e > 0: the caller
// zeroed `ws` once and gives every launch a new epoch (stale descriptors of
// earlier launches never match), so repeated scans skip the memset.
template <typename T>
int launch_scan(const T* in, T* out, long long n, int exclusive, void* ws, hipStream_t s, uint32_t epoch) {
    if (n <= 0) return 0;
    const int tiles = (int)((n + 1024LL * kLbRows - 1) / (1024LL * kLbRows));
    static int bpc_e = persistent_blocks_per_cu(
        scan_lookback_kernel<T, true, kLbRows, true, kLbMode, false, kLbPf, kLbNt>, kScanThreads);
    static int bpc_i = persistent_blocks_per_cu(
        scan_lookback_kernel<T, false, kLbRows, true, kLbMode, false, kLbPf, kLbNt>, kScanThreads);
    const int cap = device_cu_count() * (exclusive ? bpc_e : bpc_i);
    const int grid = tiles < cap ? tiles : cap;
    unsigned* timeout = lb_host_timeout();
    if (!timeout) return (int)hipErrorOutOfMemory;
    uint64_t* desc = lb_descriptors(ws);
    if (epoch == 0) CME_TRY(hipMemsetAsync(ws, 0, lb2_ws_bytes(tiles), s));
    if (epoch >= (1u << 24)) return (int)hipErrorInvalidValue;
    if (exclusive)
        hipLaunchKernelGGL((scan_lookback_kernel<T, true, kLbRows, true, kLbMode, false, kLbPf, kLbNt>), dim3(grid),
                           dim3(kScanThreads), 0, s, in, out, n, desc, tiles, timeout, epoch);
    else
        hipLaunchKernelGGL((scan_lookback_kernel<T, false, kLbRows, true, kLbMode, false, kLbPf, kLbNt>), dim3(grid),
                           dim3(kScanThreads), 0, s, in, out, n, desc, tiles, timeout, epoch);
    CME_LAUNCH_STATUS();
}

// Recursive scan-then-add; `ws` must hold sum(levels) elements (see
// cme_scan_mlevel_ws_elems). Produces an EXCLUSIVE scan.
template <typename T>
int mlevel(const T* in, T* out, long long n, int algo, T* ws, hipStream_t s) {
    const long long blocks = (n + kMLElems - 1) / kMLElems;
    T* sums = blocks > 1 ? ws : nullptr;
    if (algo == 0)
        hipLaunchKernelGGL((scan_block_kernel<T, 0>), dim3((unsigned)blocks), dim3(kMLThreads), 0, s, in, out, sums, n);
    else
        hipLaunchKernelGGL((scan_block_kernel<T, 1>), dim3((unsigned)blocks), dim3(kMLThreads), 0, s, in, out, sums, n);
    CME_TRY(hipGetLastError());
    if (blocks > 1) {
        int rc = mlevel<T>(sums, sums, blocks, algo, ws + blocks, s);
        if (rc) return rc;
        hipLaunchKernelGGL(add_offsets_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, s, out, sums, n);
        CME_TRY(hipGetLastError());
    }
    return 0;
}

}  // namespace

// Final-project driver: `iters` fused steps a <- segscan(a * xx) (bitmask
// heads) with ONE descriptor memset; iteration i uses look-back epoch i+1.
namespace {
// MULTI: up to kSpmvScanSteps steps per launch, one descriptor set per step
// (cme_spmv_scan_ws_bytes sizes the workspace for that; see segscan_kernel).
constexpr int kSpmvScanSteps = 64;
template <int ROWS, bool PF, bool LB2 = false, bool MULTI = false>
int spmv_scan_launch(float* a, const float* xx, const uint32_t* flags, long long n, int iters, void* ws,
                     hipStream_t s) {
    constexpr long long TILE = 1024LL * ROWS;
    const int tiles = (int)((n + TILE - 1) / TILE);
    static int bpc = persistent_blocks_per_cu(segscan_kernel<1, true, ROWS, PF, LB2, MULTI>, kScanThreads);
    const int grid = tiles < device_cu_count() * bpc ? tiles : device_cu_count() * bpc;
    unsigned* timeout = lb_host_timeout();
    if (!timeout) return (int)hipErrorOutOfMemory;
    if (iters >= (1 << 24)) return (int)hipErrorInvalidValue;  // epochs are 24-bit
    uint64_t* desc = lb_descriptors(ws);
    const size_t set_bytes = LB2 ? lb2_ws_bytes(tiles) : lb_ws_bytes(tiles);
    if constexpr (MULTI) {
        const long long stride = (long long)((set_bytes + 255) / 256 * 256 / sizeof(uint64_t));
        for (int it0 = 0; it0 < iters; it0 += kSpmvScanSteps) {
            const int k = iters - it0 < kSpmvScanSteps ? iters - it0 : kSpmvScanSteps;
            CME_TRY(hipMemsetAsync(ws, 0, 16 + k * stride * sizeof(uint64_t), s));
            hipLaunchKernelGGL((segscan_kernel<1, true, ROWS, PF, LB2, true>), dim3(grid), dim3(kScanThreads), 0, s, a,
                               xx, a, flags, n, desc, tiles, timeout, 1u, k, stride);
            CME_TRY(hipGetLastError());
        }
    } else {
        CME_TRY(hipMemsetAsync(ws, 0, set_bytes, s));
        for (int it = 0; it < iters; ++it)
            hipLaunchKernelGGL((segscan_kernel<1, true, ROWS, PF, LB2>), dim3(grid), dim3(kScanThreads), 0, s, a, xx,
                               a, flags, n, desc, tiles, timeout, (uint32_t)(it + 1), 1, 0LL);
    }
    CME_LAUNCH_STATUS();
}
}  // namespace
