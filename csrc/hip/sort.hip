// GPU sorting: LSD radix sort (8-bit digits) and merge-path merge sort.
//
// Parity: the hw4 OpenMP radix sort (hw/hw4/programming/radixsort.cpp:22-121:
// per-block histograms -> reduce -> exclusive scan -> push-down offsets ->
// per-block scatter) and merge sort (mergesort.cpp:31-144: recursive sort +
// parallel merge split at the median via upper_bound), moved to wave64.
//
// Radix pass (reduce-then-scan structure -- no in-launch hand-offs):
//   K1 upsweep  : block b histograms its contiguous chunk (LDS atomics) into
//                 counts[digit * nblocks + b]
//   K2 scan     : one block per digit scans that digit's row of counts over
//                 the blocks and writes the digit total (one small launch)
//   K3 downsweep: block b re-reads its chunk tile by tile (4096 keys); keys are
//                 ranked stably inside each wave with 8 ballots per item
//                 (wave64 "match"), waves are combined per digit in LDS, the
//                 tile is reordered by digit in LDS and written out so that
//                 consecutive lanes store consecutive addresses of a digit run.
//                 A running per-digit base in LDS carries the chunk across tiles;
//                 the block's digit bases are the scan of the 256 digit totals
//                 (done in its prologue) plus its own row prefixes.
// int32 / float32 keys are mapped to order-preserving uint32 codes by the
// first pass's loads and back by the last pass's stores (no extra kernels).
#include <stdlib.h>

#include "cme213/common.h"
#include "cme213/tuning.h"
#include "cme213/wave.h"

using namespace cme;

namespace {

constexpr int kRadixBits = 8;
constexpr int kBins = 1 << kRadixBits;
constexpr int kSortThreads = 256;
constexpr int kSortWaves = kSortThreads / kWave;
constexpr int kItems = 16;  // keys per lane per tile
constexpr int kSortTile = kSortThreads * kItems;  // 4096

__device__ __forceinline__ uint32_t digit_of(uint32_t k, int shift) { return (k >> shift) & (kBins - 1); }

// key codes: 0 uint32, 1 int32 (sign flip), 2 float32 (IEEE order flip)
__device__ __forceinline__ uint32_t rx_key_in(uint32_t k, int mode) {
    if (mode == 1) return k ^ 0x80000000u;
    if (mode == 2) return k ^ ((uint32_t)((int)k >> 31) | 0x80000000u);
    return k;
}
__device__ __forceinline__ uint32_t rx_key_out(uint32_t u, int mode) {
    if (mode == 1) return u ^ 0x80000000u;
    if (mode == 2) return u ^ (((uint32_t)((int)u >> 31) ^ 0xffffffffu) | 0x80000000u);
    return u;
}

__global__ __launch_bounds__(kSortThreads) void radix_upsweep_kernel(const uint32_t* __restrict__ keys, long long n,
                                                                     long long chunk, int shift, int nblocks,
                                                                     uint32_t* __restrict__ counts, int mode) {
    __shared__ uint32_t hist[kBins];
    for (int i = threadIdx.x; i < kBins; i += kSortThreads) hist[i] = 0;
    __syncthreads();
    const long long b0 = (long long)blockIdx.x * chunk;
    const long long b1 = b0 + chunk < n ? b0 + chunk : n;
    const bool vec = ((uintptr_t)keys & 15u) == 0;  // a tensor view may be 4-B aligned only
    auto add = [&](uint32_t k) { atomicAdd(&hist[digit_of(rx_key_in(k, mode), shift)], 1u); };
    // UNR 16-B loads in flight per lane before their LDS atomics (one load at
    // a time left the kernel waiting on HBM latency: wait-any 0.85 of its
    // cycles, profiles/sort_r3.md)
    constexpr int UNR = 4;
    constexpr long long STEP = (long long)kSortThreads * 4;
    long long i = b0 + threadIdx.x * 4;
    if (vec) {
        for (; i + (UNR - 1) * STEP + 3 < b1; i += UNR * STEP) {
            uint4 v[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) v[u] = *reinterpret_cast<const uint4*>(keys + i + u * STEP);
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                add(v[u].x);
                add(v[u].y);
                add(v[u].z);
                add(v[u].w);
            }
        }
    }
    for (; i < b1; i += STEP) {
        if (vec && i + 3 < b1) {
            const uint4 v = *reinterpret_cast<const uint4*>(keys + i);
            add(v.x);
            add(v.y);
            add(v.z);
            add(v.w);
        } else {
            for (long long j = i; j < b1 && j < i + 4; ++j) add(keys[j]);
        }
    }
    __syncthreads();
    for (int d = threadIdx.x; d < kBins; d += kSortThreads) counts[(size_t)d * nblocks + blockIdx.x] = hist[d];
}

// K2: block d scans row d of counts (nblocks <= kMaxRadixBlocks values, R
// consecutive per lane) in place to exclusive prefixes and writes the total
constexpr int kMaxRadixBlocks = 4096;
__global__ __launch_bounds__(1024) void radix_scan_kernel(uint32_t* __restrict__ counts, int nblocks,
                                                          uint32_t* __restrict__ totals) {
    constexpr int R = kMaxRadixBlocks / 1024;
    __shared__ uint32_t tmp[16];
    const int d = blockIdx.x, b0 = threadIdx.x * R;
    uint32_t* row = counts + (size_t)d * nblocks;
    uint32_t c[R], sum = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        c[r] = b0 + r < nblocks ? row[b0 + r] : 0u;
        sum += c[r];
    }
    uint32_t tot;
    uint32_t ex = block_exclusive_scan<16>(sum, tmp, tot, OpAdd());
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (b0 + r < nblocks) row[b0 + r] = ex;
        ex += c[r];
    }
    if (threadIdx.x == 0) totals[d] = tot;
}

// Stable rank of each lane's digit among the lanes of its wave (ballot match).
// Per bit: the lane's bit as an all-ones / zero mask (one signed bit-field
// extract), its ballot, and peers &= ~(ballot ^ mask) (keep the lanes whose
// bit agrees) -- an and-xnor of three operands, one gfx950 v_bitop3_b32 per
// 32-bit half, instead of a select between the ballot and its complement.
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid) {
    const uint64_t v = __ballot(valid);
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#pragma unroll
    for (int b = 0; b < kRadixBits; ++b) {
        uint32_t s;  // 0 or ~0: one signed bit-field extract (the compiler otherwise emits a shift pair)
        asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(s) : "v"(d), "i"(b));
        const uint64_t m = __ballot(s != 0u);
        // truth table of peers & ~(m ^ s) over (src0, src1, src2) = (0xf0, 0xcc, 0xaa)
        lo = __builtin_amdgcn_bitop3_b32(lo, (uint32_t)m, s, 0x90);
        hi = __builtin_amdgcn_bitop3_b32(hi, (uint32_t)(m >> 32), s, 0x90);
    }
    return ((uint64_t)hi << 32) | lo;
}

// ATOMIC_RANK: in-wave ranks through returning LDS atomics issued back to
// back (else one LDS read-then-write per item); PREFETCH: the next tile's keys
// load while this tile is reordered and stored (+16 VGPRs)
// DS_THREADS: 256 (4096-key tiles) or 512 (8192-key tiles: digit runs of ~32
// keys, i.e. fewer partially written lines per tile)
template <bool HAS_VALUES, bool ATOMIC_RANK = false, bool PREFETCH = true, int DS_THREADS = kSortThreads>
__global__ __launch_bounds__(DS_THREADS, DS_THREADS == 512 ? 2 : 1) void radix_downsweep_kernel(
    const uint32_t* __restrict__ keys_in, uint32_t* __restrict__ keys_out, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ vals_out, long long n, long long chunk, int shift, int nblocks,
    const uint32_t* __restrict__ prefix, const uint32_t* __restrict__ totals, int mode_in, int mode_out) {
    constexpr int kWavesD = DS_THREADS / kWave;
    constexpr int kTileD = DS_THREADS * kItems;
    static_assert(DS_THREADS >= kBins, "downsweep: one thread per digit");
    const int tid = threadIdx.x;
    __shared__ uint32_t s_keys[kTileD];
    __shared__ uint32_t s_vals[HAS_VALUES ? kTileD : 1];
    __shared__ uint32_t s_whist[kWavesD][kBins];  // per-wave running counts, then exclusive prefixes
    __shared__ uint32_t s_tile_off[kBins];            // exclusive prefix of tile digit counts
    __shared__ uint32_t s_base[kBins];                // global position of the next key of each digit
    __shared__ uint32_t s_gdiff[kBins];               // s_base - s_tile_off: tile index -> global position
    const int lane = lane_id();
    const int wid = threadIdx.x / kWave;
    const long long b0 = (long long)blockIdx.x * chunk;
    const long long b1 = b0 + chunk < n ? b0 + chunk : n;
    {  // digit bases: scan of the digit totals + this block's row prefix
        __shared__ uint32_t s_t[kWavesD];
        uint32_t tot;
        const uint32_t db = block_exclusive_scan<kWavesD>(tid < kBins ? totals[tid] : 0u, s_t, tot, OpAdd());
        if (tid < kBins) s_base[tid] = db + prefix[(size_t)tid * nblocks + blockIdx.x];
    }

    // warp-striped: item k of lane l = key t0 + wid*1024 + k*64 + l (memory order = (k, l));
    // the next tile's keys are loaded while this tile is reordered and stored
    uint32_t key[kItems], val[kItems], rank[kItems];
    // item k of this lane is a key iff k < nk (items are 64 keys apart)
    auto items_of = [&](long long t0) {
        const long long rem = b1 - (t0 + wid * (kWave * kItems) + lane);
        return rem <= 0 ? 0 : (rem >= (long long)kWave * kItems ? kItems : (int)((rem + kWave - 1) / kWave));
    };
    auto load_tile = [&](long long t0) {
        const long long base = t0 + wid * (kWave * kItems) + lane;
        const int nk = items_of(t0);
#pragma unroll
        for (int k = 0; k < kItems; ++k) {
            key[k] = k < nk ? keys_in[base + k * kWave] : 0xffffffffu;
            if constexpr (HAS_VALUES) val[k] = k < nk ? vals_in[base + k * kWave] : 0u;
        }
    };
    if (PREFETCH && b0 < b1) load_tile(b0);
    for (long long t0 = b0; t0 < b1; t0 += kTileD) {
        for (int d = threadIdx.x; d < kBins; d += DS_THREADS)
#pragma unroll
            for (int w = 0; w < kWavesD; ++w) s_whist[w][d] = 0;
        if (!PREFETCH) load_tile(t0);
        const int nk = items_of(t0);
        __syncthreads();
        if (mode_in) {  // every item: an invalid item's code is never ranked (outside the valid ballot)
#pragma unroll
            for (int k = 0; k < kItems; ++k) key[k] = rx_key_in(key[k], mode_in);
        }
        if constexpr (!ATOMIC_RANK) {
#pragma unroll
            for (int k = 0; k < kItems; ++k) {
                const bool ok = k < nk;
                const uint32_t d = digit_of(key[k], shift);
                const uint64_t peers = match_digit(d, ok);
                const uint32_t below = (uint32_t)__builtin_popcountll(peers & ((1ull << lane) - 1ull));
                const uint32_t prev = ok ? s_whist[wid][d] : 0u;
                rank[k] = ok ? prev + below : 0xffffffffu;
                // the lowest lane of each peer group publishes the new running count
                if (ok && below == 0) s_whist[wid][d] = prev + (uint32_t)__builtin_popcountll(peers);
                __builtin_amdgcn_sched_barrier(0);  // keep each item's ballots next to its LDS update
            }
        } else {
            // stable in-wave ranks: the lowest lane of each digit's peer group
            // adds the group size to the wave's running count with ONE returning
            // LDS atomic; the atomics of the 16 items issue back to back (one
            // wave's LDS operations execute in order, so item k sees items < k)
            // and their old values come back to the peers by a lane shuffle
            uint32_t old[kItems], lead[kItems];
#pragma unroll
            for (int k = 0; k < kItems; ++k) {
                const bool ok = k < nk;
                const uint32_t d = digit_of(key[k], shift);
                const uint64_t peers = match_digit(d, ok);
                const uint32_t below = (uint32_t)__builtin_popcountll(peers & ((1ull << lane) - 1ull));
                lead[k] = peers ? (uint32_t)__builtin_ctzll(peers) : (uint32_t)lane;
                old[k] = 0u;
                if (ok && below == 0) old[k] = atomicAdd(&s_whist[wid][d], (uint32_t)__builtin_popcountll(peers));
                rank[k] = ok ? below : 0xffffffffu;
                __builtin_amdgcn_sched_barrier(0);  // keep each item's ballots next to its atomic
            }
#pragma unroll
            for (int k = 0; k < kItems; ++k) {
                const uint32_t prev = (uint32_t)__shfl((int)old[k], (int)lead[k]);
                if (rank[k] != 0xffffffffu) rank[k] += prev;
            }
        }
        __syncthreads();
        // per digit: exclusive prefix across waves, tile totals, tile offsets
        for (int d = threadIdx.x; d < kBins; d += DS_THREADS) {
            uint32_t run = 0;
#pragma unroll
            for (int w = 0; w < kWavesD; ++w) {
                const uint32_t c = s_whist[w][d];
                s_whist[w][d] = run;
                run += c;
            }
            s_tile_off[d] = run;  // tile count (made exclusive below)
        }
        __syncthreads();
        // exclusive scan of the 256 tile counts (one value per thread)
        {
            __shared__ uint32_t s_tmp[kWavesD];
            uint32_t tot;
            const uint32_t c = tid < kBins ? s_tile_off[tid] : 0u;
            const uint32_t ex = block_exclusive_scan<kWavesD>(c, s_tmp, tot, OpAdd());
            __syncthreads();
            if (tid < kBins) {
                s_tile_off[tid] = ex;
                s_gdiff[tid] = s_base[tid] - ex;
            }
        }
        __syncthreads();
        // reorder the tile by digit in LDS
#pragma unroll
        for (int k = 0; k < kItems; ++k) {
            if (rank[k] != 0xffffffffu) {
                const uint32_t d = digit_of(key[k], shift);
                const uint32_t pos = s_tile_off[d] + s_whist[wid][d] + rank[k];
                s_keys[pos] = key[k];
                if constexpr (HAS_VALUES) s_vals[pos] = val[k];
            }
        }
        __syncthreads();
        if (PREFETCH && t0 + kTileD < b1) load_tile(t0 + kTileD);  // in flight during the stores
        const int tile_n = (int)((b1 - t0) < kTileD ? (b1 - t0) : kTileD);
        for (int i = threadIdx.x; i < tile_n; i += DS_THREADS) {
            const uint32_t k = s_keys[i];
            const uint32_t d = digit_of(k, shift);
            const uint32_t g = s_gdiff[d] + (uint32_t)i;
            keys_out[g] = rx_key_out(k, mode_out);
            if constexpr (HAS_VALUES) vals_out[g] = s_vals[i];
        }
        __syncthreads();
        // advance the per-digit bases by this tile's counts
        if (tid < kBins) {
            const int d = tid;
            const uint32_t next = d + 1 < kBins ? s_tile_off[d + 1] : (uint32_t)tile_n;
            s_base[d] += next - s_tile_off[d];
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------ merge sort
// Stable merge sort in two kernels (wave64, LDS-staged; the hw4 merge sort's
// median split + upper_bound merge, hw/hw4/programming/mergesort.cpp:31-144,
// becomes a merge-path split):
//   block sort : a 512-lane block sorts an 8192-key tile: 16 consecutive keys
//                per lane sorted in registers by odd-even transposition
//                (stable), then 9 rounds of merge path in LDS (runs of 16 ->
//                8192, A first on ties: stable; LDS padded one word per 16);
//   merge pass : output tile o (4096 keys) of a pass merging runs of L: the
//                block finds its two diagonal splits by a cooperative 128-ary
//                search (2 x 128 lanes, ~4 dependent rounds of global loads
//                instead of ~24), loads the A and B pieces into LDS with
//                coalesced loads, merges 16 outputs per lane from LDS and
//                stores the tile coalesced through LDS.
// Keys are uint32 codes (int32 / float32 mapped on the block sort's loads and
// back on the last pass's stores, as the radix sort does). Values optional.
constexpr int kMsThreads = 256;                  // merge pass: 4096-key output tiles
constexpr int kMsItems = 16;
constexpr int kMsTile = kMsThreads * kMsItems;    // 4096
constexpr int kBsThreads = 512;                   // block sort: 8192-key tiles (one pass fewer)
constexpr int kBsTile = kBsThreads * kMsItems;    // 8192

// LDS index padding: one pad word per 16, so lane t's run [16t, 16t+16)
// starts at bank 17t mod 32 -- the per-lane 16-strided accesses (lane-major
// loads/stores of register runs) are conflict-free (unpadded: 16-way)
__device__ __forceinline__ int lp(int i) { return i + (i >> 4); }
constexpr int lp_size(int n) { return n + n / 16; }

__device__ __forceinline__ uint32_t ms_key_in(uint32_t k, int mode) {
    if (mode == 1) return k ^ 0x80000000u;
    if (mode == 2) return k ^ ((uint32_t)((int)k >> 31) | 0x80000000u);
    return k;
}
__device__ __forceinline__ uint32_t ms_key_out(uint32_t u, int mode) {
    if (mode == 1) return u ^ 0x80000000u;
    if (mode == 2) return u ^ (((uint32_t)((int)u >> 31) ^ 0xffffffffu) | 0x80000000u);
    return u;
}

// merge-path split of diagonal `diag` between A[0, la) and B[0, lb):
// number of A elements among the first `diag` outputs, A first on ties
template <typename FA, typename FB>
__device__ __forceinline__ int ms_split(FA A, FB B, int la, int lb, int diag) {
    int lo = diag - lb > 0 ? diag - lb : 0, hi = diag < la ? diag : la;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (A(mid) <= B(diag - 1 - mid)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// sequential merge of kMsItems outputs from A = [a0, a0+la) / B = [b0, b0+lb)
// (logical LDS indices, padded on access) into registers
template <bool HAS_VALUES, int CAP>
__device__ __forceinline__ void ms_merge16(const uint32_t* sk, const uint32_t* sv, int a0, int la, int b0, int lb,
                                           int i, int j, uint32_t (&k)[kMsItems], uint32_t (&v)[kMsItems]) {
    uint32_t ka = i < la ? sk[lp(a0 + i)] : 0xffffffffu, kb = j < lb ? sk[lp(b0 + j)] : 0xffffffffu;
#pragma unroll
    for (int q = 0; q < kMsItems; ++q) {
        const bool take_a = j >= lb || (i < la && ka <= kb);
        k[q] = take_a ? ka : kb;
        if constexpr (HAS_VALUES) {
            const int x = take_a ? a0 + i : b0 + j;  // past both ends only on padding lanes
            v[q] = sv[lp(x < CAP ? x : CAP - 1)];
        }
        if (take_a) {
            ++i;
            ka = i < la ? sk[lp(a0 + i)] : 0xffffffffu;
        } else {
            ++j;
            kb = j < lb ? sk[lp(b0 + j)] : 0xffffffffu;
        }
    }
}

// coalesced tile store through LDS: lane t holds outputs [16t, 16t+16)
template <bool HAS_VALUES, int NT>
__device__ __forceinline__ void ms_store_tile(uint32_t* sk, uint32_t* sv, const uint32_t (&k)[kMsItems],
                                              const uint32_t (&v)[kMsItems], uint32_t* __restrict__ ko,
                                              uint32_t* __restrict__ vo, long long base, int cnt, int mode) {
    __syncthreads();  // every lane is done reading the tile in LDS
    const int t = threadIdx.x;
#pragma unroll
    for (int q = 0; q < kMsItems; ++q) {
        sk[lp(kMsItems * t + q)] = k[q];
        if constexpr (HAS_VALUES) sv[lp(kMsItems * t + q)] = v[q];
    }
    __syncthreads();
    for (int i = t; i < cnt; i += NT) {
        ko[base + i] = ms_key_out(sk[lp(i)], mode);
        if constexpr (HAS_VALUES) vo[base + i] = sv[lp(i)];
    }
}

template <bool HAS_VALUES>
__global__ __launch_bounds__(kBsThreads) void ms_block_sort_kernel(const uint32_t* __restrict__ ki,
                                                                   uint32_t* __restrict__ ko,
                                                                   const uint32_t* __restrict__ vi,
                                                                   uint32_t* __restrict__ vo, long long n,
                                                                   int mode_in, int mode_out) {
    __shared__ uint32_t sk[lp_size(kBsTile)];
    __shared__ uint32_t sv[HAS_VALUES ? lp_size(kBsTile) : 1];
    const int t = threadIdx.x;
    const long long base = (long long)blockIdx.x * kBsTile;
    const int cnt = (int)(n - base < kBsTile ? n - base : kBsTile);
    // coalesced load into LDS, then lane t takes keys [16t, 16t+16)
    for (int i = t; i < kBsTile; i += kBsThreads) {
        sk[lp(i)] = i < cnt ? ms_key_in(ki[base + i], mode_in) : 0xffffffffu;
        if constexpr (HAS_VALUES) sv[lp(i)] = i < cnt ? vi[base + i] : 0u;
    }
    __syncthreads();
    uint32_t k[kMsItems], v[kMsItems];
#pragma unroll
    for (int q = 0; q < kMsItems; ++q) {
        k[q] = sk[lp(kMsItems * t + q)];
        if constexpr (HAS_VALUES) v[q] = sv[lp(kMsItems * t + q)];
    }
    // odd-even transposition: swaps only strictly greater neighbours (stable);
    // padding keys (all ones) sit at the tile's end and stay behind real keys
#pragma unroll
    for (int r = 0; r < kMsItems; ++r) {
#pragma unroll
        for (int q = r & 1; q + 1 < kMsItems; q += 2) {
            if (k[q] > k[q + 1]) {
                const uint32_t x = k[q];
                k[q] = k[q + 1];
                k[q + 1] = x;
                if constexpr (HAS_VALUES) {
                    const uint32_t y = v[q];
                    v[q] = v[q + 1];
                    v[q + 1] = y;
                }
            }
        }
    }
    // merge rounds in LDS: runs of 16 << r
    for (int L = kMsItems; L < kBsTile; L <<= 1) {
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kMsItems; ++q) {
            sk[lp(kMsItems * t + q)] = k[q];
            if constexpr (HAS_VALUES) sv[lp(kMsItems * t + q)] = v[q];
        }
        __syncthreads();
        const int out0 = kMsItems * t;
        const int a0 = out0 & ~(2 * L - 1), b0 = a0 + L;
        const int diag = out0 - a0;
        const int i = ms_split([&](int x) { return sk[lp(a0 + x)]; }, [&](int x) { return sk[lp(b0 + x)]; }, L, L,
                               diag);
        ms_merge16<HAS_VALUES, kBsTile>(sk, sv, a0, L, b0, L, i, diag - i, k, v);
    }
    ms_store_tile<HAS_VALUES, kBsThreads>(sk, sv, k, v, ko, vo, base, cnt, mode_out);
}

// Cooperative merge-path search: the 128 lanes of `part` (waves 2*part and
// 2*part+1) narrow [lo, hi] 128-fold per round, one global load pair per
// lane, for a fixed `rounds` (uniform across the block: both parts pass the
// same barriers). Q(m) = A[m] <= B[diag-1-m] holds below the answer (A first
// on ties) and fails from it on; returns the answer.
__device__ __forceinline__ long long ms_coop_split(const uint32_t* __restrict__ A, const uint32_t* __restrict__ B,
                                                   long long la, long long lb, long long diag, int rounds,
                                                   uint64_t (*smask)[2]) {
    const int t = threadIdx.x, part = t >> 7, l = t & 127, w = (t >> 6) & 1;
    long long lo = diag - lb > 0 ? diag - lb : 0, hi = diag < la ? diag : la;
    for (int r = 0; r < rounds; ++r) {
        const long long step = (hi - lo + 127) / 128;
        const long long m = lo + (long long)l * step;
        const bool q = lo < hi && m < hi && A[m] <= B[diag - 1 - m];
        const uint64_t fails = __ballot(!q);
        if ((t & 63) == 0) smask[part][w] = fails;
        __syncthreads();
        const uint64_t f0 = smask[part][0], f1 = smask[part][1];
        const int f = f0 ? __builtin_ctzll(f0) : (f1 ? 64 + __builtin_ctzll(f1) : 128);
        __syncthreads();
        if (lo < hi) {
            const long long nlo = f == 0 ? lo : lo + (long long)(f - 1) * step + 1;
            const long long mf = lo + (long long)f * step;
            const long long nhi = f == 128 ? hi : (mf < hi ? mf : hi);
            lo = nlo;
            hi = nhi;
        }
    }
    return lo;
}

template <bool HAS_VALUES>
__global__ __launch_bounds__(kMsThreads) void ms_merge_pass_kernel(const uint32_t* __restrict__ ki,
                                                                   uint32_t* __restrict__ ko,
                                                                   const uint32_t* __restrict__ vi,
                                                                   uint32_t* __restrict__ vo, long long n,
                                                                   long long L, int mode_out) {
    __shared__ uint32_t sk[lp_size(kMsTile)];
    __shared__ uint32_t sv[HAS_VALUES ? lp_size(kMsTile) : 1];
    __shared__ uint64_t smask[2][2];
    __shared__ long long ssplit[2];
    const int t = threadIdx.x;
    // consecutive output tiles on one XCD: their diagonal searches probe the
    // same lines of A and B, which then hit that XCD's L2
    const long long o0 = (long long)xcd_remap(blockIdx.x, gridDim.x) * kMsTile;
    const long long o1 = o0 + kMsTile < n ? o0 + kMsTile : n;
    const long long a0 = o0 & ~(2 * L - 1);  // pair start (2L is a multiple of the tile)
    const long long la = a0 + L < n ? L : n - a0;
    const long long lb = a0 + 2 * L < n ? L : (n - a0 - la > 0 ? n - a0 - la : 0);
    const uint32_t* A = ki + a0;
    const uint32_t* B = ki + a0 + la;
    const int part = t >> 7;
    const long long diag = (part == 0 ? o0 : o1) - a0;
    int rounds = 0;  // ceil(log_128(L + 1)): candidates per search <= L + 1
    for (long long w = L + 1; w > 1; w = (w + 127) / 128) ++rounds;
    const long long sp = ms_coop_split(A, B, la, lb, diag, rounds, smask);
    if ((t & 127) == 0) ssplit[part] = sp;
    __syncthreads();
    const long long i0 = ssplit[0], i1 = ssplit[1];
    const long long j0 = (o0 - a0) - i0, j1 = (o1 - a0) - i1;
    int na = (int)(i1 - i0), nb = (int)(j1 - j0);
    if (na < 0 || nb < 0 || na + nb > kMsTile || i1 > la || j1 > lb) na = nb = 0;  // never out of range
    for (int x = t; x < na + nb; x += kMsThreads) {
        const bool ia = x < na;
        const long long g = ia ? a0 + i0 + x : a0 + la + j0 + (x - na);
        sk[lp(x)] = ki[g];
        if constexpr (HAS_VALUES) sv[lp(x)] = vi[g];
    }
    __syncthreads();
    const int cnt = na + nb;
    const int diag_l = kMsItems * t < cnt ? kMsItems * t : cnt;
    const int i = ms_split([&](int x) { return sk[lp(x)]; }, [&](int x) { return sk[lp(na + x)]; }, na, nb, diag_l);
    uint32_t k[kMsItems], v[kMsItems];
    ms_merge16<HAS_VALUES, kMsTile>(sk, sv, 0, na, na, nb, i, diag_l - i, k, v);
    ms_store_tile<HAS_VALUES, kMsThreads>(sk, sv, k, v, ko, vo, o0, cnt, mode_out);
}

}  // namespace

// blocks of the upsweep / downsweep grid: at most 1024 (4 per CU), each
// walking several 4096-key tiles -- measured on MI355X, 16M keys: 0.357 /
// 0.363 / 0.391 ms at caps 1024 / 2048 / 4096 (48M: 1.18 / 1.13 / 1.14).
// CME_RADIX_MAXBLOCKS overrides the cap (<= kMaxRadixBlocks, sweeps).
static int radix_max_blocks() {
    const long x = cme::tune_get(cme::kTuneRadixMaxBlocks);
    return x < 1 ? 1 : (x > kMaxRadixBlocks ? kMaxRadixBlocks : (int)x);
}

CME_EXPORT long long cme_radix_ws_bytes(long long n) {
    long long tiles = (n + kSortTile - 1) / kSortTile;
    long long nb = tiles < kMaxRadixBlocks ? tiles : kMaxRadixBlocks;
    return nb * kBins * 4 + kBins * 4 + 256;
}

// LSD radix sort of n keys from `in` (not modified) into `out` over bits
// [bit0, bit1), ping-ponging through `tmp` so that the last pass writes out;
// values (optional) likewise. mode: 0 uint32, 1 int32, 2 float32 keys.
// ws: cme_radix_ws_bytes(n) bytes.
// downsweep variant (CME_RADIX_DS, for A/B sweeps): bit 0 atomic ranks, bit 1
// prefetch, bit 2 8192-key tiles (512 threads). Default 2: the four arms are within 3 % of each other at 16M keys
// (0.348-0.357 ms; the ranking's LDS round trips are not what binds), the
// prefetch without atomic ranks is best at 48M (0.956 vs 0.981 ms;
// profiles/sort_r3.md)
static int radix_ds_variant() { return (int)(cme::tune_get(cme::kTuneRadixDS) & 7); }

CME_EXPORT int cme_radix_sort(const uint32_t* in, uint32_t* out, uint32_t* tmp, const uint32_t* vin, uint32_t* vout,
                              uint32_t* vtmp, long long n, int mode, int bit0, int bit1, void* ws, void* stream) {
    hipStream_t s = as_stream(stream);
    if (n <= 0) return 0;
    if (bit0 < 0 || bit1 > 32 || bit1 <= bit0 || mode < 0 || mode > 2 || (vin != nullptr) != (vout != nullptr) ||
        (vin && !vtmp) || n >= (1ll << 32))
        return (int)hipErrorInvalidValue;
    const int dsv = radix_ds_variant();
    const bool wide = (dsv & 4) != 0;  // 8192-key downsweep tiles
    const long long dtile = wide ? 2 * kSortTile : kSortTile;
    const long long tiles = (n + dtile - 1) / dtile;
    const int cap = radix_max_blocks();
    int nb = tiles < cap ? (int)tiles : cap;
    const long long chunk = ((tiles + nb - 1) / nb) * dtile;
    nb = (int)((n + chunk - 1) / chunk);
    uint32_t* counts = (uint32_t*)ws;
    uint32_t* totals = counts + (size_t)nb * kBins;
    const int npass = (bit1 - bit0 + kRadixBits - 1) / kRadixBits;
    const uint32_t* ki = in;
    const uint32_t* vi = vin;
    for (int p = 0; p < npass; ++p) {
        const bool to_out = ((npass - 1 - p) & 1) == 0;  // the last pass lands in out
        uint32_t* ko = to_out ? out : tmp;
        uint32_t* vo = vin ? (to_out ? vout : vtmp) : nullptr;
        const int shift = bit0 + kRadixBits * p;
        const int mi = p == 0 ? mode : 0, mo = p == npass - 1 ? mode : 0;
        hipLaunchKernelGGL(radix_upsweep_kernel, dim3(nb), dim3(kSortThreads), 0, s, ki, n, chunk, shift, nb, counts,
                           mi);
        hipLaunchKernelGGL(radix_scan_kernel, dim3(kBins), dim3(1024), 0, s, counts, nb, totals);
#define CME_DS(V, A, P)                                                                                           \
    do {                                                                                                          \
        if (wide)                                                                                                 \
            hipLaunchKernelGGL((radix_downsweep_kernel<V, A, P, 512>), dim3(nb), dim3(512), 0, s, ki, ko, vi, vo, n, \
                               chunk, shift, nb, counts, totals, mi, mo);                                         \
        else                                                                                                      \
            hipLaunchKernelGGL((radix_downsweep_kernel<V, A, P>), dim3(nb), dim3(kSortThreads), 0, s, ki, ko, vi,  \
                               vo, n, chunk, shift, nb, counts, totals, mi, mo);                                  \
    } while (0)
        if (vin) {
            if (dsv == 0) CME_DS(true, false, false);
            else if (dsv == 1) CME_DS(true, true, false);
            else if (dsv == 2) CME_DS(true, false, true);
            else CME_DS(true, true, true);
        } else {
            if (dsv == 0) CME_DS(false, false, false);
            else if (dsv == 1) CME_DS(false, true, false);
            else if (dsv == 2) CME_DS(false, false, true);
            else CME_DS(false, true, true);
        }
#undef CME_DS
        CME_TRY(hipGetLastError());
        ki = ko;
        vi = vo;
    }
    return 0;
}

// In-place form (sorted uint32 keys left in `keys`; keys_alt / vals_alt scratch).
CME_EXPORT int cme_radix_sort_u32(uint32_t* keys, uint32_t* keys_alt, uint32_t* vals, uint32_t* vals_alt, long long n,
                                  int bit0, int bit1, void* ws, void* stream) {
    if (n <= 1) return 0;
    const int npass = (bit1 - bit0 + kRadixBits - 1) / kRadixBits;
    if (npass & 1) {  // odd: sort into keys_alt, copy back
        int rc = cme_radix_sort(keys, keys_alt, keys, vals, vals ? vals_alt : nullptr, vals, n, 0, bit0, bit1, ws,
                                stream);
        if (rc) return rc;
        CME_TRY(hipMemcpyAsync(keys, keys_alt, n * 4, hipMemcpyDeviceToDevice, as_stream(stream)));
        if (vals) CME_TRY(hipMemcpyAsync(vals, vals_alt, n * 4, hipMemcpyDeviceToDevice, as_stream(stream)));
        return 0;
    }
    return cme_radix_sort(keys, keys, keys_alt, vals, vals, vals_alt, n, 0, bit0, bit1, ws, stream);
}

// Stable merge sort of n keys from `in` into `out` (ping-pong through `tmp`;
// `in` may equal `out`; values optional, likewise). mode: 0 uint32, 1 int32,
// 2 float32 keys.
CME_EXPORT int cme_merge_sort(const uint32_t* in, uint32_t* out, uint32_t* tmp, const uint32_t* vin, uint32_t* vout,
                              uint32_t* vtmp, long long n, int mode, void* stream) {
    hipStream_t s = as_stream(stream);
    if (n <= 0) return 0;
    if (mode < 0 || mode > 2 || (vin != nullptr) != (vout != nullptr) || (vin && !vtmp))
        return (int)hipErrorInvalidValue;
    int npass = 0;
    for (long long L = kBsTile; L < n; L <<= 1) ++npass;
    // the block sort writes where an even number of passes later lands in out
    uint32_t* d0 = (npass & 1) ? tmp : out;
    uint32_t* v0 = vin ? ((npass & 1) ? vtmp : vout) : nullptr;
    const unsigned btiles = cdiv(n, kBsTile), tiles = cdiv(n, kMsTile);
    if (vin)
        hipLaunchKernelGGL(ms_block_sort_kernel<true>, dim3(btiles), dim3(kBsThreads), 0, s, in, d0, vin, v0, n, mode,
                           npass ? 0 : mode);
    else
        hipLaunchKernelGGL(ms_block_sort_kernel<false>, dim3(btiles), dim3(kBsThreads), 0, s, in, d0, vin, v0, n,
                           mode, npass ? 0 : mode);
    CME_TRY(hipGetLastError());
    const uint32_t *ki = d0, *vi = v0;
    int p = 0;
    for (long long L = kBsTile; L < n; L <<= 1, ++p) {
        const bool last = p == npass - 1;
        uint32_t* ko = (ki == out) ? tmp : out;
        uint32_t* vo = vin ? ((vi == vout) ? vtmp : vout) : nullptr;
        if (vin)
            hipLaunchKernelGGL(ms_merge_pass_kernel<true>, dim3(tiles), dim3(kMsThreads), 0, s, ki, ko, vi, vo, n, L,
                               last ? mode : 0);
        else
            hipLaunchKernelGGL(ms_merge_pass_kernel<false>, dim3(tiles), dim3(kMsThreads), 0, s, ki, ko, vi, vo, n,
                               L, last ? mode : 0);
        CME_TRY(hipGetLastError());
        ki = ko;
        vi = vo;
    }
    return 0;
}

// In-place form (keys sorted into `keys`; keys_alt / vals_alt scratch).
CME_EXPORT int cme_merge_sort_u32(uint32_t* keys, uint32_t* keys_alt, uint32_t* vals, uint32_t* vals_alt, long long n,
                                  void* stream) {
    return cme_merge_sort(keys, keys, keys_alt, vals, vals, vals_alt, n, 0, stream);
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(radix_upsweep, 256, radix_upsweep_kernel);
CME_REGISTER_KERNEL(radix_downsweep_kv, 256, radix_downsweep_kernel<true>);
CME_REGISTER_KERNEL(ms_block_sort, 512, ms_block_sort_kernel<false>);
CME_REGISTER_KERNEL(ms_merge_pass, 256, ms_merge_pass_kernel<false>);
