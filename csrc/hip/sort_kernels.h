// Kernels and the host schedule of the GPU sorts (entry points: sort.hip
// production, hip_tune/sort_tune.hip tuning arms).
#pragma once
#include <stdlib.h>

#include <atomic>
#include <type_traits>

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

template <int UNR, bool kUpVecCheck = true>
__global__ __launch_bounds__(kSortThreads) void radix_upsweep_kernel(const uint32_t* __restrict__ keys, long long n,
                                                                     long long chunk, int shift, int nblocks,
                                                                     uint32_t* __restrict__ counts, int mode) {
    __shared__ uint32_t hist[kBins];
    for (int i = threadIdx.x; i < kBins; i += kSortThreads) hist[i] = 0;
    __syncthreads();
    const long long b0 = (long long)blockIdx.x * chunk;
    const long long b1 = b0 + chunk < n ? b0 + chunk : n;
    const bool vec = ((uintptr_t)keys & 15u) == 0;  // a tensor view may be 4-B aligned only
    // same-address lanes of one LDS atomic serialise (86 cycles per wave
    // instruction when all 64 share a digit: the high digits of small keys),
    // so a wave whose active lanes share one digit adds once
    const int lane = lane_id();
    auto add = [&](uint32_t k) {
        const uint32_t d = digit_of(rx_key_in(k, mode), shift);
        const uint32_t d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)d);
        if (__ballot(d != d0) == 0) {
            const uint64_t act = __ballot(true);
            if (lane == (int)__builtin_ctzll(act)) atomicAdd(&hist[d0], (uint32_t)__builtin_popcountll(act));
        } else {
            atomicAdd(&hist[d], 1u);
        }
    };
    // the four keys of a 16-B load: ONE uniformity check for all of them (the
    // wave's 256 consecutive keys), then either one atomic or four plain ones
    auto add4 = [&](uint4 v) {
        if (!kUpVecCheck) {
            add(v.x);
            add(v.y);
            add(v.z);
            add(v.w);
            return;
        }
        const uint32_t dx = digit_of(rx_key_in(v.x, mode), shift), dy = digit_of(rx_key_in(v.y, mode), shift);
        const uint32_t dz = digit_of(rx_key_in(v.z, mode), shift), dw = digit_of(rx_key_in(v.w, mode), shift);
        const uint32_t d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)dx);
        if (__ballot((dx ^ d0) | (dy ^ d0) | (dz ^ d0) | (dw ^ d0)) == 0) {
            const uint64_t act = __ballot(true);
            if (lane == (int)__builtin_ctzll(act)) atomicAdd(&hist[d0], 4u * (uint32_t)__builtin_popcountll(act));
        } else {
            atomicAdd(&hist[dx], 1u);
            atomicAdd(&hist[dy], 1u);
            atomicAdd(&hist[dz], 1u);
            atomicAdd(&hist[dw], 1u);
        }
    };
    // UNR 16-B loads in flight per lane before their LDS atomics (one load at
    // a time left the kernel waiting on HBM latency: wait-any 0.85 of its
    // cycles, profiles/sort_r3.md); tuning knob radix_up_unr
    constexpr long long STEP = (long long)kSortThreads * 4;
    long long i = b0 + threadIdx.x * 4;
    if (vec) {
        for (; i + (UNR - 1) * STEP + 3 < b1; i += UNR * STEP) {
            uint4 v[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) v[u] = *reinterpret_cast<const uint4*>(keys + i + u * STEP);
#pragma unroll
            for (int u = 0; u < UNR; ++u) add4(v[u]);
        }
    }
    for (; i < b1; i += STEP) {
        if (vec && i + 3 < b1) {
            add4(*reinterpret_cast<const uint4*>(keys + i));
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

// In-wave rank kinds of the downsweep:
//   kRankMatch  : ballot match (match_digit) + one LDS read-then-write per item
//   kRankGroup  : ballot match + one returning LDS atomic per peer group
//   kRankLanes  : one returning LDS atomic per LANE, no match. The lanes of a
//                 wave-wide ds_add_rtn_u32 that hit one address are applied in
//                 lane order (gfx950 LDS; benchmarks/probe_lds_atomic_order.hip:
//                 1.29e9 lanes over 1-256 distinct digits and masked lanes, none
//                 out of order), so lane l's old value counts the lower lanes of
//                 its digit: a stable rank in one LDS instruction instead of ~40
//                 VALU instructions per key. Same-address lanes serialise (86
//                 cycles per wave-instruction at one digit, 6 at 256), so a wave
//                 whose valid keys share one digit (the high digit of small
//                 keys, sorted runs) takes one atomic for the whole group.
//                 The library checks the lane order once per device before it
//                 uses this kind (cme_radix_lane_order_probe) and falls back to
//                 kRankMatch where the check fails.
enum RadixRank { kRankMatch = 0, kRankGroup = 1, kRankLanes = 2 };

// PREFETCH: the next tile's keys load while this tile is reordered and stored
// (+16 VGPRs). DS_THREADS: 256 (4096-key tiles) or 512 (8192-key tiles: digit
// runs of ~32 keys, i.e. fewer partially written lines per tile)
template <bool HAS_VALUES, int RANK = kRankMatch, bool PREFETCH = true, int DS_THREADS = kSortThreads>
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
    __shared__ int s_identity;
    {  // digit bases: scan of the digit totals + this block's row prefix
        __shared__ uint32_t s_t[kWavesD];
        uint32_t tot;
        const uint32_t td = tid < kBins ? totals[tid] : 0u;
        if (tid == 0) s_identity = 0;
        const uint32_t db = block_exclusive_scan<kWavesD>(td, s_t, tot, OpAdd());
        if (tid < kBins) s_base[tid] = db + prefix[(size_t)tid * nblocks + blockIdx.x];
        if (tid < kBins && td == (uint32_t)n) s_identity = 1;  // every key has this digit
        lds_bcast_sync();
    }
    if (s_identity) {
        // one digit holds every key: the stable pass is the identity
        // permutation (the high digits of small keys) -- a straight copy,
        // with the first / last pass's key transforms
        constexpr int U = 8;
        long long i = b0 + tid;
        for (; i + (U - 1) * DS_THREADS < b1; i += U * DS_THREADS) {
            uint32_t k[U], v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                k[u] = keys_in[i + u * DS_THREADS];
                if constexpr (HAS_VALUES) v[u] = vals_in[i + u * DS_THREADS];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                keys_out[i + u * DS_THREADS] = rx_key_out(rx_key_in(k[u], mode_in), mode_out);
                if constexpr (HAS_VALUES) vals_out[i + u * DS_THREADS] = v[u];
            }
        }
        for (; i < b1; i += DS_THREADS) {
            keys_out[i] = rx_key_out(rx_key_in(keys_in[i], mode_in), mode_out);
            if constexpr (HAS_VALUES) vals_out[i] = vals_in[i];
        }
        return;
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
        if constexpr (RANK == kRankLanes) {
#pragma unroll
            for (int k = 0; k < kItems; ++k) {
                const bool ok = k < nk;
                const uint32_t d = digit_of(key[k], shift);
                const uint64_t act = __ballot(ok);
                if (act == 0) {
                    rank[k] = 0xffffffffu;
                    continue;
                }
                const int first = (int)__builtin_ctzll(act);
                const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane((int)d, first);
                if (__ballot(ok && d != d0) == 0) {  // one digit: one atomic, ranks by lane count
                    uint32_t base = 0;
                    if (lane == first) base = atomicAdd(&s_whist[wid][d0], (uint32_t)__builtin_popcountll(act));
                    base = (uint32_t)__builtin_amdgcn_readlane((int)base, first);
                    const uint32_t below = (uint32_t)__builtin_popcountll(act & ((1ull << lane) - 1ull));
                    rank[k] = ok ? base + below : 0xffffffffu;
                } else {
                    uint32_t old = 0xffffffffu;
                    if (ok) old = atomicAdd(&s_whist[wid][d], 1u);
                    rank[k] = old;
                }
            }
        } else if constexpr (RANK == kRankMatch) {
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
                // fold the tile offset into every wave's prefix: one LDS read per key below
#pragma unroll
                for (int w = 0; w < kWavesD; ++w) s_whist[w][tid] += ex;
            }
        }
        __syncthreads();
        // reorder the tile by digit in LDS
#pragma unroll
        for (int k = 0; k < kItems; ++k) {
            if (rank[k] != 0xffffffffu) {
                const uint32_t d = digit_of(key[k], shift);
                const uint32_t pos = s_whist[wid][d] + rank[k];
                s_keys[pos] = key[k];
                if constexpr (HAS_VALUES) s_vals[pos] = val[k];
            }
        }
        __syncthreads();
        if (PREFETCH && t0 + kTileD < b1) load_tile(t0 + kTileD);  // in flight during the stores
        const int tile_n = (int)((b1 - t0) < kTileD ? (b1 - t0) : kTileD);
        // the key transform only on the last pass (a uniform branch: the
        // branch-free select chain cost ~5 VALU per key on every pass)
        auto store_tile = [&](int mo) {
            for (int i = threadIdx.x; i < tile_n; i += DS_THREADS) {
                const uint32_t k = s_keys[i];
                const uint32_t d = digit_of(k, shift);
                const uint32_t g = s_gdiff[d] + (uint32_t)i;
                keys_out[g] = mo ? rx_key_out(k, mo) : k;
                if constexpr (HAS_VALUES) vals_out[g] = s_vals[i];
            }
        };
        if (mode_out == 0)
            store_tile(0);
        else
            store_tile(mode_out);
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
//                block takes its two diagonal splits from the pass's
//                partition launch (ms_partition_kernel, 8 lanes per tile;
//                from 8M keys) or finds them by a cooperative 128-ary
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

// LDS word i of a padded buffer, the byte offset (i + i / 16) * 4 written out
// so that it folds into one v_add_lshl_u32
__device__ __forceinline__ uint32_t ldsw(const uint32_t* sk, int i) {
    return *(const uint32_t*)((const char*)sk + ((unsigned)(i + (i >> 4)) << 2));
}

// The same split by binary lifting: halving steps from smax, a power of two
// with 2 smax - 1 >= the search range (uniform across the block, so the loop
// is scalar: no divergent trip counts, no exec bookkeeping). Step st tries to
// move lo past st more candidates; a probe beyond the range counts as false
// and reads a clamped in-range index. ~11 VALU per step against ~17 plus the
// loop's exec masks for the bisection (profiles/sort_r6.md).
__device__ __forceinline__ int ms_split_lift(const uint32_t* sk, int a0, int la, int b0, int lb, int diag, int smax) {
    const int lo0 = diag - lb > 0 ? diag - lb : 0, hi0 = diag < la ? diag : la;
    const int kb = b0 + diag - 1;
    int lo = lo0;
    for (int st = smax; st > 0; st >>= 1) {
        const int m = lo + st - 1;
        const int mc = max(min(m, hi0 - 1), 0);
        const bool q = m < hi0 && ldsw(sk, a0 + mc) <= ldsw(sk, kb - mc);
        lo = q ? m + 1 : lo;
    }
    return lo;
}

// the smax of ms_split_lift for runs of la and lb keys (block-uniform)
__device__ __forceinline__ int ms_lift_top(int la, int lb) {
    const int r = la < lb ? la : lb;  // a diagonal's candidates span at most min(la, lb) + 1
    return __builtin_amdgcn_readfirstlane(r > 0 ? 1 << (31 - __builtin_clz(r)) : 0);
}

// sequential merge of kMsItems outputs from A = [a0, a0+la) / B = [b0, b0+lb)
// (logical LDS indices, padded on access) into registers. Branch-free: every
// step selects its output, advances one of the two cursors and loads that
// run's next key (a cursor never passes its run's end, at most CAP: the
// buffers hold CAP + 1 padded slots), so no lane diverges -- the divergent form spent more issue
// slots on exec-mask bookkeeping than on the merge.
template <bool HAS_VALUES, int CAP>
__device__ __forceinline__ void ms_merge16(const uint32_t* sk, const uint32_t* sv, int a0, int la, int b0, int lb,
                                           int i, int j, uint32_t (&k)[kMsItems], uint32_t (&v)[kMsItems]) {
    int pa = a0 + i, pb = b0 + j;  // cursors (logical indices; pa <= ea <= CAP, pb <= eb <= CAP)
    const int ea = a0 + la, eb = b0 + lb;
    uint32_t ka = sk[lp(pa)], kb = sk[lp(pb)];
    ka = pa < ea ? ka : 0xffffffffu;
    kb = pb < eb ? kb : 0xffffffffu;
    if constexpr (!HAS_VALUES) {
        // Keys only: equal keys are indistinguishable, so the step takes
        // min(ka, kb) and advances A on ka <= kb with no bounds test. An
        // exhausted run reads as all-ones; if the other run's key is all-ones
        // too, every remaining output is all-ones whichever cursor moves (a
        // cursor past its end keeps reading all-ones through the guard). 12
        // VALU per step instead of ~19 (profiles/sort_r6.md).
#pragma unroll
        for (int q = 0; q < kMsItems; ++q) {
            const bool take_a = ka <= kb;
            k[q] = min(ka, kb);
            pa += take_a ? 1 : 0;
            pb += take_a ? 0 : 1;
            const int np = take_a ? pa : pb;
            // byte offset (np + np / 16) * 4 written out, so it folds into one v_add_lshl_u32
            uint32_t nv = *(const uint32_t*)((const char*)sk + ((unsigned)(np + (np >> 4)) << 2));
            nv = np < (take_a ? ea : eb) ? nv : 0xffffffffu;
            ka = take_a ? nv : ka;
            kb = take_a ? kb : nv;
        }
        return;
    }
#pragma unroll
    for (int q = 0; q < kMsItems; ++q) {
        const bool take_a = pb >= eb || (pa < ea && ka <= kb);
        k[q] = take_a ? ka : kb;
        if constexpr (HAS_VALUES) {
            const int x = take_a ? pa : pb;  // past both ends only on padding lanes
            v[q] = sv[lp(x < CAP ? x : CAP - 1)];
        }
        pa += take_a ? 1 : 0;
        pb += take_a ? 0 : 1;
        const int np = take_a ? pa : pb;  // <= CAP: the spare slot at most
        const int ne = take_a ? ea : eb;
        uint32_t nv = sk[lp(np)];
        nv = np < ne ? nv : 0xffffffffu;
        ka = take_a ? nv : ka;
        kb = take_a ? kb : nv;
    }
}

// Run samples of a pass's output for the next pass's partition search: the
// first and the last key (uint32 codes) of every `st`-key tile of the array.
struct MsSamples {
    uint32_t* first;  // nullptr: none written
    uint32_t* last;
    int st;
};

// coalesced tile store through LDS: lane t holds outputs [16t, 16t+16); also
// records the tile's samples (smp.first != nullptr, block-uniform)
template <bool HAS_VALUES, int NT>
__device__ __forceinline__ void ms_store_tile(uint32_t* sk, uint32_t* sv, const uint32_t (&k)[kMsItems],
                                              const uint32_t (&v)[kMsItems], uint32_t* __restrict__ ko,
                                              uint32_t* __restrict__ vo, long long base, int cnt, int mode,
                                              MsSamples smp) {
    __syncthreads();  // every lane is done reading the tile in LDS
    const int t = threadIdx.x;
#pragma unroll
    for (int q = 0; q < kMsItems; ++q) {
        sk[lp(kMsItems * t + q)] = k[q];
        if constexpr (HAS_VALUES) sv[lp(kMsItems * t + q)] = v[q];
    }
    __syncthreads();
    if (smp.first) {
        const int nq = (cnt + smp.st - 1) / smp.st;
        for (int q = t; q < nq; q += NT) {
            const long long g = base / smp.st + q;
            const int e = (q + 1) * smp.st < cnt ? (q + 1) * smp.st : cnt;
            smp.first[g] = sk[lp(q * smp.st)];
            smp.last[g] = sk[lp(e - 1)];
        }
    }
    // coalesced stores, unrolled: lane t writes t + q*NT (LDS word lp(t) +
    // q*(NT + NT/16), immediate offsets), the key transform a compile-time
    // branch (the dynamic loop with a run-time transform cost ~12 VALU per key)
    auto out = [&](auto md) {
        constexpr int MD = decltype(md)::value;
        const bool al16 = ((reinterpret_cast<uintptr_t>(ko + base) |
                            (HAS_VALUES ? reinterpret_cast<uintptr_t>(vo + base) : 0)) & 15) == 0;
        if (cnt == NT * kMsItems && al16) {  // (the C API's in-place forms may hand in any 4-B aligned array)
            // a full tile: four consecutive keys per lane and store, 16 B
            // (lane t takes keys 4(t + q NT) .. +3: one 16-key LDS group, so
            // four contiguous padded words), a quarter of the store instructions
#pragma unroll
            for (int q = 0; q < kMsItems / 4; ++q) {
                const int i = 4 * (t + q * NT);
                const int w = lp(i);
                uint4 o{ms_key_out(sk[w], MD), ms_key_out(sk[w + 1], MD), ms_key_out(sk[w + 2], MD),
                        ms_key_out(sk[w + 3], MD)};
                *reinterpret_cast<uint4*>(ko + base + i) = o;
                if constexpr (HAS_VALUES)
                    *reinterpret_cast<uint4*>(vo + base + i) = uint4{sv[w], sv[w + 1], sv[w + 2], sv[w + 3]};
            }
            return;
        }
        const int lt = lp(t);
#pragma unroll
        for (int q = 0; q < kMsItems; ++q) {
            const int i = t + q * NT;
            if (i < cnt) {
                ko[base + i] = ms_key_out(sk[lt + q * (NT + NT / 16)], MD);
                if constexpr (HAS_VALUES) vo[base + i] = sv[lt + q * (NT + NT / 16)];
            }
        }
    };
    if (mode == 0) out(std::integral_constant<int, 0>());
    else if (mode == 1) out(std::integral_constant<int, 1>());
    else out(std::integral_constant<int, 2>());
}

template <bool HAS_VALUES, int BS = kBsThreads>
__global__ __launch_bounds__(BS) void ms_block_sort_kernel(const uint32_t* __restrict__ ki, uint32_t* __restrict__ ko,
                                                           const uint32_t* __restrict__ vi, uint32_t* __restrict__ vo,
                                                           long long n, int mode_in, int mode_out, MsSamples smp) {
    constexpr int BTILE = BS * kMsItems;
    __shared__ uint32_t sk[lp_size(BTILE) + 1];  // + the merge's out-of-run load slot
    __shared__ uint32_t sv[HAS_VALUES ? lp_size(BTILE) : 1];
    const int t = threadIdx.x;
    const long long base = (long long)blockIdx.x * BTILE;
    const int cnt = (int)(n - base < BTILE ? n - base : BTILE);
    // coalesced load into LDS, then lane t takes keys [16t, 16t+16)
    for (int i = t; i < BTILE; i += BS) {
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
            if constexpr (HAS_VALUES) {
                if (k[q] > k[q + 1]) {
                    const uint32_t x = k[q];
                    k[q] = k[q + 1];
                    k[q + 1] = x;
                    const uint32_t y = v[q];
                    v[q] = v[q + 1];
                    v[q + 1] = y;
                }
            } else {  // equal keys are indistinguishable: min / max, no compare-select
                const uint32_t lo = min(k[q], k[q + 1]), hi = max(k[q], k[q + 1]);
                k[q] = lo;
                k[q + 1] = hi;
            }
        }
    }
    // merge rounds in LDS: runs of 16 << r
    for (int L = kMsItems; L < BTILE; L <<= 1) {
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
        ms_merge16<HAS_VALUES, BTILE>(sk, sv, a0, L, b0, L, i, diag - i, k, v);
    }
    ms_store_tile<HAS_VALUES, BS>(sk, sv, k, v, ko, vo, base, cnt, mode_out, smp);
}

// Keys-only block sort by LSD radix in LDS (the base case of the merge sort,
// as the hw4 merge sort hands blocks below its threshold to std::sort,
// hw/hw4/programming/mergesort.cpp:80-84): a 1024-lane block sorts its
// 16384-key tile with four 8-bit digit passes that never leave LDS. Per pass
// every wave ranks its 1024 keys stably (items in (k, lane) order: one
// returning LDS atomic per key, or the ballot match where the device fails the
// lane-order check -- the radix downsweep's two ranking kinds), the 16 waves'
// digit counts become per-(wave, digit) bases (column prefix + block scan of
// the 256 digit totals), and the keys scatter to their digit positions. ~20
// VALU per key and pass against ~28 per key and merge round for the merge
// block sort's ten rounds (profiles/sort_r6.md). Padding keys of a partial
// tile are all-ones and, stable, stay behind every real key. LDS: 64 KiB of
// keys + 16 KiB of counts = 80 KiB and <= 64 VGPRs (8 waves per SIMD): two
// blocks per CU.
template <int RANK, int ITEMS = kMsItems, bool HAS_VALUES = false, int NT = 1024>
__global__ __launch_bounds__(NT, NT == 1024 && ITEMS == 16 && !HAS_VALUES ? 8 : 4) void ms_block_radix_kernel(
    const uint32_t* __restrict__ ki, uint32_t* __restrict__ ko, const uint32_t* __restrict__ vi,
    uint32_t* __restrict__ vo, long long n, int mode_in, int mode_out, MsSamples smp) {
    constexpr int NW = NT / kWave, TILE = NT * ITEMS;
    __shared__ uint32_t s_keys[TILE];
    __shared__ uint32_t s_vals[HAS_VALUES ? TILE : 1];
    __shared__ uint32_t s_whist[NW][kBins];
    uint32_t* s_tmp = s_keys;  // the block scan's wave totals (s_keys is idle between reload and scatter)
    const int tid = threadIdx.x, lane = lane_id(), wid = tid / kWave;
    const long long base = (long long)blockIdx.x * TILE;
    const int cnt = (int)(n - base < TILE ? n - base : TILE);
    uint32_t key[ITEMS], val[HAS_VALUES ? ITEMS : 1], rank2[ITEMS / 2];  // in-wave ranks (< 1024), two per register
    // wave-striped items: item k of lane l is key wid*1024 + k*64 + l (memory order (k, l))
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const int i = wid * (kWave * ITEMS) + k * kWave + lane;
        key[k] = i < cnt ? ms_key_in(ki[base + i], mode_in) : 0xffffffffu;
        if constexpr (HAS_VALUES) val[k] = i < cnt ? vi[base + i] : 0u;
    }
    auto put_rank = [&](int k, uint32_t r) {
        rank2[k / 2] = (k & 1) ? (rank2[k / 2] | (r << 16)) : r;
    };
    for (int shift = 0; shift < 32; shift += kRadixBits) {
#pragma unroll
        for (int w = 0; w < NW * kBins / NT; ++w) (&s_whist[0][0])[w * NT + tid] = 0u;
        __syncthreads();
        if constexpr (RANK == kRankLanes) {
#pragma unroll
            for (int k = 0; k < ITEMS; ++k) {
                const uint32_t d = digit_of(key[k], shift);
                const uint32_t d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)d);
                if (__ballot(d != d0) == 0) {  // one digit in the wave: one atomic
                    uint32_t b = 0;
                    if (lane == 0) b = atomicAdd(&s_whist[wid][d0], (uint32_t)kWave);
                    put_rank(k, (uint32_t)__builtin_amdgcn_readfirstlane((int)b) + (uint32_t)lane);
                } else {
                    put_rank(k, atomicAdd(&s_whist[wid][d], 1u));  // same-address lanes resolve in lane order
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < ITEMS; ++k) {
                const uint32_t d = digit_of(key[k], shift);
                const uint64_t peers = match_digit(d, true);
                const uint32_t below = (uint32_t)__builtin_popcountll(peers & ((1ull << lane) - 1ull));
                const uint32_t prev = s_whist[wid][d];
                put_rank(k, prev + below);
                if (below == 0) s_whist[wid][d] = prev + (uint32_t)__builtin_popcountll(peers);
                __builtin_amdgcn_sched_barrier(0);  // keep each item's ballots next to its LDS update
            }
        }
        __syncthreads();
        // per digit: exclusive prefix over the waves, then the block scan of the digit totals
        uint32_t run = 0;
        if (tid < kBins) {
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                const uint32_t c = s_whist[w][tid];
                s_whist[w][tid] = run;
                run += c;
            }
        }
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan<NW>(tid < kBins ? run : 0u, s_tmp, tot, OpAdd());
        if (tid < kBins) {
#pragma unroll
            for (int w = 0; w < NW; ++w) s_whist[w][tid] += ex;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t pos = s_whist[wid][digit_of(key[k], shift)] + ((rank2[k / 2] >> (16 * (k & 1))) & 0xffffu);
            s_keys[pos] = key[k];
            if constexpr (HAS_VALUES) s_vals[pos] = val[k];
        }
        __syncthreads();
        if (shift + kRadixBits < 32) {
#pragma unroll
            for (int k = 0; k < ITEMS; ++k) {
                key[k] = s_keys[wid * (kWave * ITEMS) + k * kWave + lane];
                if constexpr (HAS_VALUES) val[k] = s_vals[wid * (kWave * ITEMS) + k * kWave + lane];
            }
        }
    }
    if (smp.first) {  // block-uniform: the next partition's run samples
        const int nq = (cnt + smp.st - 1) / smp.st;
        for (int q = tid; q < nq; q += NT) {
            const int e = (q + 1) * smp.st < cnt ? (q + 1) * smp.st : cnt;
            smp.first[base / smp.st + q] = s_keys[q * smp.st];
            smp.last[base / smp.st + q] = s_keys[e - 1];
        }
    }
    auto out = [&](auto md) {  // unrolled coalesced stores, compile-time key transform
        constexpr int MD = decltype(md)::value;
#pragma unroll
        for (int q = 0; q < ITEMS; ++q) {
            const int i = tid + q * NT;
            if (i < cnt) {
                ko[base + i] = ms_key_out(s_keys[i], MD);
                if constexpr (HAS_VALUES) vo[base + i] = s_vals[i];
            }
        }
    };
    if (mode_out == 0) out(std::integral_constant<int, 0>());
    else if (mode_out == 1) out(std::integral_constant<int, 1>());
    else out(std::integral_constant<int, 2>());
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

// Merge-path partitions of a whole pass, G lanes per output tile: split[t]
// = the number of A keys among the first (t * tile - a0) outputs of tile
// t's pair, by a G-ary search (one load pair per lane and round, ~log_G L
// dependent rounds, no barrier). All tiles' searches run at once here, so the
// merge kernel's blocks start on their loads instead of each paying the
// search's dependent global rounds on its own critical path. G trades rounds
// (latency) against the lines each round touches (G per array and tile).
//
// With the previous kernel's run samples (sfirst / slast: first and last key
// of every `tile`-key tile) the search first narrows to one tile's width on
// candidates m = jT only: A[jT] is sfirst of A's tile j, and B[diag-1-jT] is
// the last key of a B tile (diag, jT and B's start are multiples of T), so
// those rounds read a 8-byte-per-tile array that stays in L2 instead of
// scattered lines of the keys. Only the last ~log_G T rounds touch the keys.
template <int G>
__global__ __launch_bounds__(256) void ms_partition_kernel(const uint32_t* __restrict__ ki, long long n, long long L,
                                                           long long tile, long long ntiles,
                                                           long long* __restrict__ split,
                                                           const uint32_t* __restrict__ sfirst,
                                                           const uint32_t* __restrict__ slast,
                                                           uint32_t* __restrict__ vfirst,
                                                           uint32_t* __restrict__ vlast) {
    static_assert(G == 4 || G == 8 || G == 16 || G == 32 || G == 64, "partition group: 4-64 lanes");
    const long long t = ((long long)blockIdx.x * 256 + threadIdx.x) / G;
    const int sub = threadIdx.x % G;
    const int gshift = lane_id() & ~(G - 1);  // the group's first lane in the wave
    const uint64_t gmask = G == 64 ? ~0ull : ((1ull << G) - 1);
    const bool valid = t < ntiles;
    const long long o0 = valid ? t * tile : 0;
    const long long a0 = o0 & ~(2 * L - 1);
    const long long la = a0 + L < n ? L : n - a0;
    const long long lb = a0 + 2 * L < n ? L : (n - a0 - la > 0 ? n - a0 - la : 0);
    const uint32_t* A = ki + a0;
    const uint32_t* B = ki + a0 + la;
    const long long diag = o0 - a0;
    long long lo = diag - lb > 0 ? diag - lb : 0, hi = diag < la ? diag : la;
    if (sfirst) {  // kernel-uniform
        // first j in [jlo, jhi) with Q(jT) false: x lies in ((j-1)T, jT]
        const long long j0 = (lo + tile - 1) / tile, j1 = (hi + tile - 1) / tile;
        long long jlo = j0, jhi = j1;
        const long long ga = a0 / tile, gb = (a0 + la + diag) / tile - 1;  // B[diag-1-jT] ends tile gb - j
        while (__ballot(jlo < jhi)) {
            const bool act = jlo < jhi;
            const long long step = (jhi - jlo + G - 1) / G;
            const long long j = jlo + (long long)sub * step;
            const bool q = act && j < jhi && sfirst[ga + j] <= slast[gb - j];
            const uint64_t fails = (__ballot(!q) >> gshift) & gmask;
            const int f = fails ? __builtin_ctzll(fails) : G;
            if (act) {
                const long long nlo = f == 0 ? jlo : jlo + (long long)(f - 1) * step + 1;
                const long long jf = jlo + (long long)f * step;
                jhi = f == G ? jhi : (jf < jhi ? jf : jhi);
                jlo = nlo;
            }
        }
        if (jlo < j1 && jlo * tile < hi) hi = jlo * tile;
        if (jlo > j0 && (jlo - 1) * tile + 1 > lo) lo = (jlo - 1) * tile + 1;
    }
    while (__ballot(lo < hi)) {  // until every group of the wave is done
        const bool act = lo < hi;
        const long long step = (hi - lo + G - 1) / G;
        const long long m = lo + (long long)sub * step;
        const bool q = act && m < hi && A[m] <= B[diag - 1 - m];
        const uint64_t fails = (__ballot(!q) >> gshift) & gmask;
        const int f = fails ? __builtin_ctzll(fails) : G;
        if (act) {
            const long long nlo = f == 0 ? lo : lo + (long long)(f - 1) * step + 1;
            const long long mf = lo + (long long)f * step;
            hi = f == G ? hi : (mf < hi ? mf : hi);
            lo = nlo;
        }
    }
    if (valid && sub == 0) {
        split[t] = lo;
        if (vfirst) {  // kernel-uniform: samples of the merged pair this pass would write (4-way passes)
            const long long jb = diag - lo;
            if (diag < la + lb) {
                const bool ta = lo < la && (jb >= lb || A[lo] <= B[jb]);
                vfirst[t] = ta ? A[lo] : B[jb];
            }
            if (diag > 0) {  // the key before this tile's first ends the previous tile
                uint32_t e = lo > 0 ? A[lo - 1] : 0u;
                if (jb > 0) e = max(e, B[jb - 1]);
                vlast[t - 1] = e;
            }
            if (o0 + tile >= a0 + la + lb) vlast[t] = lb > 0 ? max(A[la - 1], B[lb - 1]) : A[la - 1];
        }
    }
}

// split: the pass's partitions from ms_partition_kernel, or nullptr for the
// in-block cooperative search (NT = 256 only). NT lanes merge an output tile
// of NT * 16 keys.
template <bool HAS_VALUES, int NT = kMsThreads>
__global__ __launch_bounds__(NT) void ms_merge_pass_kernel(const uint32_t* __restrict__ ki, uint32_t* __restrict__ ko,
                                                           const uint32_t* __restrict__ vi, uint32_t* __restrict__ vo,
                                                           long long n, long long L, int mode_out,
                                                           const long long* __restrict__ split, MsSamples smp) {
    constexpr int TILE = NT * kMsItems;
    __shared__ uint32_t sk[lp_size(TILE) + 1];  // + the merge's out-of-run load slot
    __shared__ uint32_t sv[HAS_VALUES ? lp_size(TILE) : 1];
    __shared__ uint64_t smask[2][2];
    __shared__ long long ssplit[2];
    const int t = threadIdx.x;
    // consecutive output tiles on one XCD: their diagonal searches probe the
    // same lines of A and B, which then hit that XCD's L2
    const long long tile = xcd_remap(blockIdx.x, gridDim.x);
    const long long o0 = tile * TILE;
    const long long o1 = o0 + TILE < n ? o0 + TILE : n;
    const long long a0 = o0 & ~(2 * L - 1);  // pair start (2L is a multiple of the tile)
    const long long la = a0 + L < n ? L : n - a0;
    const long long lb = a0 + 2 * L < n ? L : (n - a0 - la > 0 ? n - a0 - la : 0);
    const uint32_t* A = ki + a0;
    const uint32_t* B = ki + a0 + la;
    long long i0, i1;
    if (split) {  // block-uniform
        i0 = split[tile];
        i1 = o1 - a0 == la + lb ? la : split[tile + 1];  // a tile ending its pair took all of A
    } else if constexpr (NT == 256) {
        const int part = t >> 7;
        const long long diag = (part == 0 ? o0 : o1) - a0;
        int rounds = 0;  // ceil(log_128(L + 1)): candidates per search <= L + 1
        for (long long w = L + 1; w > 1; w = (w + 127) / 128) ++rounds;
        const long long sp = ms_coop_split(A, B, la, lb, diag, rounds, smask);
        if ((t & 127) == 0) ssplit[part] = sp;
        __syncthreads();
        i0 = ssplit[0];
        i1 = ssplit[1];
    } else {
        i0 = i1 = 0;  // the host never launches this
    }
    const long long j0 = (o0 - a0) - i0, j1 = (o1 - a0) - i1;
    int na = (int)(i1 - i0), nb = (int)(j1 - j0);
    if (na < 0 || nb < 0 || na + nb > TILE || i1 > la || j1 > lb) na = nb = 0;  // never out of range
    {  // coalesced loads, unrolled (immediate LDS offsets): A's piece, then B's
        const uint32_t* pa = ki + a0 + i0;
        const uint32_t* pb = ki + a0 + la + j0 - na;  // B's x-th output slot reads pb[x]
        const int lt = lp(t), c = na + nb;
        if (c > 0) {  // block-uniform; all 16 loads in flight (clamped indices), then the LDS writes
            uint32_t kk[kMsItems], vv[HAS_VALUES ? kMsItems : 1];
#pragma unroll
            for (int q = 0; q < kMsItems; ++q) {
                const int x = min(t + q * NT, c - 1);
                const uint32_t* src = x < na ? pa : pb;
                kk[q] = src[x];
                if constexpr (HAS_VALUES) vv[q] = vi[src - ki + x];
            }
#pragma unroll
            for (int q = 0; q < kMsItems; ++q) {
                if (t + q * NT < c) {
                    sk[lt + q * (NT + NT / 16)] = kk[q];
                    if constexpr (HAS_VALUES) sv[lt + q * (NT + NT / 16)] = vv[q];
                }
            }
        }
    }
    __syncthreads();
    const int cnt = na + nb;
    const int diag_l = kMsItems * t < cnt ? kMsItems * t : cnt;
    const int i = ms_split_lift(sk, 0, na, na, nb, diag_l, ms_lift_top(na, nb));
    uint32_t k[kMsItems], v[kMsItems];
    ms_merge16<HAS_VALUES, TILE>(sk, sv, 0, na, na, nb, i, diag_l - i, k, v);
    ms_store_tile<HAS_VALUES, NT>(sk, sv, k, v, ko, vo, o0, cnt, mode_out, smp);
}

}  // namespace

// the radix sort's lane-order check (sort.hip)
extern "C" int cme_radix_lane_order(int check);

// production: 2-way merge passes only
struct MsTwoWayOnly {
    static constexpr bool kOn = false;
    static hipError_t pass(hipStream_t, const uint32_t*, uint32_t*, const uint32_t*, uint32_t*, long long,
                           long long, long long, long long, const long long*, const uint32_t*, const uint32_t*,
                           long long*, int, MsSamples) {
        return hipErrorInvalidValue;
    }
};

// Stable merge sort of n keys from `in` into `out` (ping-pong through `tmp`;
// `in` may equal `out`; values optional, likewise). mode: 0 uint32, 1 int32,
// 2 float32 keys.
inline long long ms_ws_bytes(long long n) { return (long long)cdiv(n, kMsTile) * 48 + 256; }

// merge-pass output tile (tuning knob merge_tile: 4096 or 8192 keys; 8192
// needs the partition launch)
inline int merge_tile(bool part) {
    return part && cme::tune_get(cme::kTuneMergeTile) == 8192 ? 8192 : kMsTile;
}

// ws (cme_merge_ws_bytes(n) bytes, or nullptr): with it every merge pass
// first computes all tile partitions in one launch (ms_partition_kernel);
// without it each merge block searches its own (ms_coop_split). Layout:
// split[tiles] (8 B), then the run samples first[tiles] and last[tiles]
// (4 B each) that every kernel but the last writes for the next partition,
// then the 4-way passes' pair samples vfirst[tiles] / vlast[tiles] (4 B each)
// and boundary splits b4[3 tiles] (8 B each).
// FOUR: the 4-way pass of a 4-way schedule (FOUR::kOn; its launches in
// FOUR::pass), MsTwoWayOnly in the production library.
template <class FOUR>
int ms_sort_host(const uint32_t* in, uint32_t* out, uint32_t* tmp, const uint32_t* vin, uint32_t* vout,
                 uint32_t* vtmp, long long n, int mode, void* ws, void* stream) {
    hipStream_t s = as_stream(stream);
    if (n <= 0) return 0;
    if (mode < 0 || mode > 2 || (vin != nullptr) != (vout != nullptr) || (vin && !vtmp))
        return (int)hipErrorInvalidValue;
    // block-sort tile (tuning knob merge_block: 8192 or 16384 keys; 0 = auto:
    // 16384 for keys only from 4M keys -- one merge pass fewer for one more
    // LDS round; measured 4M 0.194 -> 0.183 ms, 48M 1.52-1.55 -> 1.50, but
    // 1M 0.099 -> 0.109 and key-value 48M 2.79 -> 2.90, where the 1024-lane
    // blocks halve the resident blocks per CU; profiles/sort_r5.md)
    const long mb = cme::tune_get(cme::kTuneMergeBlock);
    // keys-only block sorts by LDS radix (knob merge_block_sort: 1 radix, 0
    // the merge-network block sort) on a device that passed the lane-order
    // check (the ballot-match ranks would spill at the VGPRs two blocks per CU
    // allow: the merge block sort instead); they also take 32768-key tiles
    // (merge_block=32768: 128 KiB of LDS, one block per CU, one merge pass
    // fewer)
    bool radix_block = false;
    if (n > kBsTile && cme::tune_get(cme::kTuneMergeBlockSort) != 0) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        const bool capturing = hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
        radix_block = cme_radix_lane_order(capturing ? 0 : 1) != 0;
    }
    // 32768-key radix tiles: asked for, or by size (one merge pass fewer pays
    // from 6M to 24M keys: 8M 0.249 -> 0.233 ms, 16M 0.389 -> 0.374; 4M and
    // 48M lose 2 %, raw_r6/merge_knobs_ab_r6.jsonl)
    const bool huge = radix_block && !vin && (mb == 32768 || (mb == 0 && n >= (6ll << 20) && n <= (24ll << 20)));
    // (key-value pairs through the radix block sort: 16384-key tiles from 4M
    // too, 48M 2.49 -> 2.40 ms, 16M 0.705 -> 0.675, 4M 0.202 -> 0.190,
    // raw_r6/merge_kv_block_ab_r6.jsonl)
    const bool big = huge || mb == 16384 || (mb == 0 && (!vin || radix_block) && n >= (4ll << 20));
    // key-value pairs: the radix block sort at 8192-key tiles (512 lanes)
    const bool radix_kv = radix_block && vin && !big;
    // key-value 16384-key radix tiles (merge_block=16384: 144 KiB LDS, one
    // block per CU, one merge pass fewer)
    const bool radix_kv_big = radix_block && vin && big;
    radix_block = radix_block && !vin && big;
    const long long btile = huge ? 4 * kBsTile : (big ? 2 * kBsTile : kBsTile);
    // partitions: tuning knob merge_part (G lanes per tile, 0 = in-block
    // searches, -1 = auto: G = 8 from 8M keys). Measured (profiles/sort_r5.md):
    // 48M int32 2.21 -> 1.59 ms, 16M 0.65 -> 0.55; at 1M and 4M the extra
    // launch per pass costs more than the searches it moves (1M 0.124 ->
    // 0.136 ms, 4M 0.222 -> 0.230).
    long part = ws ? cme::tune_get(cme::kTuneMergePart) : 0;
    if (part < 0) part = n >= (8ll << 20) ? 8 : 0;
    const int mtile = merge_tile(part != 0);
    // 4-way passes (FOUR::kOn: the tuning library's arm, with partition
    // launches and 4096-key tiles): runs of L -> 4L while at least three runs
    // remain, a last 2-way pass for an odd number of doublings
    const bool four = FOUR::kOn && part != 0 && mtile == kMsTile;
    auto next_len = [&](long long L) { return four && 2 * L < n ? 4 * L : 2 * L; };
    int npass = 0;
    for (long long L = btile; L < n; L = next_len(L)) ++npass;
    // the block sort writes where an even number of passes later lands in out
    uint32_t* d0 = (npass & 1) ? tmp : out;
    uint32_t* v0 = vin ? ((npass & 1) ? vtmp : vout) : nullptr;
    const unsigned btiles = cdiv(n, btile), tiles = cdiv(n, mtile);
    const int m0 = npass ? 0 : mode;
    // run samples (knob merge_samples, default on): written by every kernel
    // whose output a partition launch searches next
    const bool samples = part != 0 && cme::tune_get(cme::kTuneMergeSamples) != 0;
    const MsSamples none{nullptr, nullptr, mtile};
    MsSamples smp = none;
    if (samples) {
        uint32_t* sbase = (uint32_t*)((char*)ws + (size_t)cdiv(n, kMsTile) * 8);
        smp = MsSamples{sbase, sbase + cdiv(n, kMsTile), mtile};
    }
    uint32_t* vfirst = nullptr;
    uint32_t* vlast = nullptr;
    long long* b4 = nullptr;
    if (four) {
        const size_t nt = cdiv(n, kMsTile);
        vfirst = (uint32_t*)((char*)ws + nt * 16);
        vlast = vfirst + nt;
        b4 = (long long*)((char*)ws + nt * 24);
    }
    const MsSamples smp0 = npass ? smp : none;
    if (huge)
        hipLaunchKernelGGL((ms_block_radix_kernel<kRankLanes, 32>), dim3(btiles), dim3(1024), 0, s, in, d0, vin, v0,
                           n, mode, m0, smp0);
    else if (radix_block)
        hipLaunchKernelGGL(ms_block_radix_kernel<kRankLanes>, dim3(btiles), dim3(1024), 0, s, in, d0, vin, v0, n,
                           mode, m0, smp0);
    else if (radix_kv)
        hipLaunchKernelGGL((ms_block_radix_kernel<kRankLanes, kMsItems, true, kBsThreads>), dim3(btiles),
                           dim3(kBsThreads), 0, s, in, d0, vin, v0, n, mode, m0, smp0);
    else if (radix_kv_big)
        hipLaunchKernelGGL((ms_block_radix_kernel<kRankLanes, kMsItems, true, 1024>), dim3(btiles), dim3(1024), 0, s,
                           in, d0, vin, v0, n, mode, m0, smp0);
    else if (big && vin)
        hipLaunchKernelGGL((ms_block_sort_kernel<true, 2 * kBsThreads>), dim3(btiles), dim3(2 * kBsThreads), 0, s, in,
                           d0, vin, v0, n, mode, m0, smp0);
    else if (big)
        hipLaunchKernelGGL((ms_block_sort_kernel<false, 2 * kBsThreads>), dim3(btiles), dim3(2 * kBsThreads), 0, s,
                           in, d0, vin, v0, n, mode, m0, smp0);
    else if (vin)
        hipLaunchKernelGGL(ms_block_sort_kernel<true>, dim3(btiles), dim3(kBsThreads), 0, s, in, d0, vin, v0, n, mode,
                           m0, smp0);
    else
        hipLaunchKernelGGL(ms_block_sort_kernel<false>, dim3(btiles), dim3(kBsThreads), 0, s, in, d0, vin, v0, n,
                           mode, m0, smp0);
    CME_TRY(hipGetLastError());
    const uint32_t *ki = d0, *vi = v0;
    int p = 0;
    for (long long L = btile; L < n; L = next_len(L), ++p) {
        const bool last = p == npass - 1;
        const bool w4 = four && 2 * L < n;
        uint32_t* ko = (ki == out) ? tmp : out;
        uint32_t* vo = vin ? ((vi == vout) ? vtmp : vout) : nullptr;
        long long* split = part ? (long long*)ws : nullptr;
        uint32_t* pf = w4 ? vfirst : nullptr;
        uint32_t* pl = w4 ? vlast : nullptr;
        if (split) {
            const int g = part == 4 || part == 8 || part == 16 || part == 32 ? (int)part : 64;
            const dim3 grid(cdiv((long long)tiles * g, 256));
#define CME_PART(G)                                                                                               \
    hipLaunchKernelGGL(ms_partition_kernel<G>, grid, dim3(256), 0, s, ki, n, L, (long long)mtile, (long long)tiles, \
                       split, smp.first, smp.last, pf, pl)
            if (g == 4) CME_PART(4);
            else if (g == 8) CME_PART(8);
            else if (g == 16) CME_PART(16);
            else if (g == 32) CME_PART(32);
            else CME_PART(64);
#undef CME_PART
        }
        const int mo = last ? mode : 0;
        const MsSamples so = last ? none : smp;
        if (w4) {
            CME_TRY(FOUR::pass(s, ki, ko, vi, vo, n, L, (long long)mtile, (long long)tiles, split, vfirst, vlast, b4,
                               mo, so));
        } else if (mtile == 8192) {
            if (vin)
                hipLaunchKernelGGL((ms_merge_pass_kernel<true, 512>), dim3(tiles), dim3(512), 0, s, ki, ko, vi, vo, n,
                                   L, mo, split, so);
            else
                hipLaunchKernelGGL((ms_merge_pass_kernel<false, 512>), dim3(tiles), dim3(512), 0, s, ki, ko, vi, vo, n,
                                   L, mo, split, so);
        } else if (vin) {
            hipLaunchKernelGGL(ms_merge_pass_kernel<true>, dim3(tiles), dim3(kMsThreads), 0, s, ki, ko, vi, vo, n, L,
                               mo, split, so);
        } else {
            hipLaunchKernelGGL(ms_merge_pass_kernel<false>, dim3(tiles), dim3(kMsThreads), 0, s, ki, ko, vi, vo, n, L,
                               mo, split, so);
        }
        CME_TRY(hipGetLastError());
        ki = ko;
        vi = vo;
    }
    return 0;
}


