// Onesweep LSD radix sort (8-bit digits) for gfx950.
//
// Parity: the hw4 radix sort (hw/hw4/programming/radixsort.cpp:22-121: per-block
// histograms -> reduce -> exclusive scan -> push-down -> per-block scatter;
// slides/Lecture16.pdf "radix sort with scan"). The reduce-then-scan form of
// that algorithm (sort.hip, cme_radix_sort_u32) reads the keys twice per pass;
// this one reads them once per pass plus once for all passes together:
//
//   K0 hist    : ONE read of the keys builds the digit histograms of every
//                pass (LDS, then no-return global atomics into 4 x 256
//                counters; the previous call's counter set is zeroed here).
//   K1..KP pass: persistent grid, tile t = 8192 keys (512 lanes x 16). Each
//                tile ranks its keys stably in LDS (wave64 ballot "match" per
//                item, per-wave running digit counts), publishes its 256 digit
//                counts (AGGREGATE), finds the nearest predecessor whose
//                INCLUSIVE prefixes are out (one wave polls 64 tile status
//                words per probe), sums the aggregates in between (digit-
//                parallel, 2 lanes per digit, 8 loads in flight), publishes its
//                own INCLUSIVE prefixes, reorders the tile by digit in LDS and
//                writes every digit run contiguously.
//
// Hand-offs follow cdna_hip_programming.md §6 G16 R2 ("the data IS the flag"):
// every (tile, digit) aggregate and inclusive prefix is ONE 8-byte granule
// {hi = tag << 2 | state, lo = value} (two separate arrays: a granule is
// written once and never changes meaning while it is summed) written by one
// relaxed agent-scope store and re-read by relaxed agent-scope loads until
// its tag and state are valid; the per-tile status word only tells the
// poller how far back to look. Tags are unique per pass
// and call (Python hands out the call epoch; under stream capture epoch 0
// makes the launcher zero the arrays in-stream), so no per-call memset.
// Grid: co-resident (occupancy API - 1 blocks per CU), block b owns tiles
// b, b+G, ... in order, so every predecessor of a tile belongs to a running
// block: the smallest unfinished tile always progresses (no ticket counter).
// (Round 4 measured the remedy the round-3 review proposed -- one workgroup
// per tile, tile ids from a per-pass ticket so look-back predecessors are
// always earlier-dispatched: 16M int32 0.84 ms vs 0.73 for this grid, 48M
// 2.36 vs 2.14; profiles/sort_r4.md.) In-tile ranks: one returning LDS
// atomic per key where the device resolves same-address lanes in lane order
// (sort.hip kRankLanes, cme_radix_lane_order), else the ballot match.
// Spins are bounded (lookback.h lb_give_up: sticky timeout word).
//
// Keys: uint32, int32 (sign bit flipped) or float32 (IEEE order flip) --
// the transform is applied when pass 1 loads and undone when the last pass
// stores, so no separate conversion kernels run. Optional 32-bit values.
#include "cme213/common.h"
#include "cme213/tuning.h"
#include "cme213/lookback.h"
#include "cme213/wave.h"

// sort.hip: 1 if this device's returning LDS atomics resolve same-address
// lanes in lane order (checked once per device when `check`)
extern "C" int cme_radix_lane_order(int check);

using namespace cme;

namespace {

constexpr int kOsThreads = 512;
constexpr int kOsWaves = kOsThreads / kWave;
constexpr int kOsItems = 16;
constexpr int kOsTile = kOsThreads * kOsItems;  // 8192 keys
constexpr int kBins = 256;
constexpr int kHistThreads = 256;
constexpr int kMaxPasses = 4;

enum : uint32_t { kGAgg = 1u, kGInc = 2u };

// key transforms: 0 uint32, 1 int32, 2 float32 (order-preserving map to uint32)
__device__ __forceinline__ uint32_t key_in(uint32_t k, int mode) {
    if (mode == 1) return k ^ 0x80000000u;
    if (mode == 2) return k ^ ((uint32_t)((int)k >> 31) | 0x80000000u);
    return k;
}
__device__ __forceinline__ uint32_t key_out(uint32_t u, int mode) {
    if (mode == 1) return u ^ 0x80000000u;
    if (mode == 2) return u ^ (((uint32_t)((int)u >> 31) ^ 0xffffffffu) | 0x80000000u);
    return u;
}

__device__ __forceinline__ uint64_t g_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_store(uint64_t* p, uint32_t tag, uint32_t state, uint32_t value) {
    __hip_atomic_store(p, ((uint64_t)((tag << 2) | state) << 32) | value, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
// state of a granule for this pass's tag (0 = not yet published)
__device__ __forceinline__ uint32_t g_state(uint64_t g, uint32_t tag) {
    const uint32_t hi = (uint32_t)(g >> 32);
    return (hi >> 2) == tag ? (hi & 3u) : 0u;
}

// ---------------------------------------------------------------- K0
// Digit histograms of every pass in one read (16-B loads, 4 keys per lane).
// Block 0 also zeroes the counter set the NEXT call will use.
__global__ __launch_bounds__(kHistThreads) void radix_hist_kernel(const uint32_t* __restrict__ keys, long long n,
                                                                  int mode, int bit0, int npass,
                                                                  uint32_t* __restrict__ hist,
                                                                  uint32_t* __restrict__ hist_next) {
    __shared__ uint32_t h[kMaxPasses][kBins];
    for (int i = threadIdx.x; i < kMaxPasses * kBins; i += kHistThreads) (&h[0][0])[i] = 0u;
    if (blockIdx.x == 0 && hist_next)
        for (int i = threadIdx.x; i < kMaxPasses * kBins; i += kHistThreads) hist_next[i] = 0u;
    __syncthreads();
    auto add = [&](uint32_t k) {
        k = key_in(k, mode);
        for (int p = 0; p < npass; ++p) atomicAdd(&h[p][(k >> (bit0 + 8 * p)) & 255u], 1u);
    };
    // 16-B loads when the keys are 16-B aligned (a tensor view may not be)
    const long long nv = ((uintptr_t)keys & 15u) ? 0 : n / 4;
    const uint4* kv = reinterpret_cast<const uint4*>(keys);
    const long long stride = (long long)gridDim.x * kHistThreads;
    for (long long i = (long long)blockIdx.x * kHistThreads + threadIdx.x; i < nv; i += stride) {
        const uint4 v = kv[i];
        add(v.x);
        add(v.y);
        add(v.z);
        add(v.w);
    }
    for (long long i = nv * 4 + (long long)blockIdx.x * kHistThreads + threadIdx.x; i < n; i += stride)
        add(keys[i]);
    __syncthreads();
    for (int i = threadIdx.x; i < npass * kBins; i += kHistThreads) {
        const uint32_t c = (&h[0][0])[i];
        if (c) atomicAdd(hist + i, c);
    }
}

// Stable rank of each lane's digit among the lanes of its wave (ballot match).
// (per bit: the bit as an all-ones / zero mask, its ballot, and one gfx950
// v_bitop3_b32 per 32-bit half for peers &= ~(ballot ^ mask); sort.hip
// match_digit, profiles/sort_r3.md)
__device__ __forceinline__ uint64_t os_match(uint32_t d, bool valid) {
    const uint64_t v = __ballot(valid);
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        uint32_t s;
        asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(s) : "v"(d), "i"(b));
        const uint64_t m = __ballot(s != 0u);
        lo = __builtin_amdgcn_bitop3_b32(lo, (uint32_t)m, s, 0x90);
        hi = __builtin_amdgcn_bitop3_b32(hi, (uint32_t)(m >> 32), s, 0x90);
    }
    return ((uint64_t)hi << 32) | lo;
}

// ---------------------------------------------------------------- K1..KP
template <bool HAS_VALUES, bool LANES>
__global__ __launch_bounds__(kOsThreads, HAS_VALUES ? 2 : 4) void radix_onesweep_kernel(
    const uint32_t* __restrict__ kin, uint32_t* __restrict__ kout, const uint32_t* __restrict__ vin,
    uint32_t* __restrict__ vout, long long n, int shift, int mode_in, int mode_out,
    const uint32_t* __restrict__ counts, uint64_t* __restrict__ agg, uint64_t* __restrict__ inc,
    uint64_t* __restrict__ stat, int tiles, uint32_t tag, unsigned* timeout) {
    __shared__ uint32_t s_keys[kOsTile];
    __shared__ uint32_t s_vals[HAS_VALUES ? kOsTile : 1];
    __shared__ uint32_t s_cnt[kOsWaves][kBins];  // per-wave running counts, then per-wave exclusive offsets
    __shared__ uint32_t s_off[kBins];            // tile-local exclusive digit offsets
    __shared__ uint32_t s_gb[kBins];             // global position of digit run start - s_off
    __shared__ uint32_t s_dofs[kBins];           // global exclusive digit offsets of this pass
    __shared__ uint32_t s_part[kBins];
    __shared__ uint32_t s_tmp[kOsWaves];
    __shared__ int s_K;
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int wid = tid / kWave;
    const uint64_t lt = (1ull << lane) - 1ull;

    {  // global digit offsets: exclusive scan of this pass's histogram
        uint32_t tot;
        const uint32_t c = tid < kBins ? counts[tid] : 0u;
        const uint32_t ex = block_exclusive_scan<kOsWaves>(c, s_tmp, tot, OpAdd());
        if (tid < kBins) s_dofs[tid] = ex;
    }

    for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
        for (int i = tid; i < kOsWaves * kBins; i += kOsThreads) (&s_cnt[0][0])[i] = 0u;
        const long long base = (long long)t * kOsTile + wid * (kWave * kOsItems) + lane;
        // item k of this lane is a key iff k < nk (items are 64 keys apart)
        const long long rem = n - base;
        const int nk = rem <= 0 ? 0 : (rem >= (long long)kWave * kOsItems ? kOsItems : (int)((rem + kWave - 1) / kWave));
        uint32_t key[kOsItems], val[kOsItems], rank[kOsItems];
#pragma unroll
        for (int k = 0; k < kOsItems; ++k) {
            key[k] = k < nk ? kin[base + k * kWave] : 0xffffffffu;
        }
        if (mode_in) {
#pragma unroll
            for (int k = 0; k < kOsItems; ++k) key[k] = k < nk ? key_in(key[k], mode_in) : key[k];
        }
        __syncthreads();  // counters zeroed; previous tile's LDS reads done
        // stable in-tile ranks: (wave, item, lane) is memory order
        if constexpr (LANES) {
            // one returning LDS atomic per key (lanes resolve in lane order);
            // a wave whose valid keys share one digit adds once
#pragma unroll
            for (int k = 0; k < kOsItems; ++k) {
                const bool ok = k < nk;
                const uint32_t d = (key[k] >> shift) & 255u;
                const uint64_t act = __ballot(ok);
                if (act == 0) {
                    rank[k] = 0xffffffffu;
                    continue;
                }
                const int first = (int)__builtin_ctzll(act);
                const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane((int)d, first);
                if (__ballot(ok && d != d0) == 0) {
                    uint32_t base = 0;
                    if (lane == first) base = atomicAdd(&s_cnt[wid][d0], (uint32_t)__builtin_popcountll(act));
                    base = (uint32_t)__builtin_amdgcn_readlane((int)base, first);
                    rank[k] = ok ? base + (uint32_t)__builtin_popcountll(act & lt) : 0xffffffffu;
                } else {
                    uint32_t old = 0xffffffffu;
                    if (ok) old = atomicAdd(&s_cnt[wid][d], 1u);
                    rank[k] = old;
                }
            }
        } else {
            // ballot match; the scheduling barriers keep the compiler from
            // hoisting every item's 8 ballots above the LDS chain (spills)
#pragma unroll
            for (int k = 0; k < kOsItems; ++k) {
                const bool ok = k < nk;
                const uint32_t d = (key[k] >> shift) & 255u;
                const uint64_t peers = os_match(d, ok);
                const uint32_t below = (uint32_t)__builtin_popcountll(peers & lt);
                const uint32_t prev = ok ? s_cnt[wid][d] : 0u;
                rank[k] = ok ? prev + below : 0xffffffffu;
                if (ok && below == 0) s_cnt[wid][d] = prev + (uint32_t)__builtin_popcountll(peers);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if constexpr (HAS_VALUES) {  // values are only needed for the reorder: loaded after the ranking
#pragma unroll
            for (int k = 0; k < kOsItems; ++k) val[k] = k < nk ? vin[base + k * kWave] : 0u;
        }
        __syncthreads();
        // per digit: exclusive offsets across waves, tile count -> AGGREGATE
        uint32_t cnt = 0;
        if (tid < kBins) {
#pragma unroll
            for (int w = 0; w < kOsWaves; ++w) {
                const uint32_t c = s_cnt[w][tid];
                s_cnt[w][tid] = cnt;
                cnt += c;
            }
            g_store(agg + (size_t)t * kBins + tid, tag, kGAgg, cnt);
        }
        {
            uint32_t tot;
            const uint32_t ex = block_exclusive_scan<kOsWaves>(cnt, s_tmp, tot, OpAdd());
            if (tid < kBins) s_off[tid] = ex;
        }
        // status AGG after this tile's granules (only a hint: granules validate themselves)
        if (tid == 0) __hip_atomic_store(stat + t, (uint64_t)((tag << 2) | kGAgg) << 32, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();  // s_off complete
        // reorder the tile by digit in LDS now (keys / ranks die before the
        // look-back, which then has the registers to keep 8 loads in flight)
#pragma unroll
        for (int k = 0; k < kOsItems; ++k) {
            if (rank[k] != 0xffffffffu) {
                const uint32_t d = (key[k] >> shift) & 255u;
                const uint32_t pos = s_off[d] + s_cnt[wid][d] + rank[k];
                s_keys[pos] = key[k];
                if constexpr (HAS_VALUES) s_vals[pos] = val[k];
            }
        }
        // ---- look-back: wave 0 finds K = number of aggregate-only predecessors
        // before the nearest inclusive one (t-1-K; -1 = the virtual start)
        if (wid == 0) {
            int K = 0;
            unsigned spins = 0;
            while (true) {
                const int idx = t - 1 - K - lane;
                const uint32_t st = idx >= 0 ? g_state(g_load(stat + idx), tag) : kGInc;
                const uint64_t im = __ballot(st == kGInc);
                const int j = im ? __builtin_ctzll(im) : kWave;
                if (__any(lane < j && st == 0u)) {  // a predecessor has not published yet
                    if (lb_give_up(++spins, timeout, lane)) {
                        K = t;  // give up: sum whatever is there
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                K += j;
                if (j < kWave) break;
            }
            if (lane == 0) s_K = K;
        }
        lds_bcast_sync();
        const int K = s_K;
        {
            const int d = tid & (kBins - 1), h = tid >> 8;
            uint32_t sum = 0;
            for (int i0 = h; i0 < K; i0 += 2 * 8) {
                uint64_t g[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int i = i0 + 2 * q;
                    g[q] = i < K ? g_load(agg + (size_t)(t - 1 - i) * kBins + d) : 0ull;
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int i = i0 + 2 * q;
                    if (i >= K) break;
                    unsigned spins = 0;
                    while (g_state(g[q], tag) == 0u) {
                        if (lb_give_up(++spins, timeout, 0)) break;
                        __builtin_amdgcn_s_sleep(1);
                        g[q] = g_load(agg + (size_t)(t - 1 - i) * kBins + d);
                    }
                    sum += (uint32_t)g[q];
                }
            }
            if (h == 1) s_part[d] = sum;
            uint32_t incv = 0;
            if (h == 0 && t - 1 - K >= 0) {  // the inclusive prefix ending the walk
                const uint64_t* p = inc + (size_t)(t - 1 - K) * kBins + d;
                uint64_t x = g_load(p);
                unsigned spins = 0;
                while (g_state(x, tag) != kGInc) {
                    if (lb_give_up(++spins, timeout, 0)) break;
                    __builtin_amdgcn_s_sleep(1);
                    x = g_load(p);
                }
                incv = (uint32_t)x;
            }
            __syncthreads();
            if (h == 0) {
                const uint32_t prefix = incv + sum + s_part[d];
                const uint32_t tc = (d + 1 < kBins ? s_off[d + 1] : (uint32_t)min((long long)kOsTile,
                                                                                  n - (long long)t * kOsTile)) -
                                    s_off[d];
                g_store(inc + (size_t)t * kBins + d, tag, kGInc, prefix + tc);
                s_gb[d] = s_dofs[d] + prefix - s_off[d];
            }
        }
        // status INC: every INC granule store drained first (waves 0-3 store)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store(stat + t, (uint64_t)((tag << 2) | kGInc) << 32, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
        // every digit run goes out contiguously
        const int tile_n = (int)min((long long)kOsTile, n - (long long)t * kOsTile);
#pragma unroll 4
        for (int i = tid; i < tile_n; i += kOsThreads) {
            const uint32_t k = s_keys[i];
            const uint32_t g = s_gb[(k >> shift) & 255u] + (uint32_t)i;
            if ((long long)g >= n) continue;  // only after a look-back timeout: never write out of range
            kout[g] = key_out(k, mode_out);
            if constexpr (HAS_VALUES) vout[g] = s_vals[i];
        }
    }
}

template <typename K>
int occupancy_blocks_per_cu(K kernel, int threads) {
    int api = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&api, kernel, threads, 0) != hipSuccess || api < 1) api = 1;
    return api;
}

}  // namespace

// Workspace: 2 counter sets (2 x 4 x 256 u32, alternating by call epoch) +
// tile status words + (tile, digit) granules.
CME_EXPORT long long cme_radix_onesweep_ws_bytes(long long n) {
    const long long tiles = (n + kOsTile - 1) / kOsTile;
    return 2 * kMaxPasses * kBins * 4 + tiles * 8 + 2 * tiles * kBins * 8 + 256;
}

// Sort n keys from kin (not modified) into kout over bits [bit0, bit1) --
// ceil((bit1-bit0)/8) passes ping-ponging through ktmp so that the last pass
// writes kout; values (optional) likewise. mode: 0 uint32, 1 int32, 2 float32
// keys. epoch >= 1: this call's tag base (the caller increments it per call
// and re-zeroes ws before 2^27 calls); epoch 0 (stream capture): the arrays
// are zeroed in-stream first.
CME_EXPORT int cme_radix_onesweep(const uint32_t* kin, uint32_t* kout, uint32_t* ktmp, const uint32_t* vin,
                                  uint32_t* vout, uint32_t* vtmp, long long n, int mode, int bit0, int bit1,
                                  void* ws, long long epoch, void* stream) {
    hipStream_t s = as_stream(stream);
    if (n <= 0) return 0;
    if (n >= (1ll << 32) || bit0 < 0 || bit1 > 32 || bit1 <= bit0 || mode < 0 || mode > 2 ||
        (vin != nullptr) != (vout != nullptr) || (vin && !vtmp) || epoch < 0 || epoch >= (1ll << 27))
        return (int)hipErrorInvalidValue;
    const int npass = (bit1 - bit0 + 7) / 8;
    const long long tiles = (n + kOsTile - 1) / kOsTile;
    unsigned* timeout = lb_host_timeout();
    if (!timeout) return (int)hipErrorOutOfMemory;
    uint32_t* hsets = (uint32_t*)ws;
    const int set = (int)(epoch & 1);
    uint32_t* hist = hsets + set * kMaxPasses * kBins;
    uint32_t* hist_next = hsets + (set ^ 1) * kMaxPasses * kBins;
    uint64_t* stat = (uint64_t*)((char*)ws + 2 * kMaxPasses * kBins * 4);
    // aggregates and inclusive prefixes in separate arrays: an aggregate
    // granule never changes meaning while a successor sums it
    uint64_t* agg = stat + tiles;
    uint64_t* inc = agg + tiles * kBins;
    if (epoch == 0) {  // captured: zero everything this call reads, every replay
        CME_TRY(hipMemsetAsync(ws, 0, (size_t)cme_radix_onesweep_ws_bytes(n), s));
        hist_next = nullptr;
    }
    const long long nv = n / 4;
    long long hb = (nv + kHistThreads - 1) / kHistThreads;
    const long long hcap = 2ll * device_cu_count();
    hb = hb < 1 ? 1 : (hb > hcap ? hcap : hb);
    hipLaunchKernelGGL(radix_hist_kernel, dim3((unsigned)hb), dim3(kHistThreads), 0, s, kin, n, mode, bit0, npass,
                       hist, hist_next);
    CME_TRY(hipGetLastError());
    // co-resident blocks per CU: the occupancy API's answer. VGPRs bind (4
    // waves per SIMD = 2 blocks of 8 waves); the SGPR file (106 per wave: 6
    // waves per SIMD) does not, so the API's known over-report for SGPR-bound
    // kernels (common.h persistent_blocks_per_cu) does not apply here.
    // Per instantiation: the look-back needs every block of the grid resident,
    // so the grid is sized for the kernel actually launched (the ballot-match
    // fallback <V, false> may fit fewer blocks per CU than the lane-rank one;
    // ADVICE r4)
    static const int bpc[2][2] = {
        {occupancy_blocks_per_cu(radix_onesweep_kernel<false, false>, kOsThreads),
         occupancy_blocks_per_cu(radix_onesweep_kernel<false, true>, kOsThreads)},
        {occupancy_blocks_per_cu(radix_onesweep_kernel<true, false>, kOsThreads),
         occupancy_blocks_per_cu(radix_onesweep_kernel<true, true>, kOsThreads)}};
    // lane-order ranks where the device passed the check (not checked under
    // stream capture: a device not yet checked takes the ballot match)
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    const bool capturing = hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
    const bool lanes = cme::tune_get(cme::kTuneRadixOsLanes) != 0 && cme_radix_lane_order(capturing ? 0 : 1) != 0;
    const int bpc_used = bpc[vin ? 1 : 0][lanes ? 1 : 0];
    if (bpc_used < 1) return (int)hipErrorInvalidConfiguration;
    const long long cap = (long long)device_cu_count() * bpc_used;
    const int grid = (int)(tiles < cap ? tiles : cap);
    const uint32_t* src = kin;
    const uint32_t* vsrc = vin;
    for (int p = 0; p < npass; ++p) {
        // the last pass lands in kout: odd pass counts start there
        const bool to_out = ((npass - 1 - p) & 1) == 0;
        uint32_t* dst = to_out ? kout : ktmp;
        uint32_t* vdst = vin ? (to_out ? vout : vtmp) : nullptr;
        const int shift = bit0 + 8 * p;
        const uint32_t tag = (uint32_t)(epoch * kMaxPasses + p);
        const int mi = p == 0 ? mode : 0, mo = p == npass - 1 ? mode : 0;
#define CME_OS(V, L)                                                                                            \
    hipLaunchKernelGGL((radix_onesweep_kernel<V, L>), dim3(grid), dim3(kOsThreads), 0, s, src, dst, vsrc, vdst, n, \
                       shift, mi, mo, hist + p * kBins, agg, inc, stat, (int)tiles, tag, timeout)
        if (vin) {
            if (lanes)
                CME_OS(true, true);
            else
                CME_OS(true, false);
        } else {
            if (lanes)
                CME_OS(false, true);
            else
                CME_OS(false, false);
        }
#undef CME_OS
        CME_TRY(hipGetLastError());
        src = dst;
        vsrc = vdst;
    }
    return 0;
}

CME_REGISTER_KERNEL(radix_hist, 256, radix_hist_kernel);
CME_REGISTER_KERNEL(radix_onesweep, 512, radix_onesweep_kernel<false, true>);
CME_REGISTER_KERNEL(radix_onesweep_kv, 512, radix_onesweep_kernel<true, true>);
