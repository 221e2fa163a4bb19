// Single-pass decoupled look-back (Merrill & Garland) for wave64 / gfx950.
//
// Inter-workgroup hand-off follows the "data IS the flag" form for payloads
// <= 4 KB (cdna_hip_programming.md §6 Guideline 16, R2): each tile publishes
// ONE naturally aligned 8-byte granule {status/flags : 32 | value bits : 32}
// with a relaxed agent-scope atomic store (global_store ... sc1) and
// predecessors' granules are re-read with relaxed agent-scope atomic loads
// (sc1, bypassing the per-CU L1). No fences are needed and results do not
// depend on dispatch order or XCD placement. Grids are persistent and
// co-resident (sized from the occupancy API, common.h
// persistent_blocks_per_cu); block b scans tiles b, b+G, ... in order, so
// every predecessor of a tile is owned by a running block (no ordering
// ticket: a single atomic word saturates at ~88 ops/us). The workspace --
// timeout word, then the descriptor array -- is zeroed by the launcher
// (hipMemsetAsync). Spins are bounded: a tile that waits > kSpinLimit polls
// sets the timeout word and continues, so a bug can never hang the GPU; the
// Python layer reads the word (ops/scan.py lookback_timed_out; automatic
// under CME_SYNC_CHECK=1, asserted by the tests).
#pragma once
#include "common.h"
#include "wave.h"

namespace cme {

// Status word = (epoch << 8) | bits. A descriptor is valid for a launch only
// when its epoch matches, so a multi-iteration driver zeroes the array ONCE
// and gives iteration i epoch i+1 (epoch 0 never matches a zeroed word).
enum : uint32_t { kStInvalid = 0, kStAggregate = 1, kStInclusive = 2, kStFlag = 4 };
// Bounded spins: ~2^18 polls (well under a second) per wait, and the timeout
// word is STICKY -- every 256 polls a waiter re-reads it and gives up at once
// if any tile already timed out, so a broken launch (e.g. a grid that is not
// co-resident) ends in about one spin limit instead of one per tile.
constexpr unsigned kSpinLimit = 1u << 18;

__device__ __forceinline__ bool lb_give_up(unsigned spins, unsigned* timeout, int lane) {
    if (spins > kSpinLimit) {
        if (lane == 0) __hip_atomic_store(timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return true;
    }
    if ((spins & 255u) == 255u)
        return __hip_atomic_load(timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
    return false;
}

// The timeout word the kernels set lives in pinned, mapped HOST memory
// (lb_host_timeout, scan.hip): it is never reset by a launch, so a timed-out
// launch poisons the following ones (they give up at once) until the host
// reads and clears it -- ops/scan.py does that before every look-back call
// and raises, without a device synchronisation.
unsigned* lb_host_timeout();

// Workspace layout: [0, 16) unused pad, [16, 16 + 8*tiles) descriptors.
static inline unsigned* lb_timeout_word(void* ws) { return (unsigned*)ws; }
static inline uint64_t* lb_descriptors(void* ws) { return (uint64_t*)((char*)ws + 16); }
static inline size_t lb_ws_bytes(long long tiles) { return 16 + (size_t)tiles * 8; }

__device__ __forceinline__ void lb_publish(uint64_t* d, uint32_t status, uint32_t vbits, uint32_t epoch = 0) {
    __hip_atomic_store(d, ((uint64_t)((epoch << 8) | status) << 32) | vbits, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t lb_poll(uint64_t* d) {
    return __hip_atomic_load(d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Ticket: thread 0 draws the next tile id; broadcast through `lds`.
__device__ __forceinline__ int lb_ticket(unsigned* counter, int* lds) {
    if (threadIdx.x == 0) *lds = (int)__hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    int t = *lds;
    __syncthreads();
    return t;
}

template <typename T>
__device__ __forceinline__ uint32_t lb_bits(T v) {
    return __builtin_bit_cast(uint32_t, v);
}
template <typename T>
__device__ __forceinline__ T lb_val(uint64_t d) {
    return __builtin_bit_cast(T, (uint32_t)d);
}

// Wave-cooperative look-back for tile `tile` (call with one full wave).
// Returns the exclusive prefix of the tile (sum of all predecessors, or for a
// segmented scan the running value at the predecessor's end). `segmented`:
// a predecessor whose status carries kStFlag terminates the walk (a segment
// head lies inside it), like an inclusive one.
//
// Each lane inspects D consecutive predecessors per poll (window 64*D); only
// predecessors nearer than the first terminating one must be valid. Measured
// on MI355X (benchmarks/tune_scan.py): D = 1 is fastest -- wider windows
// multiply the memory-side poll traffic of spinning waves.
template <typename T, bool SEGMENTED, int D = 1, int SLEEP = 1>
__device__ T lb_lookback(uint64_t* desc, int tile, unsigned* timeout, uint32_t epoch = 0) {
    const int lane = lane_id();
    T prefix = T(0);
    int base = tile - 1;
    unsigned spins = 0;
    while (true) {
        uint64_t d[D];
        T lsum;
        bool lterm, lvalid;
        while (true) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const int idx = base - lane * D - j;
                d[j] = idx >= 0 ? lb_poll(desc + idx) : ((uint64_t)((epoch << 8) | kStInclusive) << 32);
            }
            // per lane: nearest-first fold up to (and including) the first terminator
            lsum = T(0);
            lterm = false;
            lvalid = true;
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const uint32_t hi = (uint32_t)(d[j] >> 32);
                const uint32_t st = (hi >> 8) == epoch ? (hi & 0xffu) : kStInvalid;
                if (st == kStInvalid) d[j] = 0;
                if (!lterm) {
                    lvalid = lvalid && (st != kStInvalid);
                    lsum = lsum + lb_val<T>(d[j]);
                    lterm = (st & kStInclusive) || (SEGMENTED && (st & kStFlag));
                }
            }
            const uint64_t tmask = __ballot(lterm);
            const int k = tmask ? __builtin_ctzll(tmask) : kWave;  // nearest terminating lane
            const bool need = lane <= k;
            if (!__any(need && !lvalid)) break;
            if (lb_give_up(++spins, timeout, lane)) break;
            __builtin_amdgcn_s_sleep(SLEEP);
        }
        const uint64_t tmask = __ballot(lterm);
        if (tmask) {
            const int k = __builtin_ctzll(tmask);
            prefix = prefix + wave_reduce(lane <= k ? lsum : T(0));
            return prefix;
        }
        prefix = prefix + wave_reduce(lsum);
        base -= kWave * D;
    }
}

// Probe-then-window look-back. ONE lane polls the nearest predecessor
// (tile-1) with s_sleep until it holds at least an aggregate -- one
// descriptor per poll while waiting -- then the wave reads a window of 64*D
// predecessors in one batch (D loads in flight per lane, lb_lookback). In a
// persistent grid the tiles of a round publish their aggregates at about the
// same time, so once the nearest one is valid the window almost always is,
// and the walk back to the previous round's inclusive descriptors takes one
// or two batches instead of (round position / 64) dependent 64-wide polls.
template <typename T, bool SEGMENTED, int D>
__device__ T lb_lookback_probe(uint64_t* desc, int tile, unsigned* timeout, uint32_t epoch = 0) {
    const int lane = lane_id();
    if (tile > 0) {
        for (unsigned spins = 0;; ++spins) {
            bool ok = false;
            if (lane == 0) {
                const uint32_t hi = (uint32_t)(lb_poll(desc + tile - 1) >> 32);
                ok = (hi >> 8) == epoch && (hi & 0xffu) != kStInvalid;
            }
            if (__ballot(ok)) break;
            if (lb_give_up(spins, timeout, lane)) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    return lb_lookback<T, SEGMENTED, D>(desc, tile, timeout, epoch);
}

}  // namespace cme
