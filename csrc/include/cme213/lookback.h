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
// Bounded spins: ~2^20 polls (about a second) per wait, and the timeout
// word is STICKY -- every 256 polls a waiter re-reads it and gives up at once
// if any tile already timed out, so a broken launch (e.g. a grid that is not
// co-resident) ends in about one spin limit instead of one per tile.
constexpr unsigned kSpinLimit = 1u << 20;

__device__ __forceinline__ bool lb_give_up(unsigned spins, unsigned* timeout, int lane) {
    if (spins > kSpinLimit) {
        if (lane == 0) __hip_atomic_store(timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return true;
    }
    if ((spins & 255u) == 255u)
        return __hip_atomic_load(timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
    return false;
}

// The timeout word the kernels set lives in pinned, mapped HOST memory, one
// per device (lb_host_timeout, scan.hip): it is never reset by a launch, so a
// timed-out launch poisons the following ones on that device (they give up
// at once) until the host reads and clears it -- ops/scan.py does that
// before every look-back call and raises, without a device synchronisation.
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

// ------------------------------------------------------ two-level look-back
// The one-level walk above advances the "inclusive frontier" by at most 64
// tiles per dependent poll, so a launch costs about tiles/64 sequential poll
// latencies (2^26 fp32, 8192 tiles: ~0.26 us x 128 = the measured 33 us over
// the no-look-back arm). Two levels make that ~2 polls per tile:
//   agg[t]   aggregate of tile t, published as soon as the tile is reduced,
//            never changed;
//   inc[t]   inclusive prefix through tile t, after its look-back;
//   gagg[g]  aggregate of the 64 tiles of group g, published by the group's
//            LAST tile as soon as the group's 64 aggregates are valid;
//   ginc[g]  inclusive prefix through group g (the last tile's inc).
// Tile t = 64g + j walks its own group's j predecessors (one 64-wide poll of
// agg/inc), then groups g-1, g-2, ... 64 per poll (4096 tiles per poll), each
// ending at the nearest inclusive entry. SEGMENTED: an aggregate carrying
// kStFlag (a segment head inside) also ends a walk -- its value is the running
// value at its end -- and aggregates combine as (f, v) . (f', v') =
// (f | f', f' ? v' : v + v'). Granules: hi = (epoch << 8) | status (status 0 =
// not yet published), lo = value bits; the arrays are zeroed once per launch
// (or per multi-iteration run, with a new epoch per iteration). Every wait
// depends only on aggregates published at tile start or on inclusive values
// of strictly earlier tiles, so a co-resident grid always makes progress.
struct Lb2 {
    uint64_t *agg, *inc, *gagg, *ginc;
};
static inline size_t lb2_ws_bytes(long long tiles) { return 16 + 16 * (size_t)tiles + 16 * (size_t)((tiles + 63) / 64); }
__host__ __device__ static inline Lb2 lb2_views(uint64_t* desc, long long tiles) {
    const long long groups = (tiles + 63) / 64;
    return Lb2{desc, desc + tiles, desc + 2 * tiles, desc + 2 * tiles + groups};
}
template <typename T>
__device__ __forceinline__ void lb2_put(uint64_t* d, T v, uint32_t flag = 0, uint32_t epoch = 0) {
    lb_publish(d, kStAggregate | flag, lb_bits(v), epoch);
}
__device__ __forceinline__ uint32_t lb2_status(uint64_t d, uint32_t epoch) {
    const uint32_t hi = (uint32_t)(d >> 32);
    return (hi >> 8) == epoch ? (hi & 0xffu) : 0u;
}

// One wave: lanes l < n inspect predecessor slot base - l of (a, inc).
// Returns (via *sum) the combination of the entries nearer than the
// nearest terminating one (a valid inc, or a flagged agg when SEGMENTED) plus
// that entry, and whether a terminator was found. `virt0`: slots before 0 are
// an inclusive 0 (the start of the array). `all_agg`: additionally require
// EVERY lane's aggregate and fold them all into (*gsum, *gflag) -- the group's
// last tile builds gagg from them.
template <typename T, bool SEG>
__device__ __forceinline__ bool lb2_window(const uint64_t* a, const uint64_t* inc, int base, int n, bool virt0,
                                           bool all_agg, uint32_t epoch, T* sum, T* gsum, uint32_t* gflag,
                                           unsigned* timeout) {
    const int lane = lane_id();
    for (unsigned spins = 0;; ++spins) {
        const int idx = base - lane;
        const bool act = lane < n && idx >= 0;
        const bool virt = lane < n && idx < 0 && virt0;
        const uint64_t da = act ? lb_poll((uint64_t*)a + idx) : 0;
        const uint64_t di = act ? lb_poll((uint64_t*)inc + idx) : 0;
        const uint32_t sa = lb2_status(da, epoch), si = lb2_status(di, epoch);
        const bool aval = act && sa != 0u;
        const bool aflag = SEG && aval && (sa & kStFlag);
        const bool ival = (act && si != 0u) || virt;
        const bool term = ival || aflag;
        const uint64_t tm = __ballot(term);
        const int k = tm ? __builtin_ctzll(tm) : kWave;
        bool bad = lane < k && lane < n && !virt && !aval;
        if (all_agg) bad = bad || (act && !aval);
        if (!__any(bad)) {
            // lane k contributes its inclusive value (or its flagged aggregate)
            const bool use_inc = lane == k && act && si != 0u;
            const T c = lane < k ? (aval ? lb_val<T>(da) : T(0)) : (lane == k && act ? lb_val<T>(use_inc ? di : da) : T(0));
            *sum = wave_reduce(c);
            if (all_agg) {
                // ordered segmented fold of every aggregate (nearest first):
                // stop at the nearest flagged one
                const uint64_t fm = SEG ? __ballot(aflag) : 0ull;
                const int kf = fm ? __builtin_ctzll(fm) : kWave;
                *gsum = wave_reduce(act && lane <= kf ? lb_val<T>(da) : T(0));
                *gflag = kf < kWave ? 1u : 0u;
            }
            return k < kWave;
        }
        if (lb_give_up(spins, timeout, lane)) {
            *sum = T(0);
            if (all_agg) *gsum = T(0), *gflag = 0u;
            return true;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// Exclusive prefix of tile `tile` (aggregate (tot, tot_flag) already in
// agg[]); publishes inc[tile] (and gagg / ginc for a group's last tile). For
// SEGMENTED the returned prefix is the running value entering the tile (the
// caller ignores it past the tile's first head). One wave.
template <typename T, bool SEG = false>
__device__ T lb2_lookback(Lb2 w, int tile, int tiles, T tot, uint32_t tot_flag, unsigned* timeout,
                          uint32_t epoch = 0) {
    const int lane = lane_id();
    const int g = tile >> 6, j = tile & 63;
    const bool last = j == 63 || tile == tiles - 1;
    T prefix = T(0), gsum = T(0);
    uint32_t gflag = 0u;
    bool done = false;
    if (j > 0) done = lb2_window<T, SEG>(w.agg, w.inc, tile - 1, j, false, last, epoch, &prefix, &gsum, &gflag, timeout);
    if (last && lane == 0) {  // unblock later groups before walking on
        const T gv = tot_flag ? tot : gsum + tot;
        lb2_put(w.gagg + g, gv, (tot_flag | gflag) ? kStFlag : 0u, epoch);
    }
    for (int gb = g - 1; !done && gb >= 0; gb -= kWave) {
        T s, gs;
        uint32_t gf;
        done = lb2_window<T, SEG>(w.gagg, w.ginc, gb, kWave, true, false, epoch, &s, &gs, &gf, timeout);
        prefix = prefix + s;
    }
    if (lane == 0) {
        const T incl = tot_flag ? tot : prefix + tot;
        const uint32_t fl = tot_flag ? kStFlag : 0u;  // informational only: inc always terminates a walk
        lb2_put(w.inc + tile, incl, fl, epoch);
        if (last) lb2_put(w.ginc + g, incl, fl, epoch);
    }
    return prefix;
}

}  // namespace cme
