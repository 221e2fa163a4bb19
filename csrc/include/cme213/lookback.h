// Single-pass decoupled look-back (Merrill & Garland) for wave64 / gfx950.
//
// Inter-workgroup hand-off follows the "data IS the flag" form for payloads
// <= 4 KB (cdna_hip_programming.md §6 Guideline 16, R2): each tile publishes
// ONE naturally aligned 8-byte granule {status/flags : 32 | value bits : 32}
// with a relaxed agent-scope atomic store (global_store ... sc1) and
// predecessors' granules are re-read with relaxed agent-scope atomic loads
// (sc1, bypassing the per-CU L1). No fences are needed and results do not
// depend on dispatch order or XCD placement. Tile ids come from an atomic
// ticket so every predecessor of a tile is already resident or finished
// (forward progress without co-residency assumptions). The descriptor array
// and the ticket are zeroed by the launcher (hipMemsetAsync) before EVERY
// launch. Spins are bounded: a tile that waits > kSpinLimit polls sets the
// timeout word and continues (the launcher reports it), so a bug can never
// hang the GPU.
#pragma once
#include "common.h"
#include "wave.h"

namespace cme {

enum : uint32_t { kStInvalid = 0, kStAggregate = 1, kStInclusive = 2, kStFlag = 4 };
constexpr unsigned kSpinLimit = 1u << 22;

__device__ __forceinline__ void lb_publish(uint64_t* d, uint32_t status, uint32_t vbits) {
    __hip_atomic_store(d, ((uint64_t)status << 32) | vbits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
template <typename T, bool SEGMENTED>
__device__ T lb_lookback(uint64_t* desc, int tile, unsigned* timeout) {
    const int lane = lane_id();
    T prefix = T(0);
    int base = tile - 1;
    unsigned spins = 0;
    while (true) {
        const int idx = base - lane;
        uint64_t d;
        uint32_t st;
        while (true) {
            d = idx >= 0 ? lb_poll(desc + idx) : ((uint64_t)kStInclusive << 32);
            st = (uint32_t)(d >> 32);
            if (!__any(st == kStInvalid)) break;
            if (++spins > kSpinLimit) {
                if (lane == 0) atomicOr(timeout, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const bool term = (st & kStInclusive) || (SEGMENTED && (st & kStFlag));
        const uint64_t mask = __ballot(term);
        T v = lb_val<T>(d);
        if (mask) {
            const int k = __builtin_ctzll(mask);
            v = lane <= k ? v : T(0);
            prefix = prefix + wave_reduce(v);
            return prefix;
        }
        prefix = prefix + wave_reduce(v);
        base -= kWave;
    }
}

}  // namespace cme
