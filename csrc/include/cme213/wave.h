// Wave64 cooperative primitives built on DPP (data-parallel primitives).
//
// The reference's warp-synchronous scan (hw/hw_final/programming/fp.cu:28-37)
// relies on implicit 32-lane lock-step over global memory; on CDNA the wave is
// 64 lanes and we move data between lanes in registers with DPP instead:
//   row_shr:1,2,4,8  -> Hillis-Steele inside each 16-lane row
//   row_bcast:15     -> carry row 0 -> row 1, row 2 -> row 3
//   row_bcast:31     -> carry lanes 0-31 -> lanes 32-63
// Six VALU ops per 32-bit scan, no LDS traffic (Lecture16 "intra-warp scan",
// my-refs/nvr-2008-003.pdf, re-derived for 64 lanes).
#pragma once
#include "common.h"

namespace cme {

// LDS hand-offs between lanes / waves -- the two documented patterns
// (ISA-verified: scripts/check_lds_barriers.py, profiles/lds_broadcast_isa_r6.md).
//
// lds_bcast_sync(): a value one lane (or a few) wrote to LDS, read by the
// other waves of the workgroup. The writers' ds_write must have completed
// before the barrier lets the readers go: __syncthreads() normally carries an
// s_waitcnt lgkmcnt(0) for that, but hipcc drops it when the barrier heads a
// loop and the write sits at the end of the loop body (the dataflow launch's
// ticket loop), so the wait is explicit here. Every wave executes it (it only
// waits for the wave's own LDS operations; free where the compiler already
// waits).
__device__ __forceinline__ void lds_bcast_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
}

// wave_lds_sync(): LDS written by some lanes of a wave and read by other
// lanes of the SAME wave (in-wave trees). A wave's LDS operations execute in
// order, so no s_waitcnt is needed; __builtin_amdgcn_wave_barrier is only a
// convergence / scheduling barrier that does not order memory, so the
// wavefront-scope fences keep the optimiser from moving or forwarding LDS
// accesses across it (they emit no instruction).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// DPP control codes (GFX9 encoding; gfx950 is GFX9-family).
enum : int {
    kDppRowShr1 = 0x111,
    kDppRowShr2 = 0x112,
    kDppRowShr4 = 0x114,
    kDppRowShr8 = 0x118,
    kDppWaveShl1 = 0x130,
    kDppWaveShr1 = 0x138,
    kDppRowBcast15 = 0x142,
    kDppRowBcast31 = 0x143,
};

template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t old, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, CTRL, ROW_MASK, BANK_MASK, false);
}

// Pure lane shift: lanes with no source lane read 0 (bound_ctrl) and there is
// no `old` operand, so the compiler need not copy the source register first.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_shift_u32(uint32_t src) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)src, CTRL, 0xf, 0xf, true);
}

template <typename T> struct Bits;
template <> struct Bits<float> { using U = uint32_t; };
template <> struct Bits<int> { using U = uint32_t; };
template <> struct Bits<uint32_t> { using U = uint32_t; };
template <> struct Bits<double> { using U = uint64_t; };
template <> struct Bits<long long> { using U = uint64_t; };
template <> struct Bits<unsigned long long> { using U = uint64_t; };

// Move `src` across lanes by DPP; lanes with no valid source (or masked rows)
// receive `old`. 64-bit types are moved as two 32-bit halves.
template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf, typename T>
__device__ __forceinline__ T dpp_move(T old, T src) {
    using U = typename Bits<T>::U;
    if constexpr (sizeof(T) == 4) {
        U r = dpp_u32<CTRL, ROW_MASK, BANK_MASK>(__builtin_bit_cast(U, old), __builtin_bit_cast(U, src));
        return __builtin_bit_cast(T, r);
    } else {
        U o = __builtin_bit_cast(U, old), s = __builtin_bit_cast(U, src);
        uint32_t lo = dpp_u32<CTRL, ROW_MASK, BANK_MASK>((uint32_t)o, (uint32_t)s);
        uint32_t hi = dpp_u32<CTRL, ROW_MASK, BANK_MASK>((uint32_t)(o >> 32), (uint32_t)(s >> 32));
        return __builtin_bit_cast(T, ((U)hi << 32) | lo);
    }
}

struct OpAdd {
    template <typename T> __device__ __forceinline__ T operator()(T a, T b) const { return a + b; }
    template <typename T> __device__ __forceinline__ static T identity() { return T(0); }
};
struct OpMax {
    template <typename T> __device__ __forceinline__ T operator()(T a, T b) const { return a > b ? a : b; }
    template <typename T> __device__ __forceinline__ static T identity();
};
template <> __device__ __forceinline__ float OpMax::identity<float>() { return -__builtin_huge_valf(); }
template <> __device__ __forceinline__ double OpMax::identity<double>() { return -__builtin_huge_val(); }
template <> __device__ __forceinline__ int OpMax::identity<int>() { return (int)0x80000000; }
template <> __device__ __forceinline__ uint32_t OpMax::identity<uint32_t>() { return 0u; }
struct OpMin {
    template <typename T> __device__ __forceinline__ T operator()(T a, T b) const { return a < b ? a : b; }
    template <typename T> __device__ __forceinline__ static T identity();
};
template <> __device__ __forceinline__ float OpMin::identity<float>() { return __builtin_huge_valf(); }
template <> __device__ __forceinline__ double OpMin::identity<double>() { return __builtin_huge_val(); }
template <> __device__ __forceinline__ int OpMin::identity<int>() { return 0x7fffffff; }
template <> __device__ __forceinline__ uint32_t OpMin::identity<uint32_t>() { return 0xffffffffu; }

// Inclusive scan across the 64 lanes of a wave (all lanes must be active).
template <typename Op = OpAdd, typename T>
__device__ __forceinline__ T wave_inclusive_scan(T v, Op op = Op()) {
    const T id = Op::template identity<T>();
    v = op(v, dpp_move<kDppRowShr1>(id, v));
    v = op(v, dpp_move<kDppRowShr2>(id, v));
    v = op(v, dpp_move<kDppRowShr4>(id, v));
    v = op(v, dpp_move<kDppRowShr8>(id, v));
    v = op(v, dpp_move<kDppRowBcast15, 0xa>(id, v));
    v = op(v, dpp_move<kDppRowBcast31, 0xc>(id, v));
    return v;
}

template <typename T>
__device__ __forceinline__ T wave_readlane(T v, int lane) {
    using U = typename Bits<T>::U;
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, (U)__builtin_amdgcn_readlane((int)__builtin_bit_cast(U, v), lane));
    } else {
        U u = __builtin_bit_cast(U, v);
        uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, lane);
        uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), lane);
        return __builtin_bit_cast(T, ((U)hi << 32) | lo);
    }
}

// Exclusive scan: shift the inclusive result right by one lane (wave_shr:1).
template <typename Op = OpAdd, typename T>
__device__ __forceinline__ T wave_exclusive_scan(T v, T* total = nullptr, Op op = Op()) {
    T inc = wave_inclusive_scan<Op>(v, op);
    if (total) *total = wave_readlane(inc, kWave - 1);
    return dpp_move<kDppWaveShr1>(Op::template identity<T>(), inc);
}

// Full-wave reduction; result is wave-uniform (scalar register).
template <typename Op = OpAdd, typename T>
__device__ __forceinline__ T wave_reduce(T v, Op op = Op()) {
    return wave_readlane(wave_inclusive_scan<Op>(v, op), kWave - 1);
}

// Block-wide exclusive scan for blockDim.x = NW * 64 threads. `lds` must hold
// NW values. Returns this thread's exclusive prefix and the block total.
template <int NW, typename Op = OpAdd, typename T>
__device__ __forceinline__ T block_exclusive_scan(T v, T* lds, T& total, Op op = Op()) {
    const int lane = lane_id();
    const int wid = threadIdx.x / kWave;
    T wtot;
    T ex = wave_exclusive_scan<Op>(v, &wtot, op);
    if (lane == 0) lds[wid] = wtot;
    lds_bcast_sync();
    T carry = Op::template identity<T>();
    T run = Op::template identity<T>();
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        T x = lds[w];
        if (w < wid) carry = op(carry, x);
        run = op(run, x);
    }
    total = run;
    __syncthreads();
    return op(carry, ex);
}

template <int NW, typename Op = OpAdd, typename T>
__device__ __forceinline__ T block_reduce(T v, T* lds, Op op = Op()) {
    const int lane = lane_id();
    const int wid = threadIdx.x / kWave;
    T w = wave_reduce<Op>(v, op);
    if (lane == 0) lds[wid] = w;
    lds_bcast_sync();
    T run = Op::template identity<T>();
#pragma unroll
    for (int i = 0; i < NW; ++i) run = op(run, lds[i]);
    __syncthreads();
    return run;
}

template <int CTRL, typename T>
__device__ __forceinline__ T dpp_shift(T src) {
    using U = typename Bits<T>::U;
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, dpp_shift_u32<CTRL>(__builtin_bit_cast(U, src)));
    } else {
        const U s = __builtin_bit_cast(U, src);
        const uint32_t lo = dpp_shift_u32<CTRL>((uint32_t)s);
        const uint32_t hi = dpp_shift_u32<CTRL>((uint32_t)(s >> 32));
        return __builtin_bit_cast(T, ((U)hi << 32) | lo);
    }
}

}  // namespace cme
