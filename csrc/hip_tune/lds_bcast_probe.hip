// Reproducer of the lane-0 LDS broadcast hazard seen in the dataflow launch
// (csrc/hip_tune/heat_flow.hip, profiles/lds_broadcast_isa_r6.md).
//
// The pattern: lane 0 of wave 0 fetches a value with a global atomic (so its
// ds_write issues late, right before the barrier), writes it to LDS, and the
// workgroup's other waves read it after __syncthreads(). hipcc lowers
// __syncthreads() on gfx950 to s_barrier with NO s_waitcnt lgkmcnt(0) in
// front of it when only LDS has to be ordered: LLVM's memory model assumes
// that LDS operations of all waves of a CU execute in one global order, so an
// issued ds_write precedes every ds_read issued after the barrier. Here every
// workgroup hammers LDS between the barriers (as the pipelined pass's ring
// hand-offs do, 8 workgroups per CU) and counts the iterations in which a
// wave read the PREVIOUS ticket after the barrier. WAIT = 1 adds the explicit
// wait the production kernels use (cme::lds_bcast_sync, wave.h).
#include "cme213/common.h"
#include "cme213/wave.h"

using namespace cme;

namespace {

template <bool WAIT>
__global__ __launch_bounds__(256) void lds_bcast_probe_kernel(unsigned* ticket, unsigned* stale, float* sink,
                                                              unsigned total) {
    __shared__ unsigned s_tk;
    __shared__ float4 ring[4][64];
    const int lane = lane_id();
    const int wv = (int)(threadIdx.x / 64);
    const unsigned s_addr = (unsigned)(size_t)&s_tk;  // LDS offset: the low 32 bits of the generic address
    float4 acc = {(float)lane, 0.f, 0.f, 0.f};
    unsigned bad = 0, last = 0xffffffffu;
    for (;;) {
        // lane 0 fetches the next ticket and writes it to LDS; the barrier
        // follows the ds_write in the SAME asm block, so nothing can be
        // scheduled in between: WAIT = 0 is exactly the sequence hipcc
        // emitted in heat_flow.hip (ds_write ... s_barrier), WAIT = 1 the
        // fixed one (ds_write, s_waitcnt lgkmcnt(0), s_barrier)
        if (threadIdx.x == 0) {
            const unsigned v = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if constexpr (WAIT)
                asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"v"(s_addr), "v"(v) : "memory");
            else
                asm volatile("ds_write_b32 %0, %1\n\ts_barrier" ::"v"(s_addr), "v"(v) : "memory");
        } else if (wv != 0) {
            asm volatile("s_barrier" ::: "memory");
        }
        const unsigned t = (unsigned)__builtin_amdgcn_readfirstlane((int)s_tk);
        if (t >= total) break;
        // every fetch returns a new ticket: reading the last one is stale
        if (t == last) ++bad;
        last = t;
        // LDS traffic of all waves (and of the CU's other workgroups) until
        // the next fetch, as the pipelined pass's ring hand-offs
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            ring[wv][lane] = acc;
            const float4 v = ring[(wv + 1) & 3][lane ^ (r + 1)];
            acc.x += v.y;
            acc.y += v.z;
            acc.z += v.w;
            acc.w += v.x;
        }
        __syncthreads();  // every wave has read s_tk before lane 0 overwrites it
    }
    if (lane == 0 && bad) atomicAdd(stale, bad);
    if (acc.x == 1234.5f) sink[threadIdx.x] = acc.y + acc.z + acc.w;  // keep the traffic
}

}  // namespace

// `total` tickets handed out to `blocks` workgroups of 4 waves, without
// (wait = 0) or with (wait = 1) the explicit lgkmcnt(0) wait after the LDS
// write; *stale_out = wave-iterations that read a stale ticket (synchronous).
CME_EXPORT int cme_lds_bcast_probe(int wait, int blocks, unsigned total, unsigned long long* stale_out) {
    unsigned* d = nullptr;
    float* sink = nullptr;
    CME_TRY(hipMalloc(&d, 8));
    CME_TRY(hipMalloc(&sink, 256 * sizeof(float)));
    CME_TRY(hipMemset(d, 0, 8));
    if (wait)
        hipLaunchKernelGGL(lds_bcast_probe_kernel<true>, dim3(blocks), dim3(256), 0, nullptr, d, d + 1, sink, total);
    else
        hipLaunchKernelGGL(lds_bcast_probe_kernel<false>, dim3(blocks), dim3(256), 0, nullptr, d, d + 1, sink, total);
    CME_TRY(hipGetLastError());
    unsigned h[2] = {0, 0};
    CME_TRY(hipMemcpy(h, d, 8, hipMemcpyDeviceToHost));
    CME_TRY(hipFree(d));
    CME_TRY(hipFree(sink));
    *stale_out = h[1];
    return 0;
}
