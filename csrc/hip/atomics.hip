// Atomics and reductions from the lectures (slides/Lecture05 Monte-Carlo pi;
// slides/Lecture21 atomics: atomicAdd histogram, atomicInc work queue,
// hierarchical global max), for wave64.
//
//  monte_carlo_pi : counter-based RNG (SplitMix64 of (seed, global sample id):
//                   reproducible for any grid), per-lane hit counts, DPP wave
//                   reduce, LDS block reduce, ONE 64-bit atomic per block
//  global_max     : float max via order-preserving int mapping; wave/block
//                   reduction first, one atomicMax per block (hierarchical)
//  workqueue_sums : ragged segments pulled by persistent blocks from an atomic
//                   ticket (dequeue), each segment summed by one wave
#include "cme213/common.h"
#include "cme213/wave.h"

using namespace cme;

// x*x + y*y rounded twice, like the host evaluation of the same sample stream
#pragma clang fp contract(off)

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void mc_pi_kernel(long long samples, uint64_t seed,
                                                    unsigned long long* __restrict__ hits) {
    __shared__ unsigned long long lds[4];
    unsigned long long c = 0;
    const long long stride = (long long)gridDim.x * 256;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < samples; i += stride) {
        const uint64_t r = splitmix64(seed ^ (uint64_t)i * 0xD1B54A32D192ED03ull);
        const float x = (float)(uint32_t)r * 2.3283064365386963e-10f;  // [0,1)
        const float y = (float)(uint32_t)(r >> 32) * 2.3283064365386963e-10f;
        c += (x * x + y * y <= 1.0f);
    }
    const unsigned long long tot = block_reduce<4>(c, lds, OpAdd());
    if (threadIdx.x == 0) atomicAdd(hits, tot);
}

__device__ __forceinline__ int f2ord(float f) {
    const int i = __builtin_bit_cast(int, f);
    return i >= 0 ? i : i ^ 0x7fffffff;
}

// Hierarchical max (Lecture21): lane -> wave (DPP) -> block (LDS) -> one
// atomicMax per block on an order-preserving int image of the float. Lanes
// stream 16-B vectors, four independent loads in flight per iteration.
__global__ __launch_bounds__(256) void global_max_kernel(const float* __restrict__ in, long long n,
                                                         int* __restrict__ out) {
    __shared__ float lds[4];
    float m = -__builtin_huge_valf();
    const long long n4 = ((uintptr_t)in % 16) ? 0 : n / 4;
    const float4* in4 = reinterpret_cast<const float4*>(in);
    const long long stride = (long long)gridDim.x * 256;
    long long i = blockIdx.x * 256LL + threadIdx.x;
    for (; i + 3 * stride < n4; i += 4 * stride) {
        const float4 a = in4[i], b = in4[i + stride], c = in4[i + 2 * stride], d = in4[i + 3 * stride];
        m = fmaxf(m, fmaxf(fmaxf(fmaxf(a.x, a.y), fmaxf(a.z, a.w)), fmaxf(fmaxf(b.x, b.y), fmaxf(b.z, b.w))));
        m = fmaxf(m, fmaxf(fmaxf(fmaxf(c.x, c.y), fmaxf(c.z, c.w)), fmaxf(fmaxf(d.x, d.y), fmaxf(d.z, d.w))));
    }
    for (; i < n4; i += stride) {
        const float4 a = in4[i];
        m = fmaxf(m, fmaxf(fmaxf(a.x, a.y), fmaxf(a.z, a.w)));
    }
    for (long long j = 4 * n4 + blockIdx.x * 256LL + threadIdx.x; j < n; j += stride) m = fmaxf(m, in[j]);
    const float b = block_reduce<4>(m, lds, OpMax());
    if (threadIdx.x == 0) atomicMax(out, f2ord(b));
}

__global__ __launch_bounds__(256) void workqueue_kernel(const int* __restrict__ offsets, int nseg,
                                                        const float* __restrict__ v, float* __restrict__ out,
                                                        unsigned* __restrict__ head) {
    const int lane = lane_id();
    // bounded: a wave can never dequeue more than nseg + 1 times
    for (int iter = 0; iter <= nseg; ++iter) {
        unsigned t = 0;
        if (lane == 0) t = atomicAdd(head, 1u);  // dequeue one segment per wave
        const int seg = (int)__shfl(t, 0, kWave);
        if (seg >= nseg) return;  // every wave reaches this exit
        const int b = offsets[seg], e = offsets[seg + 1];
        float s = 0.f;
        for (int i = b + lane; i < e; i += kWave) s += v[i];
        s = wave_reduce(s);
        if (lane == 0) out[seg] = s;
    }
}

}  // namespace

CME_EXPORT int cme_monte_carlo_pi(long long samples, unsigned long long seed, unsigned long long* hits,
                                  void* stream) {
    hipStream_t s = as_stream(stream);
    CME_TRY(hipMemsetAsync(hits, 0, 8, s));
    hipLaunchKernelGGL(mc_pi_kernel, dim3(stream_grid(samples, 256, 4)), dim3(256), 0, s, samples, (uint64_t)seed,
                       hits);
    CME_LAUNCH_STATUS();
}

// out: one int (order-mapped float); decode on the host.
CME_EXPORT int cme_global_max(const float* in, long long n, int* out, void* stream) {
    hipStream_t s = as_stream(stream);
    CME_TRY(hipMemsetAsync(out, 0x80, 4, s));  // 0x80808080: far below any mapped float
    hipLaunchKernelGGL(global_max_kernel, dim3(stream_grid((n + 15) / 16, 256, 4)), dim3(256), 0, s, in, n, out);
    CME_LAUNCH_STATUS();
}

// head: one uint of scratch (zeroed here). Grid: 4 blocks of 256 per CU.
CME_EXPORT int cme_workqueue_segment_sums(const int* offsets, int nseg, const float* v, float* out, unsigned* head,
                                          void* stream) {
    hipStream_t s = as_stream(stream);
    CME_TRY(hipMemsetAsync(head, 0, 4, s));
    hipLaunchKernelGGL(workqueue_kernel, dim3(4 * kNumCU), dim3(256), 0, s, offsets, nseg, v, out, head);
    CME_LAUNCH_STATUS();
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(monte_carlo_pi, 256, mc_pi_kernel);
CME_REGISTER_KERNEL(global_max, 256, global_max_kernel);
