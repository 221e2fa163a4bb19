// Probe: do the lanes of ONE wave-wide returning LDS atomic add that hit the
// same address see each other in lane order (lane i's old value counts every
// lower lane on its address)? If so, `old = atomicAdd(&count[wave][digit], 1)`
// is a stable in-wave radix rank in one LDS instruction, instead of the
// 8-ballot digit match of csrc/hip/sort.hip (~40 VALU instructions per key).
//
// Checks every lane of every wave-instruction over many random digit
// patterns at several digit entropies (1 .. 256 distinct digits per wave,
// inactive lanes mixed in), and times the instruction per entropy.
//
//   hipcc --offload-arch=gfx950 -O3 -o build/probe_lds_atomic_order benchmarks/probe_lds_atomic_order.hip
//   ./build/probe_lds_atomic_order
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr int kThreads = 256;
constexpr int kBins = 256;

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// digit of lane `lane` in trial t: `ndist` distinct values, some lanes inactive
__device__ __forceinline__ uint32_t digit_of(uint32_t seed, int ndist) {
    const uint32_t h = hash32(seed);
    return ndist >= kBins ? (h & 255u) : ((h % (uint32_t)ndist) * 37u) & 255u;
}

__global__ __launch_bounds__(kThreads) void order_kernel(int trials, int ndist, int inactive_pct,
                                                         unsigned* __restrict__ bad, unsigned* __restrict__ checked) {
    __shared__ uint32_t cnt[kThreads / 64][kBins];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < (kThreads / 64) * kBins; i += kThreads) (&cnt[0][0])[i] = 0;
    __syncthreads();
    unsigned nbad = 0, nchk = 0;
    for (int t = 0; t < trials; ++t) {
        const uint32_t seed = (blockIdx.x * 977u + t) * 131u + w * 7919u;
        const uint32_t d = digit_of(seed * 64u + lane, ndist);
        const bool on = (hash32(seed ^ (lane * 0x9e3779b9u)) % 100u) >= (uint32_t)inactive_pct;
        // expected: running count before this instruction + lower active lanes with the same digit
        const uint32_t before = cnt[w][d];
        uint32_t lower = 0;
        for (int l = 0; l < 64; ++l) {
            const uint32_t dl = __shfl((int)d, l);
            const int onl = __shfl((int)on, l);
            if (l < lane && onl && dl == d) ++lower;
        }
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
        uint32_t old = 0;
        if (on) old = atomicAdd(&cnt[w][d], 1u);
        __builtin_amdgcn_wave_barrier();
        if (on) {
            ++nchk;
            if (old != before + lower) ++nbad;
        }
    }
    atomicAdd(bad, nbad);
    atomicAdd(checked, nchk);
}

// cycles per returning LDS atomic wave-instruction at a digit entropy
__global__ __launch_bounds__(kThreads) void time_kernel(int iters, int ndist, unsigned long long* __restrict__ cyc,
                                                        unsigned* __restrict__ sink) {
    __shared__ uint32_t cnt[kThreads / 64][kBins];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < (kThreads / 64) * kBins; i += kThreads) (&cnt[0][0])[i] = 0;
    __syncthreads();
    uint32_t d[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = digit_of((blockIdx.x * 16u + k) * 64u + lane + w * 4096u, ndist);
    uint32_t acc = 0;
    const unsigned long long t0 = wall_clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 16; ++k) acc += atomicAdd(&cnt[w][d[k]], 1u);
    }
    __syncthreads();
    const unsigned long long t1 = wall_clock64();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    if (acc == 0xdeadbeefu) sink[0] = acc;
}

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            return 1;                                                            \
        }                                                                        \
    } while (0)

int main() {
    unsigned *bad, *chk, *sink;
    unsigned long long* cyc;
    const int blocks = 1024;
    CK(hipMalloc(&bad, 4));
    CK(hipMalloc(&chk, 4));
    CK(hipMalloc(&sink, 4));
    CK(hipMalloc(&cyc, blocks * 8));
    int wall_mhz = 100;
    {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, 0) == hipSuccess && v > 0) wall_mhz = v / 1000;
    }
    const int dists[] = {1, 2, 3, 4, 8, 16, 64, 256};
    const int inact[] = {0, 10, 50};
    unsigned total_bad = 0, total_chk = 0;
    for (int nd : dists)
        for (int ip : inact) {
            CK(hipMemset(bad, 0, 4));
            CK(hipMemset(chk, 0, 4));
            hipLaunchKernelGGL(order_kernel, dim3(blocks), dim3(kThreads), 0, 0, 256, nd, ip, bad, chk);
            CK(hipGetLastError());
            unsigned hb = 0, hc = 0;
            CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&hc, chk, 4, hipMemcpyDeviceToHost));
            printf("{\"probe\": \"lds_atomic_lane_order\", \"distinct_digits\": %d, \"inactive_pct\": %d, "
                   "\"lanes_checked\": %u, \"out_of_order\": %u}\n",
                   nd, ip, hc, hb);
            total_bad += hb;
            total_chk += hc;
        }
    unsigned long long* hcyc = new unsigned long long[blocks];
    for (int nd : dists) {
        const int iters = 64;
        hipLaunchKernelGGL(time_kernel, dim3(blocks), dim3(kThreads), 0, 0, iters, nd, cyc, sink);
        CK(hipGetLastError());
        CK(hipMemcpy(hcyc, cyc, blocks * 8, hipMemcpyDeviceToHost));
        double s = 0;
        for (int b = 0; b < blocks; ++b) s += (double)hcyc[b];
        const double ns_per_block = s / blocks * 1000.0 / wall_mhz;
        // 4 waves per block, 16 * iters instructions per wave
        printf("{\"probe\": \"lds_atomic_rtn_time\", \"distinct_digits\": %d, \"ns_per_wave_instr_per_block\": %.2f}\n",
               nd, ns_per_block / (16.0 * iters));
    }
    delete[] hcyc;
    printf("{\"probe\": \"summary\", \"lanes_checked\": %u, \"out_of_order\": %u, \"lane_ordered\": %s}\n", total_chk,
           total_bad, total_bad == 0 ? "true" : "false");
    return total_bad == 0 ? 0 : 3;
}
