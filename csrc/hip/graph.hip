// PageRank-style CSR propagation (hw1 p2):
//   out[i] = 0.5/N + 0.5 * sum_{j in row i} in[e_j] * inv_deg[e_j]
// (hw/hw1/programming/pagerank.cu:70-83; solution 1-D grid, block 128).
//
// MI355X design:
//  * prescaled gather: the propagate kernel also emits y[i] = out[i]*inv[i]
//    for the NEXT sweep, so each edge costs one 4-B random gather instead of
//    two (the float product is the same one the reference computes per edge,
//    so the thread-per-row variant stays bitwise equal to the CPU oracle);
//  * `scalar`: one lane per row (the reference mapping) -- keeps the CPU sum
//    order exactly;
//  * `group`: G lanes per row (G = 4/8/16), edges strided across the group and
//    reduced with DPP row shifts; coalesces the edge-index reads (rows have
//    1..15 edges) at the cost of a different summation order.
#include "cme213/common.h"
#include "cme213/wave.h"

// Keep a*b+c as two roundings, like the CPU oracle (bitwise parity).
#pragma clang fp contract(off)

namespace {

__global__ __launch_bounds__(256) void prescale_kernel(const float* __restrict__ x, const float* __restrict__ inv,
                                                       float* __restrict__ y, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = x[i] * inv[i];
}

// Reference arithmetic (two gathers per edge), thread per row.
__global__ __launch_bounds__(256) void pr_ref_kernel(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ edges,
                                                     const float* __restrict__ in, float* __restrict__ out,
                                                     const float* __restrict__ inv, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float sum = 0.f;
    const uint32_t e1 = idx[i + 1];
    uint32_t j = idx[i];
    for (; j + 4 <= e1; j += 4) {  // loads first, same summation order
        uint32_t c[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) c[q] = edges[j + q];
#pragma unroll
        for (int q = 0; q < 4; ++q) sum += in[c[q]] * inv[c[q]];
    }
    for (; j < e1; ++j) {
        uint32_t e = edges[j];
        sum += in[e] * inv[e];
    }
    out[i] = 0.5f / (float)n + 0.5f * sum;
}

// Prescaled, thread per row; writes out and the next sweep's y.
__global__ __launch_bounds__(256) void pr_scalar_kernel(const uint32_t* __restrict__ idx,
                                                        const uint32_t* __restrict__ edges,
                                                        const float* __restrict__ y_in, float* __restrict__ out,
                                                        float* __restrict__ y_out, const float* __restrict__ inv,
                                                        int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t b = idx[i], e = idx[i + 1];
    float sum = 0.f;
    uint32_t j = b;
    for (; j + 4 <= e; j += 4) {  // 4 edge loads in flight, then 4 gathers (same summation order)
        uint32_t c[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) c[q] = edges[j + q];
#pragma unroll
        for (int q = 0; q < 4; ++q) sum += y_in[c[q]];
    }
    for (; j < e; ++j) sum += y_in[edges[j]];
    float o = 0.5f / (float)n + 0.5f * sum;
    out[i] = o;
    y_out[i] = o * inv[i];
}

template <int G>
__global__ __launch_bounds__(256) void pr_group_kernel(const uint32_t* __restrict__ idx,
                                                       const uint32_t* __restrict__ edges,
                                                       const float* __restrict__ y_in, float* __restrict__ out,
                                                       float* __restrict__ y_out, const float* __restrict__ inv,
                                                       int n) {
    const int gid = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / G);
    const int sub = threadIdx.x % G;
    float sum = 0.f;
    if (gid < n) {
        const uint32_t b = idx[gid], e = idx[gid + 1];
        for (uint32_t j = b + sub; j < e; j += G) sum += y_in[edges[j]];
    }
    // reduce within aligned groups of G lanes (G <= 16: inside a DPP row)
    if constexpr (G >= 2) sum += __shfl_xor(sum, 1, 64);
    if constexpr (G >= 4) sum += __shfl_xor(sum, 2, 64);
    if constexpr (G >= 8) sum += __shfl_xor(sum, 4, 64);
    if constexpr (G >= 16) sum += __shfl_xor(sum, 8, 64);
    if (gid < n && sub == 0) {
        float o = 0.5f / (float)n + 0.5f * sum;
        out[gid] = o;
        y_out[gid] = o * inv[gid];
    }
}

// Column-blocked sweep (one launch per source block b of B): the edges are
// pre-sorted by (block of the gathered node, row), so a launch gathers only
// from y[b*bs, (b+1)*bs) -- 2 MB for 2^21 nodes and B = 4, resident in every
// XCD's 4 MB L2 while the edge stream passes through -- instead of the whole
// 8 MB vector (half of each gather line missing L2 into the Infinity Cache).
// Per row the block sums are accumulated in `acc` in block order; the last
// block applies 0.5/N + 0.5*sum and emits out and the next sweep's y.
template <int G>
__global__ __launch_bounds__(256) void pr_blocked_kernel(const uint32_t* __restrict__ rp,
                                                         const uint32_t* __restrict__ edges,
                                                         const float* __restrict__ y_in, float* __restrict__ acc,
                                                         float* __restrict__ out, float* __restrict__ y_out,
                                                         const float* __restrict__ inv, int n, int first, int last) {
    const int gid = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / G);
    const int sub = threadIdx.x % G;
    float sum = 0.f;
    if (gid < n) {
        const uint32_t b = rp[gid], e = rp[gid + 1];
        for (uint32_t j = b + sub; j < e; j += G) sum += y_in[__builtin_nontemporal_load(edges + j)];
    }
    if constexpr (G >= 2) sum += __shfl_xor(sum, 1, 64);
    if constexpr (G >= 4) sum += __shfl_xor(sum, 2, 64);
    if constexpr (G >= 8) sum += __shfl_xor(sum, 4, 64);
    if (gid < n && sub == 0) {
        const float a = first ? sum : acc[gid] + sum;
        if (last) {
            const float o = 0.5f / (float)n + 0.5f * a;
            out[gid] = o;
            y_out[gid] = o * inv[gid];
        } else {
            acc[gid] = a;
        }
    }
}

}  // namespace

// One blocked sweep: `blocks` launches over the (block, row)-sorted edges;
// rp holds blocks*n + 1 offsets (row i of block b: [rp[b*n+i], rp[b*n+i+1])).
CME_EXPORT int cme_pr_propagate_blocked(const uint32_t* rp, const uint32_t* edges, const float* y_in, float* acc,
                                        float* out, float* y_out, const float* inv, int n, int blocks, int group,
                                        void* stream) {
    hipStream_t s = as_stream(stream);
    if (blocks < 1) return (int)hipErrorInvalidValue;
    for (int b = 0; b < blocks; ++b) {
        const uint32_t* r = rp + (size_t)b * n;
        const int first = b == 0, last = b == blocks - 1;
        switch (group) {
            case 1:
                hipLaunchKernelGGL(pr_blocked_kernel<1>, dim3(cdiv(n, 256)), dim3(256), 0, s, r, edges, y_in, acc, out,
                                   y_out, inv, n, first, last);
                break;
            case 2:
                hipLaunchKernelGGL(pr_blocked_kernel<2>, dim3(cdiv((size_t)n * 2, 256)), dim3(256), 0, s, r, edges,
                                   y_in, acc, out, y_out, inv, n, first, last);
                break;
            case 4:
                hipLaunchKernelGGL(pr_blocked_kernel<4>, dim3(cdiv((size_t)n * 4, 256)), dim3(256), 0, s, r, edges,
                                   y_in, acc, out, y_out, inv, n, first, last);
                break;
            case 8:
                hipLaunchKernelGGL(pr_blocked_kernel<8>, dim3(cdiv((size_t)n * 8, 256)), dim3(256), 0, s, r, edges,
                                   y_in, acc, out, y_out, inv, n, first, last);
                break;
            default: return (int)hipErrorInvalidValue;
        }
        CME_TRY(hipGetLastError());
    }
    return 0;
}

CME_EXPORT int cme_pr_prescale(const float* x, const float* inv, float* y, int n, void* stream) {
    hipLaunchKernelGGL(prescale_kernel, dim3(cdiv(n, 256)), dim3(256), 0, as_stream(stream), x, inv, y, n);
    CME_LAUNCH_STATUS();
}

CME_EXPORT int cme_pr_propagate_ref(const uint32_t* idx, const uint32_t* edges, const float* in, float* out,
                                    const float* inv, int n, void* stream) {
    hipLaunchKernelGGL(pr_ref_kernel, dim3(cdiv(n, 256)), dim3(256), 0, as_stream(stream), idx, edges, in, out, inv, n);
    CME_LAUNCH_STATUS();
}

// group: 1 (scalar) or 2/4/8/16 lanes per row.
CME_EXPORT int cme_pr_propagate(const uint32_t* idx, const uint32_t* edges, const float* y_in, float* out,
                                float* y_out, const float* inv, int n, int group, void* stream) {
    hipStream_t s = as_stream(stream);
    switch (group) {
        case 1:
            hipLaunchKernelGGL(pr_scalar_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, idx, edges, y_in, out, y_out,
                               inv, n);
            break;
        case 2:
            hipLaunchKernelGGL(pr_group_kernel<2>, dim3(cdiv((size_t)n * 2, 256)), dim3(256), 0, s, idx, edges, y_in,
                               out, y_out, inv, n);
            break;
        case 4:
            hipLaunchKernelGGL(pr_group_kernel<4>, dim3(cdiv((size_t)n * 4, 256)), dim3(256), 0, s, idx, edges, y_in,
                               out, y_out, inv, n);
            break;
        case 8:
            hipLaunchKernelGGL(pr_group_kernel<8>, dim3(cdiv((size_t)n * 8, 256)), dim3(256), 0, s, idx, edges, y_in,
                               out, y_out, inv, n);
            break;
        case 16:
            hipLaunchKernelGGL(pr_group_kernel<16>, dim3(cdiv((size_t)n * 16, 256)), dim3(256), 0, s, idx, edges,
                               y_in, out, y_out, inv, n);
            break;
        default: return (int)hipErrorInvalidValue;
    }
    CME_LAUNCH_STATUS();
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(pagerank_ref, 256, pr_ref_kernel);
CME_REGISTER_KERNEL(pagerank_group8, 256, pr_group_kernel<8>);
CME_REGISTER_KERNEL(pagerank_blocked2, 256, pr_blocked_kernel<2>);
