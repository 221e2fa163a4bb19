// Lecture micro-studies (slides/Lecture04), wave64 edition.
//
//  divergence     : every lane runs one of two equally long dependent FMA
//                   chains selected by (threadIdx.x / stride) & 1. With
//                   stride >= 64 each wave takes one path; below 64 both
//                   paths execute under EXEC masks (2x the issue slots) --
//                   the warp-serialisation experiment of slides 4-12 with the
//                   threshold at the 64-lane wave instead of the 32-lane warp.
//  strided_copy   : out[i] = in[i * stride + offset] -- the coalescing study
//                   of slides 13-20: effective bandwidth vs. stride (bytes
//                   fetched per useful byte) and vs. misalignment offset.
#include "cme213/common.h"

namespace {

__global__ __launch_bounds__(256) void divergence_kernel(float* __restrict__ out, long long n, int stride, int work) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float x = (float)(i & 1023) * 1e-3f;
    if ((threadIdx.x / stride) & 1) {
        for (int k = 0; k < work; ++k) x = __builtin_fmaf(x, 1.0001f, 0.5f);
    } else {
        for (int k = 0; k < work; ++k) x = __builtin_fmaf(x, 0.9999f, -0.25f);
    }
    out[i] = x;
}

__global__ __launch_bounds__(256) void strided_copy_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                           long long n, int stride, int offset) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
        out[i] = in[i * stride + offset];
}

}  // namespace

CME_EXPORT int cme_divergence(float* out, long long n, int stride, int work, void* stream) {
    if (stride < 1) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(divergence_kernel, dim3(cdiv(n, 256)), dim3(256), 0, as_stream(stream), out, n, stride, work);
    CME_LAUNCH_STATUS();
}

// `in` must hold (n - 1) * stride + offset + 1 floats.
CME_EXPORT int cme_strided_copy(const float* in, float* out, long long n, int stride, int offset, void* stream) {
    if (stride < 1 || offset < 0) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(strided_copy_kernel, dim3(stream_grid(n, 256)), dim3(256), 0, as_stream(stream), in, out, n,
                       stride, offset);
    CME_LAUNCH_STATUS();
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(divergence, 256, divergence_kernel);
CME_REGISTER_KERNEL(strided_copy, 256, strided_copy_kernel);
