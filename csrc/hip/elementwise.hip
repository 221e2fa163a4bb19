// Streaming element-wise kernels: Caesar shift cipher (hw1 p1), copy (HBM
// calibration), and the fused multiply used by the SpMV-scan.
//
// The reference studies bytes-per-lane on Fermi (hw/hw1/programming/cipher.cu:
// 64-92: uchar / packed uint / uint2 = 1/4/8 B per thread, block 512, 2-D grid
// to dodge the 65535 limit). On CDNA4 the same ladder is 1/4/8/16 B per lane;
// 16 B (dwordx4) is what the memory pipe wants. Kernels are grid-stride with a
// grid sized to fill 256 CUs, and each lane keeps UNROLL independent 16-B loads
// in flight. Byte-wise adds on packed words are carry-free (SWAR), so every
// width gives the same bytes as the scalar reference for any shift/input.
#include "cme213/common.h"

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Byte-wise (mod 256) add of two packed 32-bit words, no inter-byte carries.
__device__ __forceinline__ uint32_t add_bytes(uint32_t a, uint32_t b) {
    return ((a & 0x7f7f7f7fu) + (b & 0x7f7f7f7fu)) ^ ((a ^ b) & 0x80808080u);
}

__global__ __launch_bounds__(256) void shift_u8_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                       size_t n, uint8_t shift) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = (uint8_t)(in[i] + shift);
}

__global__ __launch_bounds__(256) void shift_u32_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                        size_t n, uint32_t s4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = add_bytes(in[i], s4);
}

__global__ __launch_bounds__(256) void shift_u64_kernel(const uint2* __restrict__ in, uint2* __restrict__ out,
                                                        size_t n, uint32_t s4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint2 v = in[i];
        out[i] = make_uint2(add_bytes(v.x, s4), add_bytes(v.y, s4));
    }
}

template <int UNROLL>
__global__ __launch_bounds__(256) void shift_u128_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                                         size_t n, uint32_t s4) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    auto f = [s4](u32x4 v) {
        u32x4 r;
        r.x = add_bytes(v.x, s4);
        r.y = add_bytes(v.y, s4);
        r.z = add_bytes(v.z, s4);
        r.w = add_bytes(v.w, s4);
        return r;
    };
    for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = __builtin_nontemporal_load(&in[i + u * stride]);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) __builtin_nontemporal_store(f(v[u]), &out[i + u * stride]);
    }
    for (; i < n; i += stride) out[i] = f(in[i]);
}

// Copy-rate calibration space: UNROLL x {nt, plain} x grid size.
template <int UNROLL, bool NT>
__global__ __launch_bounds__(256) void copy_tune_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                                        size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            if constexpr (NT) v[u] = __builtin_nontemporal_load(&in[i + u * stride]);
            else v[u] = in[i + u * stride];
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            if constexpr (NT) __builtin_nontemporal_store(v[u], &out[i + u * stride]);
            else out[i + u * stride] = v[u];
        }
    }
    for (; i < n; i += stride) out[i] = in[i];
}

// One-shot copy: a block moves ONE contiguous 256 x UNROLL-vector tile and
// exits (no grid stride): tens of thousands of short-lived blocks keep more
// bytes in flight than a persistent grid. Non-temporal loads and stores.
template <int UNROLL>
__global__ __launch_bounds__(256) void copy_flat_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                                        size_t n) {
    const size_t b0 = (size_t)blockIdx.x * 256 * UNROLL + threadIdx.x;
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
        if (b0 + u * 256 < n) v[u] = __builtin_nontemporal_load(&in[b0 + u * 256]);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
        if (b0 + u * 256 < n) __builtin_nontemporal_store(v[u], &out[b0 + u * 256]);
}

// Block-contiguous copy: each block streams one contiguous chunk (no grid stride).
template <int UNROLL>
__global__ __launch_bounds__(256) void copy_chunk_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                                         size_t n, size_t per_block) {
    size_t b0 = blockIdx.x * per_block;
    size_t b1 = b0 + per_block < n ? b0 + per_block : n;
    for (size_t i = b0 + threadIdx.x; i < b1; i += 256 * UNROLL) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            if (i + u * 256 < b1) v[u] = in[i + u * 256];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            if (i + u * 256 < b1) out[i + u * 256] = v[u];
    }
}

// a[i] *= b[i] (float), 16 B per lane.
__global__ __launch_bounds__(256) void mul_f32_kernel(float* __restrict__ a, const float* __restrict__ b, size_t n4,
                                                      size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
        float4 x = reinterpret_cast<float4*>(a)[i];
        float4 y = reinterpret_cast<const float4*>(b)[i];
        x.x *= y.x;
        x.y *= y.y;
        x.z *= y.z;
        x.w *= y.w;
        reinterpret_cast<float4*>(a)[i] = x;
    }
    for (size_t i = n4 * 4 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) a[i] *= b[i];
}

}  // namespace

// width: 1, 4, 8 or 16 bytes per lane. Pointers must be aligned to `width`;
// the tail (< width bytes) is processed by the byte kernel.
CME_EXPORT int cme_shift_cipher(const uint8_t* in, uint8_t* out, long long n, int shift, int width, int block,
                                void* stream) {
    hipStream_t s = as_stream(stream);
    const uint8_t sh = (uint8_t)shift;
    const uint32_t s4 = 0x01010101u * sh;
    if (block <= 0) block = 256;
    size_t body = 0;
    if (width == 1) {
        hipLaunchKernelGGL(shift_u8_kernel, dim3(stream_grid(n, block)), dim3(block), 0, s, in, out, (size_t)n, sh);
        CME_LAUNCH_STATUS();
    }
    if (width == 4) {
        size_t m = n / 4;
        if (m) hipLaunchKernelGGL(shift_u32_kernel, dim3(stream_grid(m, block)), dim3(block), 0, s,
                                  (const uint32_t*)in, (uint32_t*)out, m, s4);
        body = m * 4;
    } else if (width == 8) {
        size_t m = n / 8;
        if (m) hipLaunchKernelGGL(shift_u64_kernel, dim3(stream_grid(m, block)), dim3(block), 0, s,
                                  (const uint2*)in, (uint2*)out, m, s4);
        body = m * 8;
    } else if (width == 16) {
        size_t m = n / 16;
        if (m) hipLaunchKernelGGL(shift_u128_kernel<4>, dim3(stream_grid(m, block, 4)), dim3(block), 0, s,
                                  (const u32x4*)in, (u32x4*)out, m, s4);
        body = m * 16;
    } else {
        return (int)hipErrorInvalidValue;
    }
    if ((size_t)n > body)
        hipLaunchKernelGGL(shift_u8_kernel, dim3(1), dim3(64), 0, s, in + body, out + body, (size_t)n - body, sh);
    CME_LAUNCH_STATUS();
}

CME_EXPORT int cme_copy_bytes(const void* in, void* out, long long nbytes, void* stream) {
    hipStream_t s = as_stream(stream);
    size_t m = (size_t)nbytes / 16;
    // measured best on MI355X (benchmarks/tune_copy.py, profiles/copy_tune_r2.log):
    // one-shot 4 KB tiles, one 16-B non-temporal vector per lane: 6.54 TB/s
    // on 1 GiB (round 1's grid-stride persistent copy: 5.96)
    if (m) hipLaunchKernelGGL(copy_flat_kernel<1>, dim3(cdiv(m, 256)), dim3(256), 0, s, (const u32x4*)in,
                              (u32x4*)out, m);
    size_t body = m * 16;
    if ((size_t)nbytes > body)
        hipLaunchKernelGGL(shift_u8_kernel, dim3(1), dim3(64), 0, s, (const uint8_t*)in + body, (uint8_t*)out + body,
                           (size_t)nbytes - body, (uint8_t)0);
    CME_LAUNCH_STATUS();
}

CME_EXPORT int cme_mul_f32(float* a, const float* b, long long n, void* stream) {
    size_t n4 = (size_t)n / 4;
    hipLaunchKernelGGL(mul_f32_kernel, dim3(stream_grid(n4 ? n4 : 1, 256)), dim3(256), 0, as_stream(stream), a, b,
                       n4, (size_t)n);
    CME_LAUNCH_STATUS();
}

// mode 0: grid-stride (unroll 1/2/4/8, nt 0/1, blocks/CU); mode 1: chunked.
CME_EXPORT int cme_copy_tune(const void* in, void* out, long long nbytes, int mode, int unroll, int nt,
                             int blocks_per_cu, void* stream) {
    hipStream_t s = as_stream(stream);
    size_t m = (size_t)nbytes / 16;
    const u32x4* a = (const u32x4*)in;
    u32x4* b = (u32x4*)out;
    unsigned grid = (unsigned)(256 * blocks_per_cu);
    if (mode == 2) {  // one-shot tiles of 256 x unroll vectors
        switch (unroll) {
            case 1: hipLaunchKernelGGL(copy_flat_kernel<1>, dim3(cdiv(m, 256)), dim3(256), 0, s, a, b, m); break;
            case 2: hipLaunchKernelGGL(copy_flat_kernel<2>, dim3(cdiv(m, 512)), dim3(256), 0, s, a, b, m); break;
            case 4: hipLaunchKernelGGL(copy_flat_kernel<4>, dim3(cdiv(m, 1024)), dim3(256), 0, s, a, b, m); break;
            default: hipLaunchKernelGGL(copy_flat_kernel<8>, dim3(cdiv(m, 2048)), dim3(256), 0, s, a, b, m); break;
        }
        CME_LAUNCH_STATUS();
    }
    if (mode == 1) {
        size_t per = (m + grid - 1) / grid;
        hipLaunchKernelGGL(copy_chunk_kernel<4>, dim3(grid), dim3(256), 0, s, a, b, m, per);
        CME_LAUNCH_STATUS();
    }
#define CT(U, N) hipLaunchKernelGGL((copy_tune_kernel<U, N>), dim3(grid), dim3(256), 0, s, a, b, m)
    if (nt) {
        switch (unroll) { case 1: CT(1, true); break; case 2: CT(2, true); break; case 4: CT(4, true); break;
                          default: CT(8, true); }
    } else {
        switch (unroll) { case 1: CT(1, false); break; case 2: CT(2, false); break; case 4: CT(4, false); break;
                          default: CT(8, false); }
    }
#undef CT
    CME_LAUNCH_STATUS();
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(shift_cipher_u128, 256, shift_u128_kernel<4>);
CME_REGISTER_KERNEL(copy_chunk, 256, copy_chunk_kernel<4>);
