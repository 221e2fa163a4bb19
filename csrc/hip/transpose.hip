// Matrix transpose ladder (slides/Lecture06-07; my-refs/MatrixTranspose.pdf;
// my-refs/cuda_many_cores.pdf pp.14-17), re-derived for wave64 / gfx950 LDS.
//
// out[c][r] = in[r][c], in is rows x cols (row-major, fp32).
//
//  0 copy        : same-shape copy with the transpose's grid (the paper's
//                  "copy" upper bound)
//  1 naive       : 1 thread/element, coalesced reads, stride-`rows` writes
//  2 lds         : 64x64 LDS tile, no padding (column reads of a 64-float row
//                  pitch: every lane of a 32-lane group hits one bank)
//  3 lds_pad     : +1 float padding (pitch 65: conflict-free)
//  4 lds_swizzle : no padding, XOR swizzle col ^ (row & 63): conflict-free
//  5 diagonal    : lds_pad with the paper's diagonal block reordering
//                  (partition camping); on MI355X the analogous lever is
//  6 xcd         : lds_pad with the bijective XCD-aware block remap
//  7 vec         : 64x64 tile, 16-B global loads AND stores, pad-65 LDS
//                  (2-way conflicts on the scalar LDS side, 4x fewer global
//                  instructions) -- the production variant
#include "cme213/common.h"

namespace {

constexpr int kT = 64;  // tile edge

__global__ __launch_bounds__(256) void copy_kernel(const float* __restrict__ in, float* __restrict__ out, int rows,
                                                   int cols) {
    const int x = blockIdx.x * kT + threadIdx.x % 64;
    const int y0 = blockIdx.y * kT + threadIdx.x / 64;
    if (x >= cols) return;
    for (int y = y0; y < blockIdx.y * kT + kT && y < rows; y += 4) out[(size_t)y * cols + x] = in[(size_t)y * cols + x];
}

__global__ __launch_bounds__(256) void naive_kernel(const float* __restrict__ in, float* __restrict__ out, int rows,
                                                    int cols) {
    const int x = blockIdx.x * kT + threadIdx.x % 64;
    const int y0 = blockIdx.y * kT + threadIdx.x / 64;
    if (x >= cols) return;
    for (int y = y0; y < blockIdx.y * kT + kT && y < rows; y += 4) out[(size_t)x * rows + y] = in[(size_t)y * cols + x];
}

// MODE: 0 no pad, 1 pad, 2 swizzle. REMAP: 0 none, 1 diagonal, 2 xcd.
template <int MODE, int REMAP>
__global__ __launch_bounds__(256) void tile_kernel(const float* __restrict__ in, float* __restrict__ out, int rows,
                                                   int cols) {
    constexpr int P = MODE == 1 ? kT + 1 : kT;
    __shared__ float tile[kT * P];
    int bx = blockIdx.x, by = blockIdx.y;
    if constexpr (REMAP == 1) {  // diagonal reordering (square grids)
        if (gridDim.x == gridDim.y) {
            by = blockIdx.x;
            bx = (blockIdx.x + blockIdx.y) % gridDim.x;
        }
    } else if constexpr (REMAP == 2) {
        const unsigned lin = blockIdx.y * gridDim.x + blockIdx.x;
        const unsigned r = xcd_remap(lin, gridDim.x * gridDim.y);
        bx = r % gridDim.x;
        by = r / gridDim.x;
    }
    const int tx = threadIdx.x % 64, ty = threadIdx.x / 64;
    const int x0 = bx * kT, y0 = by * kT;
    auto idx = [](int r, int c) { return MODE == 2 ? r * P + (c ^ (r & 63)) : r * P + c; };
#pragma unroll 4
    for (int i = 0; i < kT; i += 4) {
        const int y = y0 + ty + i, x = x0 + tx;
        if (y < rows && x < cols) tile[idx(ty + i, tx)] = in[(size_t)y * cols + x];
    }
    __syncthreads();
#pragma unroll 4
    for (int i = 0; i < kT; i += 4) {
        const int oy = x0 + ty + i, ox = y0 + tx;  // output row = input column
        if (oy < cols && ox < rows) out[(size_t)oy * rows + ox] = tile[idx(tx, ty + i)];
    }
}

// 16-B global accesses on both sides. Requires rows % 4 == 0 && cols % 4 == 0.
__global__ __launch_bounds__(256) void vec_kernel(const float* __restrict__ in, float* __restrict__ out, int rows,
                                                  int cols) {
    constexpr int P = kT + 1;
    __shared__ float tile[kT * P];
    const int t = threadIdx.x;
    const unsigned lin = blockIdx.y * gridDim.x + blockIdx.x;
    const unsigned r = xcd_remap(lin, gridDim.x * gridDim.y);
    const int bx = r % gridDim.x, by = r / gridDim.x;
    const int x0 = bx * kT, y0 = by * kT;
    const int c4 = (t % 16) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int rr = t / 16 + 16 * i;
        const int y = y0 + rr, x = x0 + c4;
        if (y < rows && x < cols) {
            const float4 v = *reinterpret_cast<const float4*>(in + (size_t)y * cols + x);
            tile[(c4 + 0) * P + rr] = v.x;  // store transposed: tile[col][row]
            tile[(c4 + 1) * P + rr] = v.y;
            tile[(c4 + 2) * P + rr] = v.z;
            tile[(c4 + 3) * P + rr] = v.w;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int oc = t / 16 + 16 * i;  // output row within tile (= input column)
        const int oy = x0 + oc, ox = y0 + c4;
        if (oy < cols && ox < rows) {
            const float* s = &tile[oc * P + c4];
            *reinterpret_cast<float4*>(out + (size_t)oy * rows + ox) = make_float4(s[0], s[1], s[2], s[3]);
        }
    }
}

}  // namespace

CME_EXPORT int cme_transpose_f32(const float* in, float* out, int rows, int cols, int variant, void* stream) {
    hipStream_t s = as_stream(stream);
    dim3 grid(cdiv(cols, kT), cdiv(rows, kT));
    switch (variant) {
        case 0: hipLaunchKernelGGL(copy_kernel, grid, dim3(256), 0, s, in, out, rows, cols); break;
        case 1: hipLaunchKernelGGL(naive_kernel, grid, dim3(256), 0, s, in, out, rows, cols); break;
        case 2: hipLaunchKernelGGL((tile_kernel<0, 0>), grid, dim3(256), 0, s, in, out, rows, cols); break;
        case 3: hipLaunchKernelGGL((tile_kernel<1, 0>), grid, dim3(256), 0, s, in, out, rows, cols); break;
        case 4: hipLaunchKernelGGL((tile_kernel<2, 0>), grid, dim3(256), 0, s, in, out, rows, cols); break;
        case 5: hipLaunchKernelGGL((tile_kernel<1, 1>), grid, dim3(256), 0, s, in, out, rows, cols); break;
        case 6: hipLaunchKernelGGL((tile_kernel<1, 2>), grid, dim3(256), 0, s, in, out, rows, cols); break;
        case 7:
            if ((rows % 4) || (cols % 4) || ((uintptr_t)in % 16) || ((uintptr_t)out % 16))
                hipLaunchKernelGGL((tile_kernel<1, 2>), grid, dim3(256), 0, s, in, out, rows, cols);
            else
                hipLaunchKernelGGL(vec_kernel, grid, dim3(256), 0, s, in, out, rows, cols);
            break;
        default: return (int)hipErrorInvalidValue;
    }
    CME_LAUNCH_STATUS();
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(transpose_naive, 256, naive_kernel);
CME_REGISTER_KERNEL(transpose_lds_pad, 256, tile_kernel<1, 0>);
CME_REGISTER_KERNEL(transpose_vec, 256, vec_kernel);
