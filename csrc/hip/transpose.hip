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
//  7 vec         : 16-B global loads AND stores, pad-(TR+1) LDS, tile shape
//                  and block order from a measured sweep (vec_tile_kernel)
//                  -- the production variant
//  8 vec_xcd     : 64x64 vector tile in XCD-aware block order
//  9 naive_1d    : 1-D grid, one lane per element (the lecture's first rung)
// 10 coarse      : LDS tile written to its TRANSPOSED tile position but with
//                  element order unchanged (the paper's "coarse-grained"
//                  diagnostic: isolates the cost of the tile-level scatter)
// 11 fine        : elements transposed WITHIN each tile, tile kept in place
//                  (the paper's "fine-grained" diagnostic)
// The paper's second timing mode (loop INSIDE the kernel, no launch cost per
// repetition) is cme_transpose_reps_f32.
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

__global__ __launch_bounds__(256) void naive_1d_kernel(const float* __restrict__ in, float* __restrict__ out, int rows,
                                                       int cols) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long long)rows * cols) return;
    const int r = (int)(i / cols), c = (int)(i % cols);
    out[(size_t)c * rows + r] = in[i];
}

// MODE 0 coarse, 1 fine (square matrices; pad-65 LDS tile)
template <int MODE>
__global__ __launch_bounds__(256) void grain_kernel(const float* __restrict__ in, float* __restrict__ out, int rows,
                                                    int cols) {
    constexpr int P = kT + 1;
    __shared__ float tile[kT * P];
    const int tx = threadIdx.x % 64, ty = threadIdx.x / 64;
    const int x0 = blockIdx.x * kT, y0 = blockIdx.y * kT;
#pragma unroll 4
    for (int i = 0; i < kT; i += 4) {
        const int y = y0 + ty + i, x = x0 + tx;
        if (y < rows && x < cols) tile[(ty + i) * P + tx] = in[(size_t)y * cols + x];
    }
    __syncthreads();
#pragma unroll 4
    for (int i = 0; i < kT; i += 4) {
        if constexpr (MODE == 0) {  // tile moves, elements keep their order
            const int oy = x0 + ty + i, ox = y0 + tx;
            if (oy < cols && ox < rows) out[(size_t)oy * rows + ox] = tile[(ty + i) * P + tx];
        } else {  // tile stays, elements transposed
            const int oy = y0 + ty + i, ox = x0 + tx;
            if (oy < rows && ox < cols) out[(size_t)oy * cols + ox] = tile[tx * P + ty + i];
        }
    }
}

// lds_pad transpose repeated `reps` times inside ONE launch (the paper's
// in-kernel loop timing mode, my-refs/MatrixTranspose.pdf pp.4-5).
__global__ __launch_bounds__(256) void tile_reps_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                        int rows, int cols, int reps) {
    constexpr int P = kT + 1;
    __shared__ float tile[kT * P];
    const int tx = threadIdx.x % 64, ty = threadIdx.x / 64;
    const int x0 = blockIdx.x * kT, y0 = blockIdx.y * kT;
    for (int r = 0; r < reps; ++r) {
#pragma unroll 4
        for (int i = 0; i < kT; i += 4) {
            const int y = y0 + ty + i, x = x0 + tx;
            if (y < rows && x < cols) tile[(ty + i) * P + tx] = in[(size_t)y * cols + x];
        }
        __syncthreads();
#pragma unroll 4
        for (int i = 0; i < kT; i += 4) {
            const int oy = x0 + ty + i, ox = y0 + tx;
            if (oy < cols && ox < rows) out[(size_t)oy * rows + ox] = tile[tx * P + ty + i];
        }
        __syncthreads();
    }
}

// Generalised vector tile: TR input rows x TC input columns per 256-thread
// block (16-B global loads and stores; the transposed tile lives in LDS with
// a +1 pitch). Taller tiles give longer contiguous output-row segments
// (TR floats), wider tiles longer input-row segments (TC floats) -- at 8192^2
// (beyond the 256 MB MALL) 256-B segments at a 32 KB stride leave HBM
// bandwidth on the table. REMAP: 0 none, 1 XCD-aware, 2 diagonal.
// NT: non-temporal (streaming) output stores. K: tiles per block, stacked
// along the input rows -- all K tiles' loads are issued before any LDS
// write, so a block keeps K x 16 KB in flight.
// Picks v[(k + rot) & 3] with a lane-dependent rot (selects, no indexing).
__device__ __forceinline__ float pick4(const float4& v, int e) {
    const float lo = (e & 1) ? v.y : v.x, hi = (e & 1) ? v.w : v.z;
    return (e & 2) ? hi : lo;
}

// LDS bank rule (cdna_hip_programming.md §2 LDS): ds_write_b32 / ds_read_b32
// address 32 banks ((a/4) % 32) per 32-lane half-wave. With the +1 pitch
// (P = TR + 1 odd) the element at column c, row r sits in bank (c + r) % 32,
// and the lanes of one half-wave that hold columns 4j..4j+3 (j = 0..15) hit
// bank 4j + k for element k: lanes j and j + 8 collide (2-way, measured
// 4.19M SQ_LDS_BANK_CONFLICT cycles per 8192^2 dispatch). ROT rotates the
// element order by 2 for j >= 8, so a half-wave's 32 accesses cover 32
// distinct banks in every write and read step.
template <int TR, int TC, int REMAP, bool NT = false, int K = 1, bool ROT = false>
__global__ __launch_bounds__(256) void vec_tile_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                       int rows, int cols) {
    constexpr int P = TR + 1;
    __shared__ float tile[K][TC * P];
    const int t = threadIdx.x;
    int bx = blockIdx.x, by = blockIdx.y;
    if constexpr (REMAP == 1) {
        const unsigned lin = blockIdx.y * gridDim.x + blockIdx.x;
        const unsigned r = xcd_remap(lin, gridDim.x * gridDim.y);
        bx = r % gridDim.x;
        by = r / gridDim.x;
    } else if constexpr (REMAP == 2) {
        if (gridDim.x == gridDim.y) {
            by = blockIdx.x;
            bx = (blockIdx.x + blockIdx.y) % gridDim.x;
        }
    }
    const int x0 = bx * TC;
    constexpr int LPR = TC / 4;              // lanes per input row
    constexpr int RPP = 256 / LPR;           // rows per pass
    const int c4 = (t % LPR) * 4;
    float4 v[K][TR / RPP];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int y0 = (by * K + k) * TR;
#pragma unroll
        for (int i = 0; i < TR / RPP; ++i) {
            const int y = y0 + t / LPR + RPP * i, x = x0 + c4;
            v[k][i] = (y < rows && x < cols) ? *reinterpret_cast<const float4*>(in + (size_t)y * cols + x)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    const int rot_w = ROT ? ((t % LPR) >> 3) * 2 : 0;  // lanes holding columns 32..63 of the tile
#pragma unroll
    for (int k = 0; k < K; ++k) {
#pragma unroll
        for (int i = 0; i < TR / RPP; ++i) {
            const int rr = t / LPR + RPP * i;
            if constexpr (ROT) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int ee = (e + rot_w) & 3;
                    tile[k][(c4 + ee) * P + rr] = pick4(v[k][i], ee);
                }
            } else {
                tile[k][(c4 + 0) * P + rr] = v[k][i].x;
                tile[k][(c4 + 1) * P + rr] = v[k][i].y;
                tile[k][(c4 + 2) * P + rr] = v[k][i].z;
                tile[k][(c4 + 3) * P + rr] = v[k][i].w;
            }
        }
    }
    __syncthreads();
    constexpr int LPO = TR / 4;              // lanes per output row
    constexpr int OPP = 256 / LPO;           // output rows per pass
    const int r4 = (t % LPO) * 4;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int y0 = (by * K + k) * TR;
#pragma unroll
        for (int i = 0; i < TC / OPP; ++i) {
            const int oc = t / LPO + OPP * i;
            const int oy = x0 + oc, ox = y0 + r4;
            if (oy < cols && ox < rows) {
                const float* s = &tile[k][oc * P + r4];
                typedef float v4f __attribute__((ext_vector_type(4)));
                v4f o;
                if constexpr (ROT) {
                    const int rot_r = ((t % LPO) >> 3) * 2;
                    float g[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) g[e] = s[(e + rot_r) & 3];  // rotated read order
                    // g[e] holds row r4 + ((e + rot_r) & 3): undo the rotation
                    const float4 gg = make_float4(g[0], g[1], g[2], g[3]);
                    o = v4f{pick4(gg, (0 - rot_r) & 3), pick4(gg, (1 - rot_r) & 3), pick4(gg, (2 - rot_r) & 3),
                            pick4(gg, (3 - rot_r) & 3)};
                } else {
                    o = v4f{s[0], s[1], s[2], s[3]};
                }
                v4f* dst = reinterpret_cast<v4f*>(out + (size_t)oy * rows + ox);
                if constexpr (NT)
                    __builtin_nontemporal_store(o, dst);
                else
                    *dst = o;
            }
        }
    }
}

template <int TR, int TC, int REMAP, bool NT = false, int K = 1, bool ROT = false>
int launch_vec_tile(const float* in, float* out, int rows, int cols, hipStream_t s) {
    if constexpr ((size_t)K * TC * (TR + 1) * 4 > 160 * 1024) {
        return (int)hipErrorInvalidValue;  // does not fit the 160 KB LDS of a CU
    } else {
        dim3 grid(cdiv(cols, TC), cdiv(rows, TR * K));
        hipLaunchKernelGGL((vec_tile_kernel<TR, TC, REMAP, NT, K, ROT>), grid, dim3(256), 0, s, in, out, rows, cols);
        CME_LAUNCH_STATUS();
    }
}

}  // namespace

// Tuning sweep entry (benchmarks/tune_transpose.py): tile rows tr in
// {64, 128, 256}, tile cols tc in {64, 128}; remap bits 0-1: 0 none, 1
// XCD-aware, 2 diagonal; bit 2: non-temporal stores; bit 3: 2 tiles per block.
CME_EXPORT int cme_transpose_tune(const float* in, float* out, int rows, int cols, int tr, int tc, int remap,
                                  void* stream) {
    hipStream_t s = as_stream(stream);
    if ((rows % 4) || (cols % 4)) return (int)hipErrorInvalidValue;
#define CME_VT(TR, TC)                                                                      \
    if (tr == TR && tc == TC) {                                                             \
        switch (remap) {                                                                    \
            case 0: return launch_vec_tile<TR, TC, 0>(in, out, rows, cols, s);              \
            case 1: return launch_vec_tile<TR, TC, 1>(in, out, rows, cols, s);              \
            case 2: return launch_vec_tile<TR, TC, 2>(in, out, rows, cols, s);              \
            case 4: return launch_vec_tile<TR, TC, 0, true>(in, out, rows, cols, s);        \
            case 6: return launch_vec_tile<TR, TC, 2, true>(in, out, rows, cols, s);        \
            case 8: return launch_vec_tile<TR, TC, 0, false, 2>(in, out, rows, cols, s);    \
            case 9: return launch_vec_tile<TR, TC, 1, false, 2>(in, out, rows, cols, s);    \
            case 12: return launch_vec_tile<TR, TC, 0, true, 2>(in, out, rows, cols, s);    \
            case 13: return launch_vec_tile<TR, TC, 1, true, 2>(in, out, rows, cols, s);    \
            case 22: return launch_vec_tile<TR, TC, 2, true, 1, true>(in, out, rows, cols, s); \
            case 20: return launch_vec_tile<TR, TC, 0, true, 1, true>(in, out, rows, cols, s); \
            default: return (int)hipErrorInvalidValue;                                      \
        }                                                                                   \
    }
    CME_VT(64, 64)
    CME_VT(128, 64)
    CME_VT(256, 64)
    CME_VT(64, 128)
    CME_VT(128, 128)
    CME_VT(256, 128)
#undef CME_VT
    return (int)hipErrorInvalidValue;
}

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
        case 8:
            if ((rows % 4) || (cols % 4) || ((uintptr_t)in % 16) || ((uintptr_t)out % 16)) {
                hipLaunchKernelGGL((tile_kernel<1, 2>), grid, dim3(256), 0, s, in, out, rows, cols);
            } else if (variant == 8) {
                return launch_vec_tile<64, 64, 1>(in, out, rows, cols, s);
            } else {
                // benchmarks/tune_transpose.py (profiles/transpose_tune_r2.log):
                // square -> 64x64 tiles in diagonal order with non-temporal
                // output stores (6.88 TB/s at 8192^2, 6.54 at 4096^2, 5.16 at
                // 16384^2; round 1's plain stores: 5.35 / 6.39 / 4.92);
                // otherwise 64x128 tiles, non-temporal stores
                // The LDS element order is rotated per lane group (ROT): 0 bank
                // conflicts (profiles/transpose_pmc_r2.md) at the same speed.
                if (rows == cols) return launch_vec_tile<64, 64, 2, true, 1, true>(in, out, rows, cols, s);
                return launch_vec_tile<64, 128, 0, true, 1, true>(in, out, rows, cols, s);
            }
            break;
        case 9:
            hipLaunchKernelGGL(naive_1d_kernel, dim3(cdiv((size_t)rows * cols, 256)), dim3(256), 0, s, in, out, rows,
                               cols);
            break;
        case 10:
        case 11:
            if (rows != cols) return (int)hipErrorInvalidValue;  // diagnostics: square only
            if (variant == 10)
                hipLaunchKernelGGL((grain_kernel<0>), grid, dim3(256), 0, s, in, out, rows, cols);
            else
                hipLaunchKernelGGL((grain_kernel<1>), grid, dim3(256), 0, s, in, out, rows, cols);
            break;
        default: return (int)hipErrorInvalidValue;
    }
    CME_LAUNCH_STATUS();
}

CME_EXPORT int cme_transpose_reps_f32(const float* in, float* out, int rows, int cols, int reps, void* stream) {
    dim3 grid(cdiv(cols, kT), cdiv(rows, kT));
    hipLaunchKernelGGL(tile_reps_kernel, grid, dim3(256), 0, as_stream(stream), in, out, rows, cols, reps);
    CME_LAUNCH_STATUS();
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(transpose_naive, 256, naive_kernel);
CME_REGISTER_KERNEL(transpose_lds_pad, 256, tile_kernel<1, 0>);
CME_REGISTER_KERNEL(transpose_vec, 256, vec_tile_kernel<64, 64, 2>);
