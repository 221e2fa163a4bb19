// Sparse matrix-vector multiply y = A x in the Bell & Garland formats
// (refs/Bell SC 2009.pdf; slides/Lecture22.pdf; refs/Baskaran IBM 2009.pdf),
// re-derived for wave64:
//
//  csr_scalar : one lane per row (CSR-scalar)
//  csr_vector : G = 2..64 lanes per row, strided nnz, DPP/shuffle reduce
//               (Baskaran's half-warp-per-row, generalised; G picked from the
//               mean row length by the host)
//  ell        : column-major padded ELLPACK (col < 0 = padding), lane per row,
//               fully coalesced
//  dia        : diagonal format, offsets + column-major diagonals, no column
//               indices at all (structured Laplacians)
//  coo        : flat segmented reduction: each wave takes 64*4 consecutive
//               nonzeros, DPP segmented scan by row, one atomic add per
//               (row segment x wave) -- load-balanced regardless of row lengths
//  hyb        : ELL for the first K entries of each row + COO for the rest
//  csr_aligned: Baskaran's alignment fix (refs/Baskaran IBM 2009.pdf
//               pp.4-8: rows zero-padded so each starts on a 16-B boundary
//               and spans whole 4-nnz vectors): G lanes per row, each lane
//               takes 4 consecutive nonzeros with one 16-B value load and one
//               16-B index load
#include "cme213/common.h"
#include "cme213/tuning.h"
#include "cme213/wave.h"

using namespace cme;

namespace {

__global__ __launch_bounds__(256) void csr_scalar_kernel(int nrows, const int* __restrict__ rp,
                                                         const int* __restrict__ col, const float* __restrict__ val,
                                                         const float* __restrict__ x, float* __restrict__ y,
                                                         float beta) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows) return;
    float s = 0.f;
    const int e = rp[r + 1];
    int j = rp[r];
    for (; j + 4 <= e; j += 4) {  // 4 index/value loads in flight, then 4 gathers
        int c[4];
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            c[q] = col[j + q];
            v[q] = val[j + q];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) s += v[q] * x[c[q]];
    }
    for (; j < e; ++j) s += val[j] * x[col[j]];
    y[r] = beta == 0.f ? s : beta * y[r] + s;
}

template <int G>
__global__ __launch_bounds__(256) void csr_vector_kernel(int nrows, const int* __restrict__ rp,
                                                         const int* __restrict__ col, const float* __restrict__ val,
                                                         const float* __restrict__ x, float* __restrict__ y,
                                                         float beta) {
    const int r = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / G);
    const int sub = threadIdx.x % G;
    float s = 0.f;
    if (r < nrows) {
        const int b = rp[r], e = rp[r + 1];
        for (int j = b + sub; j < e; j += G) s += val[j] * x[col[j]];
    }
#pragma unroll
    for (int off = G / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (r < nrows && sub == 0) y[r] = beta == 0.f ? s : beta * y[r] + s;
}

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// NT: the column / value stream is read with non-temporal loads, so it does
// not evict the gathered vector x from L2 (a 1M-column fp32 x is 4 MB, one
// XCD's L2): the random gathers then hit L2 instead of the Infinity Cache
template <int G, bool NT>
__global__ __launch_bounds__(256) void csr_vec4_kernel(int nrows, const int* __restrict__ rp,
                                                       const int* __restrict__ col, const float* __restrict__ val,
                                                       const float* __restrict__ x, float* __restrict__ y,
                                                       float beta) {
    const int r = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / G);
    const int sub = threadIdx.x % G;
    float s = 0.f;
    if (r < nrows) {
        const int b = rp[r], e = rp[r + 1];  // multiples of 4 (aligned CSR)
        for (int j = b + 4 * sub; j < e; j += 4 * G) {
            i32x4 c;
            f32x4 v;
            if constexpr (NT) {
                c = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(col + j));
                v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(val + j));
            } else {
                c = *reinterpret_cast<const i32x4*>(col + j);
                v = *reinterpret_cast<const f32x4*>(val + j);
            }
            s += v.x * x[c.x] + v.y * x[c.y] + v.z * x[c.z] + v.w * x[c.w];
        }
    }
#pragma unroll
    for (int off = G / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (r < nrows && sub == 0) y[r] = beta == 0.f ? s : beta * y[r] + s;
}

// CSR-stream (short rows; the row-blocked scheme of CSR-adaptive): a
// workgroup owns R consecutive rows. Its whole nonzero range [rp[r0],
// rp[r0+R]) -- contiguous in col / val -- is streamed with coalesced loads,
// every product val * x[col] lands in LDS, then T = 256 / R lanes per row sum
// the row's products out of LDS and one coalesced store writes the R results.
// CSR-vector gives each short row a whole group of lanes: on the 1M 5-point
// Laplacian (5 nnz per row) 59 of its 64 lanes idle and every row issues its
// own partial 4-B loads (389 GFLOP/s warm; refs/Bell SC 2009.pdf §3-4 names
// this weakness of CSR-vector, refs/Baskaran IBM 2009.pdf pp.4-8 the
// alignment cure). Here every lane of every load instruction carries a
// useful nonzero. A block whose rows hold more than kStreamCap nonzeros
// (skewed rows) falls back to one wave per row reading global memory, so any
// CSR matrix is correct; the host picks R from the mean row length so that
// R * mean sits well under the cap.
constexpr int kStreamCap = 4096;  // products per block in LDS (16 KB)

// R rows per 256-lane workgroup: T = 256 / R lanes per row (R <= 256) or
// R / 256 rows per lane (R = 512) in the reduction. The nonzero range is read
// as 16-B (4-entry) pieces of col and val -- the aligned body of the range,
// up to three pieces per lane in flight before their gathers -- plus a head
// and a tail of at most 3 entries each read singly.
template <int R>
__global__ __launch_bounds__(256) void csr_stream_kernel(int nrows, const int* __restrict__ rp,
                                                         const int* __restrict__ col, const float* __restrict__ val,
                                                         const float* __restrict__ x, float* __restrict__ y,
                                                         float beta) {
    static_assert(R == 64 || R == 128 || R == 256 || R == 512 || R == 1024,
                  "csr_stream: 64 / 128 / 256 / 512 / 1024 rows per block");
    constexpr int T = R <= 256 ? 256 / R : 1;    // lanes per row
    constexpr int RPT = R <= 256 ? 1 : R / 256;  // rows per lane
    __shared__ float prod[kStreamCap];
    __shared__ int srp[R + 1];
    const int tid = threadIdx.x;
    const int r0 = blockIdx.x * R;
    const int nr = min(R, nrows - r0);
    // the range ends first (uniform: scalar loads), so the col / val loads
    // issue beside the row-pointer loads instead of one round trip after them
    const int base = __builtin_amdgcn_readfirstlane(rp[r0]);
    const int end = __builtin_amdgcn_readfirstlane(rp[r0 + nr]);
    const int nnz = end - base;
    for (int i = tid; i <= nr; i += 256) srp[i] = rp[r0 + i];
    if (nnz <= kStreamCap) {
        const int a0 = min((base + 3) & ~3, end);  // first 16-B boundary of the range
        const int a1 = max(end & ~3, a0);          // last
        // head [base, a0) and tail [a1, end): at most 3 entries each
        if (tid < a0 - base) prod[tid] = val[base + tid] * x[col[base + tid]];
        if (tid >= 64 && tid - 64 < end - a1) {
            const int j = a1 + tid - 64;
            prod[j - base] = val[j] * x[col[j]];
        }
        const int npc = (a1 - a0) >> 2;  // 4-entry pieces of the aligned body
        typedef int i32x4v __attribute__((ext_vector_type(4)));
        typedef float f32x4v __attribute__((ext_vector_type(4)));
        for (int p0 = 0; p0 < npc; p0 += 3 * 256) {
            i32x4v c[3];
            f32x4v v[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const int pc = p0 + q * 256 + tid;
                if (pc < npc) {
                    c[q] = *reinterpret_cast<const i32x4v*>(col + a0 + 4 * pc);
                    v[q] = *reinterpret_cast<const f32x4v*>(val + a0 + 4 * pc);
                } else {
                    c[q] = i32x4v{0, 0, 0, 0};
                    v[q] = f32x4v{0.f, 0.f, 0.f, 0.f};
                }
            }
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const int pc = p0 + q * 256 + tid;
                if (pc < npc) {
                    float* d = prod + (a0 - base) + 4 * pc;
                    d[0] = v[q].x * x[c[q].x];
                    d[1] = v[q].y * x[c[q].y];
                    d[2] = v[q].z * x[c[q].z];
                    d[3] = v[q].w * x[c[q].w];
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            const int row = (RPT > 1 ? tid + k * 256 : tid / T), sub = tid % T;
            float s = 0.f;
            if (row < nr) {
                const int e = srp[row + 1] - base;
                for (int j = srp[row] - base + sub; j < e; j += T) s += prod[j];
            }
#pragma unroll
            for (int off = T / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
            if (row < nr && sub == 0) {
                float* yp = y + r0 + row;
                *yp = beta == 0.f ? s : beta * *yp + s;
            }
        }
        return;
    }
    // a block of long rows: one wave per row, 64 lanes strided over global
    __syncthreads();  // the row pointers in LDS
    const int w = tid / 64, lane = tid % 64;
    for (int row = w; row < nr; row += 4) {
        const int b = srp[row], e = srp[row + 1];
        float s = 0.f;
        for (int j = b + lane; j < e; j += 64) s += val[j] * x[col[j]];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        if (lane == 0) {
            float* yp = y + r0 + row;
            *yp = beta == 0.f ? s : beta * *yp + s;
        }
    }
}

// CSR-short (mean row length <= 8, the 5-point Laplacian of config #4): one
// lane per row and RPT rows per lane (rows r0 + t + 256 k, so every load
// instruction of a wave walks consecutive rows). A row's first kShortNB
// entries are ONE batch of guarded col / val loads -- the row length comes
// with the row pointers -- so a 5-entry row costs three dependent round trips
// (rp, then col / val, then x) where csr_scalar's 4-entry loop plus remainder
// costs five; RPT rows per lane put every round trip of the lane's rows in
// flight together (half the waves, each with twice the loads outstanding).
// Entries past kShortNB (long rows) run a loop. Summation in entry order.
constexpr int kShortNB = 8;

template <int RPT>
__global__ __launch_bounds__(256) void csr_short_kernel(int nrows, const int* __restrict__ rp,
                                                        const int* __restrict__ col, const float* __restrict__ val,
                                                        const float* __restrict__ x, float* __restrict__ y,
                                                        float beta) {
    const int r0 = blockIdx.x * (256 * RPT) + threadIdx.x;
    int b[RPT], e[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int r = r0 + 256 * k;
        b[k] = r < nrows ? rp[r] : 0;
        e[k] = r < nrows ? rp[r + 1] : 0;
    }
    int c[RPT][kShortNB];
    float v[RPT][kShortNB];
#pragma unroll
    for (int k = 0; k < RPT; ++k)
#pragma unroll
        for (int q = 0; q < kShortNB; ++q) {
            const bool in = b[k] + q < e[k];
            c[k][q] = in ? col[b[k] + q] : -1;
            v[k][q] = in ? val[b[k] + q] : 0.f;
        }
    float xv[RPT][kShortNB];
#pragma unroll
    for (int k = 0; k < RPT; ++k)
#pragma unroll
        for (int q = 0; q < kShortNB; ++q) xv[k][q] = c[k][q] >= 0 ? x[c[k][q]] : 0.f;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int r = r0 + 256 * k;
        if (r >= nrows) continue;
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < kShortNB; ++q)
            if (c[k][q] >= 0) s += v[k][q] * xv[k][q];
        for (int j = b[k] + kShortNB; j < e[k]; ++j) s += val[j] * x[col[j]];
        y[r] = beta == 0.f ? s : beta * y[r] + s;
    }
}

// CSR-wave (short rows, config #4's 5-point Laplacian): one wave per 64
// consecutive rows and no workgroup barrier. The wave's nonzero range
// [rp[r0], rp[r0 + 64]) is contiguous in col / val, so its lanes stream it
// with coalesced loads (entry s + lane + 64 q: every load instruction carries
// 64 useful consecutive entries, against csr_scalar's 64 rows x 20-B stride,
// ~10 lines per instruction, re-touched by each of a row's loads), gather x
// for each entry and leave the PRODUCT in the wave's LDS slice; then lane l
// sums its row's products out of the slice in entry order. The slice is the
// wave's own (wave_lds_sync: in-wave ordering). A wave whose range exceeds the
// slice takes the lane-per-row loop over global memory.
constexpr int kWaveCap = 1024;  // products per wave: 4 KB, 16 KB per 256-lane workgroup

__global__ __launch_bounds__(256) void csr_wave_kernel(int nrows, const int* __restrict__ rp,
                                                       const int* __restrict__ col, const float* __restrict__ val,
                                                       const float* __restrict__ x, float* __restrict__ y,
                                                       float beta) {
    __shared__ float prod[4][kWaveCap];
    const int lane = lane_id(), w = (int)(threadIdx.x / kWave);
    const int r0 = (blockIdx.x * 4 + w) * kWave;
    if (r0 >= nrows) return;  // wave-uniform; no workgroup barrier below
    const int r = r0 + lane;
    const bool valid = r < nrows;
    const int b = valid ? rp[r] : 0;
    const int e = valid ? rp[r + 1] : 0;
    const int rl = r0 + kWave < nrows ? r0 + kWave : nrows;
    const int s0 = __builtin_amdgcn_readfirstlane(b);  // lane 0 is valid: rp[r0]
    const int cnt = __builtin_amdgcn_readfirstlane(rp[rl]) - s0;
    float acc = 0.f;
    if (cnt <= kWaveCap) {
        float* pw = prod[w];
        int q = lane;
        for (; q + 3 * kWave < cnt; q += 4 * kWave) {  // 4 col / val pairs in flight, then 4 gathers
            int c[4];
            float v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                c[k] = col[s0 + q + k * kWave];
                v[k] = val[s0 + q + k * kWave];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) pw[q + k * kWave] = v[k] * x[c[k]];
        }
        for (; q < cnt; q += kWave) pw[q] = val[s0 + q] * x[col[s0 + q]];
        wave_lds_sync();
        for (int j = b - s0; j < e - s0; ++j) acc += pw[j];
    } else {
        for (int j = b; j < e; ++j) acc += val[j] * x[col[j]];
    }
    if (valid) y[r] = beta == 0.f ? acc : beta * y[r] + acc;
}

// All column / value loads of a group of 4 entries are issued before the
// dependent x gathers (the row loop is a load-latency chain otherwise);
// padding (col < 0) is masked without a branch. Summation order is k order.
__global__ __launch_bounds__(256) void ell_kernel(int nrows, int K, const int* __restrict__ col,
                                                  const float* __restrict__ val, const float* __restrict__ x,
                                                  float* __restrict__ y, float beta) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows) return;
    float s = 0.f;
    int k = 0;
    for (; k + 4 <= K; k += 4) {
        int c[4];
        float v[4], xv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            c[j] = col[(size_t)(k + j) * nrows + r];
            v[j] = val[(size_t)(k + j) * nrows + r];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) xv[j] = x[c[j] < 0 ? 0 : c[j]];
#pragma unroll
        for (int j = 0; j < 4; ++j) s += c[j] >= 0 ? v[j] * xv[j] : 0.f;
    }
    for (; k < K; ++k) {
        const int c = col[(size_t)k * nrows + r];
        const float v = val[(size_t)k * nrows + r];
        const float xv = x[c < 0 ? 0 : c];
        s += c >= 0 ? v * xv : 0.f;
    }
    y[r] = beta == 0.f ? s : beta * y[r] + s;
}

__global__ __launch_bounds__(256) void dia_kernel(int nrows, int ncols, int ndiag, const int* __restrict__ offsets,
                                                  const float* __restrict__ data, const float* __restrict__ x,
                                                  float* __restrict__ y, float beta) {
    __shared__ int s_off[64];
    for (int i = threadIdx.x; i < ndiag && i < 64; i += blockDim.x) s_off[i] = offsets[i];
    __syncthreads();
    const int r = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;  // see dia4_kernel
    if (r >= nrows) return;
    float s = 0.f;
    int d = 0;
    for (; d + 4 <= ndiag; d += 4) {  // loads of 4 diagonals in flight
        int c[4];
        float v[4], xv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            c[j] = r + (d + j < 64 ? s_off[d + j] : offsets[d + j]);
            v[j] = data[(size_t)(d + j) * nrows + r];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) xv[j] = x[c[j] < 0 ? 0 : (c[j] >= ncols ? ncols - 1 : c[j])];
#pragma unroll
        for (int j = 0; j < 4; ++j) s += (c[j] >= 0 && c[j] < ncols) ? v[j] * xv[j] : 0.f;
    }
    for (; d < ndiag; ++d) {
        const int c = r + (d < 64 ? s_off[d] : offsets[d]);
        const float v = data[(size_t)d * nrows + r];
        const float xv = x[c < 0 ? 0 : (c >= ncols ? ncols - 1 : c)];
        s += (c >= 0 && c < ncols) ? v * xv : 0.f;
    }
    y[r] = beta == 0.f ? s : beta * y[r] + s;
}

// DIA, 4 consecutive rows per lane: the diagonals are read with 16-B loads
// and y is written with one 16-B store (the one-row kernel above issues 4-B
// accesses: 66 % of the copy rate on the 16M-row 5-point Laplacian with the
// MALL defeated, benchmarks/bench_spmv.py). x is gathered per row (its lines
// are shared by the neighbouring diagonals and rows: L1/L2 hits). Needs
// nrows % 4 == 0 (16-B aligned diagonals); the launcher falls back otherwise.
__global__ __launch_bounds__(256) void dia4_kernel(int nrows, int ncols, int ndiag, const int* __restrict__ offsets,
                                                   const float* __restrict__ data, const float* __restrict__ x,
                                                   float* __restrict__ y, float beta) {
    __shared__ int s_off[64];
    for (int i = threadIdx.x; i < ndiag && i < 64; i += blockDim.x) s_off[i] = offsets[i];
    __syncthreads();
    // XCD-aware order: each XCD gets a contiguous range of row blocks, so the
    // x lines a diagonal offset re-reads (rows r +- off) hit that XCD's L2
    const int r0 = (xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x) * 4;
    if (r0 >= nrows) return;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
    for (int d = 0; d < ndiag; ++d) {
        const int off = d < 64 ? s_off[d] : offsets[d];
        const float4 v = *reinterpret_cast<const float4*>(data + (size_t)d * nrows + r0);
        const int c = r0 + off;
        float xv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int cj = c + j;
            xv[j] = (cj >= 0 && cj < ncols) ? x[cj] : 0.f;
        }
        s.x += v.x * xv[0];
        s.y += v.y * xv[1];
        s.z += v.z * xv[2];
        s.w += v.w * xv[3];
    }
    float4* yp = reinterpret_cast<float4*>(y + r0);
    if (beta != 0.f) {
        const float4 o = *yp;
        s.x += beta * o.x;
        s.y += beta * o.y;
        s.z += beta * o.z;
        s.w += beta * o.w;
    }
    *yp = s;
}

// COO: entries sorted by row. Each wave handles 256 consecutive entries as
// 4 rounds of 64; segmented (by row) inclusive scan via DPP, lanes that end a
// row segment (next lane has another row, or last lane) atomically add.
__global__ __launch_bounds__(256) void coo_kernel(long long nnz, const int* __restrict__ row,
                                                  const int* __restrict__ col, const float* __restrict__ val,
                                                  const float* __restrict__ x, float* __restrict__ y) {
    const int lane = lane_id();
    const long long wave = (blockIdx.x * (long long)blockDim.x + threadIdx.x) / kWave;
    const long long base = wave * 256;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const long long i = base + k * 64 + lane;
        const bool ok = i < nnz;
        const int r = ok ? row[i] : -1;
        float v = ok ? val[i] * x[col[i]] : 0.f;
        // head flag: first lane or row differs from previous lane
        const int rprev = dpp_move<kDppWaveShr1>(-2, r);
        uint32_t f = (lane == 0 || rprev != r) ? 1u : 0u;
#define SEG_STEP(CTRL, RM)                                 \
    {                                                      \
        float vs = dpp_move<CTRL, RM>(0.0f, v);            \
        uint32_t fs = dpp_move<CTRL, RM>(0u, f);           \
        v = f ? v : vs + v;                                \
        f = f | fs;                                        \
    }
        SEG_STEP(kDppRowShr1, 0xf)
        SEG_STEP(kDppRowShr2, 0xf)
        SEG_STEP(kDppRowShr4, 0xf)
        SEG_STEP(kDppRowShr8, 0xf)
        SEG_STEP(kDppRowBcast15, 0xa)
        SEG_STEP(kDppRowBcast31, 0xc)
#undef SEG_STEP
        const int rnext = dpp_move<kDppWaveShl1>(-3, r);
        const bool tail = (lane == kWave - 1) || (rnext != r);
        if (ok && tail) atomicAdd(&y[r], v);
    }
}

__global__ void scale_kernel(float* y, int n, float beta) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = beta == 0.f ? 0.f : beta * y[i];
}

// Distributed SpMV halo pieces (models/dist_spmv.py). Send side: the x
// entries each peer needs, packed back to back in peer order (one launch for
// all peers). Receive side: after the interior product y = A_int x_local, the
// compact boundary rows add their off-rank columns from the received halo.
__global__ void gather_kernel(const float* __restrict__ x, const int* __restrict__ idx, float* __restrict__ out,
                              int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = x[idx[i]];
}

__global__ void halo_csr_kernel(int nb, const int* __restrict__ rows, const int* __restrict__ rp,
                                const int* __restrict__ col, const float* __restrict__ val,
                                const float* __restrict__ h, float* __restrict__ y) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    float s = 0.f;
    for (int j = rp[b]; j < rp[b + 1]; ++j) s += val[j] * h[col[j]];
    y[rows[b]] += s;  // rows are distinct: no atomics
}

}  // namespace

CME_EXPORT int cme_gather_f32(int n, const float* x, const int* idx, float* out, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(gather_kernel, dim3(cdiv(n, 256)), dim3(256), 0, as_stream(stream), x, idx, out, n);
    CME_LAUNCH_STATUS();
}

CME_EXPORT int cme_spmv_halo(int nb, const int* rows, const int* rp, const int* col, const float* val, const float* h,
                             float* y, void* stream) {
    if (nb <= 0) return 0;
    hipLaunchKernelGGL(halo_csr_kernel, dim3(cdiv(nb, 256)), dim3(256), 0, as_stream(stream), nb, rows, rp, col, val,
                       h, y);
    CME_LAUNCH_STATUS();
}

// y = A x (+ beta y). group: 1 scalar, else lanes per row (2..64).
CME_EXPORT int cme_spmv_csr(int nrows, const int* rp, const int* col, const float* val, const float* x, float* y,
                            int group, float beta, void* stream) {
    hipStream_t s = as_stream(stream);
    switch (group) {
        case 1: hipLaunchKernelGGL(csr_scalar_kernel, dim3(cdiv(nrows, 256)), dim3(256), 0, s, nrows, rp, col, val, x, y, beta); break;
#define V(G) case G: hipLaunchKernelGGL(csr_vector_kernel<G>, dim3(cdiv((size_t)nrows * G, 256)), dim3(256), 0, s, nrows, rp, col, val, x, y, beta); break;
        V(2) V(4) V(8) V(16) V(32) V(64)
#undef V
        default: return (int)hipErrorInvalidValue;
    }
    CME_LAUNCH_STATUS();
}

// CSR-stream: rows_per_block 64 / 128 / 256 / 512 (the host picks it from the mean
// row length: csr_stream_kernel).
CME_EXPORT int cme_spmv_csr_stream(int nrows, const int* rp, const int* col, const float* val, const float* x,
                                   float* y, int rows_per_block, float beta, void* stream) {
    hipStream_t s = as_stream(stream);
    if (nrows <= 0) return 0;
    switch (rows_per_block) {
#define V(R) case R: hipLaunchKernelGGL(csr_stream_kernel<R>, dim3(cdiv(nrows, R)), dim3(256), 0, s, nrows, rp, col, val, x, y, beta); break;
        V(64) V(128) V(256) V(512) V(1024)
#undef V
        default: return (int)hipErrorInvalidValue;
    }
    CME_LAUNCH_STATUS();
}

// CSR-wave: one wave per 64 rows (csr_wave_kernel).
CME_EXPORT int cme_spmv_csr_wave(int nrows, const int* rp, const int* col, const float* val, const float* x, float* y,
                                 float beta, void* stream) {
    hipStream_t s = as_stream(stream);
    if (nrows <= 0) return 0;
    hipLaunchKernelGGL(csr_wave_kernel, dim3(cdiv(nrows, 256)), dim3(256), 0, s, nrows, rp, col, val, x, y, beta);
    CME_LAUNCH_STATUS();
}

// CSR-short: rows_per_lane 1 / 2 / 4 (csr_short_kernel).
CME_EXPORT int cme_spmv_csr_short(int nrows, const int* rp, const int* col, const float* val, const float* x,
                                  float* y, int rows_per_lane, float beta, void* stream) {
    hipStream_t s = as_stream(stream);
    if (nrows <= 0) return 0;
    switch (rows_per_lane) {
#define V(R) case R: hipLaunchKernelGGL(csr_short_kernel<R>, dim3(cdiv(nrows, 256 * R)), dim3(256), 0, s, nrows, rp, col, val, x, y, beta); break;
        V(1) V(2) V(4)
#undef V
        default: return (int)hipErrorInvalidValue;
    }
    CME_LAUNCH_STATUS();
}

// Aligned CSR (every rp[i] % 4 == 0, col/val 16-B aligned): group 1..64;
// nnz = col/val length (selects the stream loads).
CME_EXPORT int cme_spmv_csr_aligned(int nrows, long long nnz, const int* rp, const int* col, const float* val,
                                    const float* x, float* y, int group, float beta, void* stream) {
    hipStream_t s = as_stream(stream);
    if (((uintptr_t)col % 16) || ((uintptr_t)val % 16)) return (int)hipErrorInvalidValue;
    // CME_SPMV_NT: 0 plain stream loads, 1 non-temporal, 2 (default) non-temporal
    // only when the col/val stream cannot stay in the 256 MB Infinity Cache
    // between calls. Measured (profiles/spmv_nt_r4.md): non-temporal wins cold
    // (5pt-16M 211 vs 219 us, random-1M 104 vs 111) but loses whenever the
    // stream is cache-resident across calls (27pt-1M warm 50 vs 40 us, skew-1M
    // 1.50 vs 1.26 ms, every column-blocked case).
    const int mode = cme::tune_get(cme::kTuneSpmvNT);
    const bool nt = mode == 2 ? nnz * 8 > (256ll << 20) : mode != 0;
    switch (group) {
#define V(G)                                                                                                      \
    case G:                                                                                                       \
        if (nt)                                                                                                   \
            hipLaunchKernelGGL((csr_vec4_kernel<G, true>), dim3(cdiv((size_t)nrows * G, 256)), dim3(256), 0, s,    \
                               nrows, rp, col, val, x, y, beta);                                                  \
        else                                                                                                      \
            hipLaunchKernelGGL((csr_vec4_kernel<G, false>), dim3(cdiv((size_t)nrows * G, 256)), dim3(256), 0, s,   \
                               nrows, rp, col, val, x, y, beta);                                                  \
        break;
        V(1) V(2) V(4) V(8) V(16) V(32) V(64)
#undef V
        default: return (int)hipErrorInvalidValue;
    }
    CME_LAUNCH_STATUS();
}

CME_EXPORT int cme_spmv_ell(int nrows, int K, const int* col, const float* val, const float* x, float* y, float beta,
                            void* stream) {
    hipLaunchKernelGGL(ell_kernel, dim3(cdiv(nrows, 256)), dim3(256), 0, as_stream(stream), nrows, K, col, val, x, y,
                       beta);
    CME_LAUNCH_STATUS();
}

CME_EXPORT int cme_spmv_dia(int nrows, int ncols, int ndiag, const int* offsets, const float* data, const float* x,
                            float* y, float beta, void* stream) {
    // 4 rows per lane only when that still leaves >= 1M lanes (16 waves per
    // SIMD): with 1M rows its 250K lanes lose to the one-row kernel (27-point
    // Laplacian 41 vs 30 us, 5-point 11.0 vs 10.2 us; 16M-row 5-point 99 vs
    // 117 us -- profiles/spmv_r2.md). CME_SPMV_DIA1 forces the one-row kernel.
    const bool one_row = cme::tune_get(cme::kTuneSpmvDia1) != 0;
    if (nrows % 4 == 0 && nrows >= (4 << 20) && !one_row) {
        hipLaunchKernelGGL(dia4_kernel, dim3(cdiv(nrows / 4, 256)), dim3(256), 0, as_stream(stream), nrows, ncols,
                           ndiag, offsets, data, x, y, beta);
        CME_LAUNCH_STATUS();
    }
    hipLaunchKernelGGL(dia_kernel, dim3(cdiv(nrows, 256)), dim3(256), 0, as_stream(stream), nrows, ncols, ndiag,
                       offsets, data, x, y, beta);
    CME_LAUNCH_STATUS();
}

// y = beta*y + A x for COO (beta applied first, then atomics accumulate).
CME_EXPORT int cme_spmv_coo(int nrows, long long nnz, const int* row, const int* col, const float* val, const float* x,
                            float* y, float beta, int accumulate, void* stream) {
    hipStream_t s = as_stream(stream);
    if (!accumulate) hipLaunchKernelGGL(scale_kernel, dim3(cdiv(nrows, 256)), dim3(256), 0, s, y, nrows, beta);
    if (nnz > 0) {
        const long long waves = (nnz + 255) / 256;
        hipLaunchKernelGGL(coo_kernel, dim3(cdiv(waves * 64, 256)), dim3(256), 0, s, nnz, row, col, val, x, y);
    }
    CME_LAUNCH_STATUS();
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(spmv_csr_scalar, 256, csr_scalar_kernel);
CME_REGISTER_KERNEL(spmv_csr_short2, 256, csr_short_kernel<2>);
CME_REGISTER_KERNEL(spmv_csr_vector8, 256, csr_vector_kernel<8>);
CME_REGISTER_KERNEL(spmv_csr_aligned4, 256, csr_vec4_kernel<4, true>);
CME_REGISTER_KERNEL(spmv_ell, 256, ell_kernel);
CME_REGISTER_KERNEL(spmv_dia, 256, dia_kernel);
CME_REGISTER_KERNEL(spmv_dia4, 256, dia4_kernel);
CME_REGISTER_KERNEL(spmv_coo, 256, coo_kernel);
CME_REGISTER_KERNEL(spmv_csr_stream256, 256, csr_stream_kernel<256>);
