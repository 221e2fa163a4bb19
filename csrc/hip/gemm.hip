// SGEMM ladder (slides/Lecture09 slides 5-18): C = alpha*A*B + beta*C,
// row-major A[M][K], B[K][N], C[M][N], fp32.
//
//  naive : one lane per C element, K-loop from global memory (matrixMul_slow)
//  lds   : 64x64 block tile, BK=16, LDS staging, 4x4 register blocking per
//          lane (the lecture's shared-memory tiled kernel, on the f32 VALU)
//  mfma  : 128x128x32 block tile on the matrix cores with the exact-f32
//          v_mfma_f32_32x32x2_f32 (same 64 FLOP/clk/SIMD as the VALU peak but
//          no VALU issue pressure), 4 waves as 2x2, each 64x64 = 2x2 MFMA
//          tiles; register-prefetched double-buffered LDS; XCD-aware block
//          remap. Requires M, N % 128 == 0 and K % 32 == 0 (else `lds`).
#include "cme213/common.h"

namespace {

__global__ __launch_bounds__(256) void sgemm_naive_kernel(int M, int N, int K, float alpha, const float* __restrict__ A,
                                                          const float* __restrict__ B, float beta,
                                                          float* __restrict__ C) {
    const int col = blockIdx.x * 64 + threadIdx.x % 64;
    const int row = blockIdx.y * 4 + threadIdx.x / 64;
    if (row >= M || col >= N) return;
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += A[(size_t)row * K + k] * B[(size_t)k * N + col];
    C[(size_t)row * N + col] = alpha * s + (beta == 0.f ? 0.f : beta * C[(size_t)row * N + col]);
}

constexpr int LT = 64, LK = 16;
__global__ __launch_bounds__(256) void sgemm_lds_kernel(int M, int N, int K, float alpha, const float* __restrict__ A,
                                                        const float* __restrict__ B, float beta,
                                                        float* __restrict__ C) {
    __shared__ float As[LK][LT + 1];  // k-major, padded
    __shared__ float Bs[LK][LT];
    const int tx = threadIdx.x % 16, ty = threadIdx.x / 16;  // 16 x 16 lanes, 4x4 outputs each
    const int r0 = blockIdx.y * LT, c0 = blockIdx.x * LT;
    float acc[4][4] = {};
    for (int k0 = 0; k0 < K; k0 += LK) {
        for (int i = threadIdx.x; i < LT * LK; i += 256) {
            const int r = i / LK, k = i % LK;  // A tile: row r, col k
            As[k][r] = (r0 + r < M && k0 + k < K) ? A[(size_t)(r0 + r) * K + k0 + k] : 0.f;
            const int kb = i / LT, c = i % LT;  // B tile: row kb, col c
            Bs[kb][c] = (k0 + kb < K && c0 + c < N) ? B[(size_t)(k0 + kb) * N + c0 + c] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < LK; ++k) {
            float a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = As[k][ty * 4 + i];
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = Bs[k][tx * 4 + j];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] += a[i] * b[j];
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = r0 + ty * 4 + i, c = c0 + tx * 4 + j;
            if (r < M && c < N)
                C[(size_t)r * N + c] = alpha * acc[i][j] + (beta == 0.f ? 0.f : beta * C[(size_t)r * N + c]);
        }
}

typedef float f32x16 __attribute__((ext_vector_type(16)));
// native 4-vector: HIP's float4 struct is copied with memcpy through a stack
// slot when held in a register array (80 B/lane of scratch in this kernel)
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int MT = 128, MK = 32, APAD = MT + 1;

// Block order: xcd_remap gives each XCD a contiguous range of linear tile
// ids; GM > 0 then walks them in groups of GM tile rows (column-major inside
// the group), so the ~64 tiles an XCD runs at once form a GM x (64/GM) patch
// that shares GM A panels and 64/GM B panels in its L2, instead of one tile
// row that streams 64 different B panels.
template <int GM>
__global__ __launch_bounds__(256) void sgemm_mfma_kernel(int M, int N, int K, float alpha, const float* __restrict__ A,
                                                         const float* __restrict__ B, float beta,
                                                         float* __restrict__ C) {
    __shared__ float As[2][MK * APAD];  // [k][row], padded
    __shared__ float Bs[2][MK * MT];    // [k][col]
    const int t = threadIdx.x;
    const int lane = t & 63, wid = t >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const unsigned nbx = N / MT, nby = M / MT;
    const unsigned lin = xcd_remap(blockIdx.x, nbx * nby);
    int bx, by;
    if (GM > 0 && nby % GM == 0) {
        const unsigned per = GM * nbx, g = lin / per, w = lin % per;
        by = g * GM + w % GM;
        bx = w / GM;
    } else {
        bx = lin % nbx;
        by = lin / nbx;
    }
    const int r0 = by * MT, c0 = bx * MT;

    f32x4 ra[4], rb[4];
    // global -> registers (A: 8 lanes per row along k; B: 32 lanes per k-row)
#define CME_GLOAD(k0)                                                                      \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                        \
        ra[i] = *reinterpret_cast<const f32x4*>(A + (size_t)(r0 + t / 8 + 32 * i) * K + (k0) + (t % 8) * 4); \
        rb[i] = *reinterpret_cast<const f32x4*>(B + (size_t)((k0) + t / 32 + 8 * i) * N + c0 + (t % 32) * 4); \
    }
    // registers -> LDS (A transposed to k-major, padded)
#define CME_LSTORE(buf)                                                                    \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                        \
        const int r = t / 8 + 32 * i, k4 = (t % 8) * 4;                                    \
        As[buf][(k4 + 0) * APAD + r] = ra[i].x;                                            \
        As[buf][(k4 + 1) * APAD + r] = ra[i].y;                                            \
        As[buf][(k4 + 2) * APAD + r] = ra[i].z;                                            \
        As[buf][(k4 + 3) * APAD + r] = ra[i].w;                                            \
        *reinterpret_cast<f32x4*>(&Bs[buf][(t / 32 + 8 * i) * MT + (t % 32) * 4]) = rb[i]; \
    }
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

    CME_GLOAD(0);
    CME_LSTORE(0);
    __syncthreads();
    int buf = 0;
    const int lrow = lane & 31, lk = lane >> 5;
    for (int k0 = 0; k0 < K; k0 += MK) {
        const bool more = k0 + MK < K;
        if (more) {
            CME_GLOAD(k0 + MK);  // prefetch next tile into registers
        }
#pragma unroll
        for (int kk = 0; kk < MK; kk += 2) {
            float a[2], b[2];
#pragma unroll
            for (int m = 0; m < 2; ++m) a[m] = As[buf][(kk + lk) * APAD + wm * 64 + m * 32 + lrow];
#pragma unroll
            for (int n = 0; n < 2; ++n) b[n] = Bs[buf][(kk + lk) * MT + wn * 64 + n * 32 + lrow];
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int n = 0; n < 2; ++n)
                    acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m], b[n], acc[m][n], 0, 0, 0);
        }
        if (more) {
            CME_LSTORE(buf ^ 1);
            __syncthreads();
            buf ^= 1;
        }
    }
#undef CME_GLOAD
#undef CME_LSTORE
    // C/D map: col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = r0 + wm * 64 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                const int col = c0 + wn * 64 + n * 32 + (lane & 31);
                float* cp = C + (size_t)row * N + col;
                *cp = alpha * acc[m][n][r] + (beta == 0.f ? 0.f : beta * *cp);
            }
}

// GEMV y = alpha*A x + beta*y, row-major A[M][K] (the dense matvecs of
// slides/Lecture20.pdf: column-block and 2-D block partitions). A is read once
// and is the whole cost, so this is an HBM-streaming kernel, not an MFMA one:
// G lanes share a row, each lane streams 16-B vectors of it at stride G with
// U loads in flight, A loaded non-temporal so x (re-read by every row) stays
// in L2; the G partial sums reduce with cross-lane shuffles. VEC=false is the
// scalar-load variant for K*sizeof(T) % 16 != 0 or unaligned operands.
template <typename T, int G, bool VEC>
__global__ __launch_bounds__(256) void gemv_kernel(int M, int K, T alpha, const T* __restrict__ A,
                                                   const T* __restrict__ x, T beta, T* __restrict__ y) {
    constexpr int W = 16 / sizeof(T), U = 4;
    typedef T V __attribute__((ext_vector_type(W)));
    const int lane = threadIdx.x % G;
    const long long row = (long long)blockIdx.x * (256 / G) + threadIdx.x / G;
    if (row >= M) return;  // whole G-lane groups leave together: the shuffles stay within live groups
    const T* a = A + row * K;
    T s = 0;
    int k0 = 0;
    if constexpr (VEC) {
        const V* av = reinterpret_cast<const V*>(a);
        const V* xv = reinterpret_cast<const V*>(x);
        const int nv = K / W;
        int v = lane;
        for (; v + (U - 1) * G < nv; v += U * G) {
            V ra[U], rx[U];
#pragma unroll
            for (int u = 0; u < U; ++u) ra[u] = __builtin_nontemporal_load(av + v + u * G);
#pragma unroll
            for (int u = 0; u < U; ++u) rx[u] = xv[v + u * G];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int w = 0; w < W; ++w) s += ra[u][w] * rx[u][w];
        }
        for (; v < nv; v += G) {
            const V ra = __builtin_nontemporal_load(av + v), rx = xv[v];
#pragma unroll
            for (int w = 0; w < W; ++w) s += ra[w] * rx[w];
        }
        k0 = nv * W;
    }
    for (int k = k0 + lane; k < K; k += G) s += a[k] * x[k];
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, G);
    if (lane == 0) y[row] = alpha * s + (beta == T(0) ? T(0) : beta * y[row]);
}

template <typename T>
int launch_gemv(int M, int K, T alpha, const T* A, const T* x, T beta, T* y, hipStream_t s) {
    constexpr int W = 16 / sizeof(T);
    const bool vec = K % W == 0 && (uintptr_t)A % 16 == 0 && (uintptr_t)x % 16 == 0;
    // lanes per row: enough that each lane streams ~2 vectors per row, 4..64
    const int nv = (K + W - 1) / W;
    int G = 4;
    while (G < 64 && 2 * G < nv) G *= 2;
    const dim3 grid(cdiv(M, 256 / G));
    switch (G * 2 + vec) {
#define GV(g)                                                                                                         \
    case 2 * g: hipLaunchKernelGGL((gemv_kernel<T, g, false>), grid, dim3(256), 0, s, M, K, alpha, A, x, beta, y); break; \
    case 2 * g + 1: hipLaunchKernelGGL((gemv_kernel<T, g, true>), grid, dim3(256), 0, s, M, K, alpha, A, x, beta, y); break;
        GV(4) GV(8) GV(16) GV(32) GV(64)
#undef GV
        default: return (int)hipErrorInvalidValue;
    }
    CME_LAUNCH_STATUS();
}

}  // namespace

// y = alpha*A x + beta*y; dtype 0 f32, 4 f64 (codes of the CPU backend)
CME_EXPORT int cme_gemv(int M, int K, double alpha, const void* A, const void* x, double beta, void* y, int dtype,
                        void* stream) {
    if (M <= 0) return 0;
    hipStream_t s = as_stream(stream);
    if (dtype == 0)
        return launch_gemv<float>(M, K, (float)alpha, (const float*)A, (const float*)x, (float)beta, (float*)y, s);
    if (dtype == 4) return launch_gemv<double>(M, K, alpha, (const double*)A, (const double*)x, beta, (double*)y, s);
    return (int)hipErrorInvalidValue;
}

constexpr int kSgemmGroup = 8;

// tuning arms of the mfma kernel (benchmarks/tune_sgemm.py): arm = group rows
CME_EXPORT int cme_sgemm_tune(int M, int N, int K, const float* A, const float* B, float* C, int arm, void* stream) {
    if (M % MT || N % MT || K % MK) return (int)hipErrorInvalidValue;
    hipStream_t s = as_stream(stream);
    const dim3 grid((M / MT) * (N / MT));
    switch (arm) {
#define ARM(g) case g: hipLaunchKernelGGL(sgemm_mfma_kernel<g>, grid, dim3(256), 0, s, M, N, K, 1.f, A, B, 0.f, C); break;
        ARM(0) ARM(1) ARM(2) ARM(4) ARM(8) ARM(16)
#undef ARM
        default: return (int)hipErrorInvalidValue;
    }
    CME_LAUNCH_STATUS();
}

// variant: 0 naive, 1 lds, 2 mfma (falls back to lds when shapes don't tile)
CME_EXPORT int cme_sgemm(int M, int N, int K, float alpha, const float* A, const float* B, float beta, float* C,
                         int variant, void* stream) {
    hipStream_t s = as_stream(stream);
    if (variant == 2 && (M % MT || N % MT || K % MK || ((uintptr_t)A % 16) || ((uintptr_t)B % 16))) variant = 1;
    switch (variant) {
        case 0:
            hipLaunchKernelGGL(sgemm_naive_kernel, dim3(cdiv(N, 64), cdiv(M, 4)), dim3(256), 0, s, M, N, K, alpha, A,
                               B, beta, C);
            break;
        case 1:
            hipLaunchKernelGGL(sgemm_lds_kernel, dim3(cdiv(N, LT), cdiv(M, LT)), dim3(256), 0, s, M, N, K, alpha, A, B,
                               beta, C);
            break;
        case 2:
            hipLaunchKernelGGL(sgemm_mfma_kernel<kSgemmGroup>, dim3((M / MT) * (N / MT)), dim3(256), 0, s, M, N, K,
                               alpha, A, B, beta, C);
            break;
        default: return (int)hipErrorInvalidValue;
    }
    CME_LAUNCH_STATUS();
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(sgemm_naive, 256, sgemm_naive_kernel);
CME_REGISTER_KERNEL(sgemm_lds, 256, sgemm_lds_kernel);
CME_REGISTER_KERNEL(sgemm_mfma, 256, sgemm_mfma_kernel<kSgemmGroup>);
