// SGEMM ladder (slides/Lecture09 slides 5-18): C = alpha*A*B + beta*C,
// row-major A[M][K], B[K][N], C[M][N], fp32.
//
//  naive : one lane per C element, K-loop from global memory (matrixMul_slow)
//  lds   : 64x64 block tile, BK=16, LDS staging, 4x4 register blocking per
//          lane (the lecture's shared-memory tiled kernel, on the f32 VALU)
//  mfma  : matrix cores with the exact-f32 v_mfma_f32_32x32x2_f32 (same 64
//          FLOP/clk/SIMD as the VALU peak but no VALU issue pressure), one
//          generic tile kernel (sgemm_tile_kernel): 256x256x32 block, 8 waves
//          of 64x128 when M, N % 256 == 0, else 128x128x32 with 4 waves of
//          64x64; double-buffered LDS filled from registers mid-tile, global
//          loads two tiles ahead, vector LDS operand reads, XCD-aware block
//          order. Requires M, N % 128 == 0 and K % 32 == 0 (else `lds`).
//          8192^3: 144 TFLOP/s = 94 % of hipBLASLt (profiles/sgemm_notes.md).
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
constexpr int MT = 128, MK = 32;

// Generic MFMA tile: BM x BN block, WGM x WGN waves (each a (BM/WGM) x
// (BN/WGN) patch of 32x32 v_mfma_f32_32x32x2_f32 tiles), K tile 32.
//   * LDS double-buffered: A k-major with an odd pitch (BM+1, conflict-free
//     transposed scalar stores), B k-major [32][BN] with 16-B stores;
//   * the next K tile is loaded into registers at the top of a tile and
//     written to the other LDS buffer at k-step STORE_AT, so only the barrier
//     remains at the tile end;
//   * LDS operands are read one k-step ahead of the MFMAs that use them;
//   * block order: xcd_remap gives each XCD a contiguous range of linear
//     tile ids; GM > 0 walks them in groups of GM tile rows (column-major
//     inside the group), so the tiles an XCD runs at once form a patch that
//     shares A and B panels in its L2 (measured neutral at 8192^3: the
//     operands stream from MALL fast enough either way).
// Requires M % BM == 0, N % BN == 0, K % 32 == 0, 16-B aligned A and B.
// DEEP: the registers are refilled right after they are stored (tile k+2
// loaded during tile k), so the loads have a whole tile of MFMA work to land
// before the next store needs them, instead of STORE_AT k-steps.
// SB: scheduling barriers pin the one-step-ahead LDS reads in front of the
// MFMAs (left alone, the machine scheduler sinks them behind the MFMAs and
// reuses their registers, re-exposing the LDS latency every k-step).
// VR: vector LDS reads. A wave's TM (TN) sub-tiles take interleaved rows
// (columns) -- sub-tile m holds rows TM*i + m -- so a lane's TM A operands
// and TN B operands of one k-step are contiguous: one ds_read_b64/b128 each
// instead of ds_read2_b32 pairs (half the LDS cycles per MFMA), and the
// epilogue stores TN adjacent columns as one vector. The A pitch becomes
// BM + TM (aligned vectors; its transposed scalar stores go 2-way, free).
template <int BM, int BN, int WGM, int WGN, int STORE_AT, int GM, bool DEEP = false, bool SB = false, bool VR = false>
__global__ __launch_bounds__(64 * WGM * WGN) void sgemm_tile_kernel(int M, int N, int K, float alpha,
                                                                    const float* __restrict__ A,
                                                                    const float* __restrict__ B, float beta,
                                                                    float* __restrict__ C) {
    constexpr int WTM = BM / WGM, WTN = BN / WGN, TM = WTM / 32, TN = WTN / 32;
    constexpr int NT = 64 * WGM * WGN, KT = 32, AP = VR ? BM + TM : BM + 1;
    static_assert(!VR || ((TM == 2 || TM == 4) && (TN == 2 || TN == 4)), "vector reads need 2 or 4 sub-tiles");
    typedef float VA __attribute__((ext_vector_type(TM)));
    typedef float VB __attribute__((ext_vector_type(TN)));
    constexpr int NA = BM * KT / 4 / NT, NB = KT * BN / 4 / NT;
    static_assert(NA * NT * 4 == BM * KT && NB * NT * 4 == KT * BN, "tile does not split over the block");
    static_assert(TM * 32 == WTM && TN * 32 == WTN, "wave tile must be a multiple of 32");
    __shared__ float As[2][KT * AP];
    __shared__ float Bs[2][KT * BN];
    const int t = threadIdx.x;
    const int lane = t & 63, wid = t >> 6;
    const int wm = wid / WGN, wn = wid % WGN;
    const unsigned nbx = N / BN, nby = M / BM;
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
    const int r0 = by * BM, c0 = bx * BN;

    f32x4 ra[NA], rb[NB];
    auto gload = [&](int k0) {
#pragma unroll
        for (int i = 0; i < NA; ++i)
            ra[i] = *reinterpret_cast<const f32x4*>(A + (size_t)(r0 + t / 8 + (NT / 8) * i) * K + k0 + (t % 8) * 4);
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int e = t + NT * i;
            rb[i] = *reinterpret_cast<const f32x4*>(B + (size_t)(k0 + e / (BN / 4)) * N + c0 + (e % (BN / 4)) * 4);
        }
    };
    auto lstore = [&](int b) {
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int r = t / 8 + (NT / 8) * i, k4 = (t % 8) * 4;
            As[b][(k4 + 0) * AP + r] = ra[i].x;
            As[b][(k4 + 1) * AP + r] = ra[i].y;
            As[b][(k4 + 2) * AP + r] = ra[i].z;
            As[b][(k4 + 3) * AP + r] = ra[i].w;
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int e = t + NT * i;
            *reinterpret_cast<f32x4*>(&Bs[b][(e / (BN / 4)) * BN + (e % (BN / 4)) * 4]) = rb[i];
        }
    };
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

    gload(0);
    lstore(0);
    if (DEEP && KT < K) gload(KT);
    __syncthreads();
    int buf = 0;
    const int lrow = lane & 31, lk = lane >> 5;
    for (int k0 = 0; k0 < K; k0 += KT) {
        const bool more = k0 + KT < K;
        if (!DEEP && more) gload(k0 + KT);
        const float* as = As[buf] + lk * AP + wm * WTM + (VR ? lrow * TM : lrow);
        const float* bs = Bs[buf] + lk * BN + wn * WTN + (VR ? lrow * TN : lrow);
        float a[2][TM], b[2][TN];
        auto lread = [&](int kk, int x) {
            if constexpr (VR) {
                const VA va = *reinterpret_cast<const VA*>(as + kk * AP);
                const VB vb = *reinterpret_cast<const VB*>(bs + kk * BN);
#pragma unroll
                for (int m = 0; m < TM; ++m) a[x][m] = va[m];
#pragma unroll
                for (int n = 0; n < TN; ++n) b[x][n] = vb[n];
            } else {
#pragma unroll
                for (int m = 0; m < TM; ++m) a[x][m] = as[kk * AP + m * 32];
#pragma unroll
                for (int n = 0; n < TN; ++n) b[x][n] = bs[kk * BN + n * 32];
            }
        };
        lread(0, 0);
#pragma unroll
        for (int kk = 0; kk < KT; kk += 2) {
            const int c = (kk / 2) & 1;
            if (kk + 2 < KT) lread(kk + 2, c ^ 1);
            if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
            if (kk == STORE_AT && more) {
                lstore(buf ^ 1);
                if (DEEP && k0 + 2 * KT < K) gload(k0 + 2 * KT);
            }
#pragma unroll
            for (int m = 0; m < TM; ++m)
#pragma unroll
                for (int n = 0; n < TN; ++n)
                    acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[c][m], b[c][n], acc[m][n], 0, 0, 0);
            if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
        }
        if (more) {
            if (STORE_AT >= KT) {
                lstore(buf ^ 1);
                if (DEEP && k0 + 2 * KT < K) gload(k0 + 2 * KT);
            }
            __syncthreads();
            buf ^= 1;
        }
    }
    // C/D map: col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
    if constexpr (VR) {
#pragma unroll
        for (int m = 0; m < TM; ++m)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = r0 + wm * WTM + TM * ((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) + m;
                VB* cp = reinterpret_cast<VB*>(C + (size_t)row * N + c0 + wn * WTN + TN * (lane & 31));
                VB v;
#pragma unroll
                for (int n = 0; n < TN; ++n) v[n] = alpha * acc[m][n][r];
                if (beta != 0.f) v += beta * *cp;
                *cp = v;
            }
    } else {
#pragma unroll
        for (int m = 0; m < TM; ++m)
#pragma unroll
            for (int n = 0; n < TN; ++n)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = r0 + wm * WTM + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    const int col = c0 + wn * WTN + n * 32 + (lane & 31);
                    float* cp = C + (size_t)row * N + col;
                    *cp = alpha * acc[m][n][r] + (beta == 0.f ? 0.f : beta * *cp);
                }
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
// production: 256x256 block, 8 waves of 64x128, vector LDS reads, tile k+2
// loaded during tile k (tune arm 74); 128x128 (arm 79) when the 256 grid
// would leave CUs idle (2048^3: 64 blocks, 36 vs 101 TFLOP/s) or the shape
// does not tile by 256
#define CME_SGEMM_256 sgemm_tile_kernel<256, 256, 4, 2, 0, kSgemmGroup, true, false, true>
#define CME_SGEMM_128 sgemm_tile_kernel<128, 128, 2, 2, 0, kSgemmGroup, true, false, true>

// tuning arms of the MFMA tile kernel (benchmarks/tune_sgemm.py; results in
// profiles/sgemm_tune_r2.log): id -> <BM, BN, WGM, WGN, STORE_AT, GM, DEEP, SB, VR>
CME_EXPORT int cme_sgemm_tune(int M, int N, int K, const float* A, const float* B, float* C, int arm, void* stream) {
    if (K % MK) return (int)hipErrorInvalidValue;
    hipStream_t s = as_stream(stream);
    switch (arm) {
#define TILE(id, bm, bn, wm, wn, st, g, ...)                                                                   \
    case id:                                                                                                  \
        if (M % bm || N % bn) return (int)hipErrorInvalidValue;                                               \
        hipLaunchKernelGGL((sgemm_tile_kernel<bm, bn, wm, wn, st, g, ##__VA_ARGS__>), dim3((M / bm) * (N / bn)),   \
                           dim3(64 * wm * wn), 0, s, M, N, K, 1.f, A, B, 0.f, C);                              \
        break;
        TILE(0, 128, 128, 2, 2, 32, 0)  // the round-1 kernel: row-major order, store after the loop
        TILE(8, 128, 128, 2, 2, 32, 8)
        TILE(40, 128, 128, 2, 2, 16, 8) TILE(41, 256, 128, 2, 2, 16, 8) TILE(43, 256, 256, 2, 4, 16, 8)
        TILE(44, 256, 256, 4, 2, 16, 8) TILE(45, 128, 256, 2, 4, 16, 8) TILE(55, 256, 256, 4, 4, 16, 8)
        TILE(57, 256, 256, 4, 2, 4, 8) TILE(58, 256, 256, 4, 2, 4, 8, true) TILE(67, 256, 256, 4, 2, 0, 8, true, true)
        TILE(72, 256, 256, 4, 2, 4, 8, false, false, true) TILE(73, 256, 256, 4, 2, 0, 8, true, true, true)
        TILE(74, 256, 256, 4, 2, 0, 8, true, false, true) TILE(75, 256, 256, 4, 4, 0, 8, true, false, true)
        TILE(76, 128, 128, 2, 2, 16, 8, false, false, true) TILE(77, 256, 256, 2, 4, 0, 8, true, false, true)
        TILE(78, 128, 256, 2, 4, 0, 8, true, false, true) TILE(79, 128, 128, 2, 2, 0, 8, true, false, true)
        TILE(80, 128, 128, 2, 2, 0, 8, true, true, false) TILE(81, 256, 128, 4, 2, 0, 8, true, false, true)
#undef TILE
        default: return (int)hipErrorInvalidValue;
    }
    CME_LAUNCH_STATUS();
}

// variant: 0 naive, 1 lds, 2 mfma (falls back to lds when shapes don't tile)
CME_EXPORT int cme_sgemm(int M, int N, int K, float alpha, const float* A, const float* B, float beta, float* C,
                         int variant, void* stream) {
    hipStream_t s = as_stream(stream);
    // the MFMA epilogue stores (and, with beta != 0, loads) 16-B vectors of C: an
    // offset view of C that is not 16-B aligned takes the LDS kernel too
    if (variant == 2 && (M % MT || N % MT || K % MK || ((uintptr_t)A % 16) || ((uintptr_t)B % 16) ||
                         ((uintptr_t)C % 16)))
        variant = 1;
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
            if (M % 256 == 0 && N % 256 == 0 && (long long)(M / 256) * (N / 256) >= device_cu_count())
                hipLaunchKernelGGL((CME_SGEMM_256), dim3((M / 256) * (N / 256)), dim3(512), 0, s, M, N, K, alpha, A, B,
                                   beta, C);
            else
                hipLaunchKernelGGL((CME_SGEMM_128), dim3((M / MT) * (N / MT)), dim3(256), 0, s, M, N, K, alpha, A, B,
                                   beta, C);
            break;
        default: return (int)hipErrorInvalidValue;
    }
    CME_LAUNCH_STATUS();
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(sgemm_naive, 256, sgemm_naive_kernel);
CME_REGISTER_KERNEL(sgemm_lds, 256, sgemm_lds_kernel);
CME_REGISTER_KERNEL(sgemm_mfma128, 256, CME_SGEMM_128);
CME_REGISTER_KERNEL(sgemm_mfma256, 512, CME_SGEMM_256);
