// Tuning arms of the look-back scan and the fused SpMV-scan (libcme213_tune.so
// only, `make TUNE=1`); production entry points are in csrc/hip/scan.hip.
#include "../hip/scan_kernels.h"

// Diagnostic/tuning arms of the look-back scan (f32 exclusive): rows = 4/8/16
// vectors per lane, lookback = 0 skips the cross-tile pass (wrong results;
// isolates the hand-off cost).
// Tuning arms. lookback: 0 off (timing only, wrong result); 1 persistent
// co-resident grid (production); 2 one tile per block (grid = tiles, relies on
// in-order workgroup dispatch for forward progress); 3/4 as 1/2 with a 2-wide
// look-back window per lane; 5 persistent at half the co-resident grid;
// 6 persistent with the look-back wave prefetching after its look-back;
// 7 / 8 / 9 / 10 persistent, probe-then-window look-back (lookback.h
// lb_lookback_probe) with a 64 x 4 / 8 / 16 / 1 window.
template <int R, bool L, int D, bool LATE = false, int PF = 1, bool NTS = false>
int scan_tune_launch(const float* in, float* out, long long n, int lookback, void* ws, hipStream_t s) {
    const long long tile = 1024LL * R;
    const int tiles = (int)((n + tile - 1) / tile);
    // co-resident capacity of THIS instantiation (arms differ in VGPRs)
    int bpc = persistent_blocks_per_cu(scan_lookback_kernel<float, true, R, L, D, LATE, PF, NTS>, kScanThreads);
    if (lookback == 5) bpc = bpc > 1 ? bpc / 2 : 1;
    int grid = tiles < device_cu_count() * bpc ? tiles : device_cu_count() * bpc;
    if (lookback == 2 || lookback == 4) grid = tiles;
    if (!lb_host_timeout()) return (int)hipErrorOutOfMemory;
    CME_TRY(hipMemsetAsync(ws, 0, D == 200 ? lb2_ws_bytes(tiles) : lb_ws_bytes(tiles), s));
    hipLaunchKernelGGL((scan_lookback_kernel<float, true, R, L, D, LATE, PF, NTS>), dim3(grid), dim3(kScanThreads), 0, s, in,
                       out, n, lb_descriptors(ws), tiles, lb_host_timeout());
    CME_LAUNCH_STATUS();
}

template <int R>
int scan_tune_rows(const float* in, float* out, long long n, int lookback, void* ws, hipStream_t s) {
    switch (lookback) {
        case 0: return scan_tune_launch<R, false, 1>(in, out, n, lookback, ws, s);
        case 3:
        case 4: return scan_tune_launch<R, true, 2>(in, out, n, lookback, ws, s);
        case 6: return scan_tune_launch<R, true, 1, true>(in, out, n, lookback, ws, s);
        case 7: return scan_tune_launch<R, true, -4>(in, out, n, lookback, ws, s);
        case 8: return scan_tune_launch<R, true, -8>(in, out, n, lookback, ws, s);
        case 9: return scan_tune_launch<R, true, -16>(in, out, n, lookback, ws, s);
        case 10: return scan_tune_launch<R, true, -1>(in, out, n, lookback, ws, s);
        case 11: return scan_tune_launch<R, true, 104>(in, out, n, lookback, ws, s);
        case 12: return scan_tune_launch<R, true, 116>(in, out, n, lookback, ws, s);
        case 13: return scan_tune_launch<R, true, 100>(in, out, n, lookback, ws, s);
        case 14: return scan_tune_launch<R, true, 200>(in, out, n, lookback, ws, s);
        case 15: return scan_tune_launch<R, true, 200, false, 2>(in, out, n, lookback, ws, s);
        case 16: return scan_tune_launch<R, true, 1, false, 2>(in, out, n, lookback, ws, s);
        case 17: return scan_tune_launch<R, false, 1, false, 2>(in, out, n, lookback, ws, s);
        case 18: return scan_tune_launch<R, true, 200, false, 2, true>(in, out, n, lookback, ws, s);
        case 19: return scan_tune_launch<R, false, 1, false, 2, true>(in, out, n, lookback, ws, s);
        default: return scan_tune_launch<R, true, 1>(in, out, n, lookback, ws, s);
    }
}

CME_EXPORT int cme_scan_tune(const float* in, float* out, long long n, int rows, int lookback, void* ws,
                             void* stream) {
    hipStream_t s = as_stream(stream);
    switch (rows) {
        case 4: return scan_tune_rows<4>(in, out, n, lookback, ws, s);
        case 8: return scan_tune_rows<8>(in, out, n, lookback, ws, s);
        case 16: return scan_tune_rows<16>(in, out, n, lookback, ws, s);
        default: return (int)hipErrorInvalidValue;
    }
}
// Tuning entry (benchmarks/tune_scan.py --spmv): rows 4/8/16 x mode: bit 0
// prefetch the next tile before the look-back, bit 1 two-level look-back,
// bit 2 all steps in one launch (with bit 1).
CME_EXPORT int cme_spmv_scan_tune(float* a, const float* xx, const uint32_t* flags, long long n, int iters, void* ws,
                                  int rows, int mode, void* stream) {
    if (n <= 0 || iters <= 0) return 0;
    hipStream_t s = as_stream(stream);
#define SPT(R)                                                                             \
    switch (mode & 7) {                                                                    \
        case 0: return spmv_scan_launch<R, false, false>(a, xx, flags, n, iters, ws, s);       \
        case 1: return spmv_scan_launch<R, true, false>(a, xx, flags, n, iters, ws, s);        \
        case 2: return spmv_scan_launch<R, false, true>(a, xx, flags, n, iters, ws, s);        \
        case 3: return spmv_scan_launch<R, true, true>(a, xx, flags, n, iters, ws, s);         \
        case 6: return spmv_scan_launch<R, false, true, true>(a, xx, flags, n, iters, ws, s);  \
        case 7: return spmv_scan_launch<R, true, true, true>(a, xx, flags, n, iters, ws, s);   \
        default: return (int)hipErrorInvalidValue;                                         \
    }
    if (rows == 1) SPT(1)
    if (rows == 2) SPT(2)
    if (rows == 4) SPT(4)
    if (rows == 8) SPT(8)
    if (rows == 16) SPT(16)
#undef SPT
    return (int)hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------
// Tuning arms of the Blelloch tile-parallel reduce-then-scan (f32, exclusive;
// production: scan_kernels.h launch_tree_rts, BASELINE config #3).
// benchmarks/tune_tree_scan.py times them cold.
//   arm 0 production                    arm 1 K1 grid 2048
//   arm 2 K1 two tiles in flight        arm 3 K1 one tile per block (grid = tiles)
//   arm 4 K3 grid 2048                  arm 5 = 2 + 4
//   arm 6 K2 fused into K1: the last K1 block to finish (one device-scope
//         atomic per block) scans the tile sums, saving a launch
//   arm 7 = 2 + 6
// ws: 4 B per 4096-element tile, then a 256-B aligned counter word (arms 6-7;
// it must start zeroed, the last block leaves it zeroed).
namespace {
template <int PF>
__global__ __launch_bounds__(256) void tile_reduce_tune_kernel(const float* __restrict__ in, long long n, int ntiles,
                                                               float* __restrict__ tsum, unsigned* __restrict__ counter) {
    __shared__ float lds[4];
    __shared__ unsigned s_last;
    Vec4<float> q[PF][4];
    const int G = (int)gridDim.x;
    int tile = blockIdx.x;
#pragma unroll
    for (int p = 0; p < PF; ++p)
        if (tile + p * G < ntiles) tile_load4(in, (long long)(tile + p * G) * kTreeTile, n, q[p]);
    for (; tile < ntiles; tile += G) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) acc = acc + ((q[0][k].x + q[0][k].y) + (q[0][k].z + q[0][k].w));
#pragma unroll
        for (int p = 0; p + 1 < PF; ++p)
#pragma unroll
            for (int k = 0; k < 4; ++k) q[p][k] = q[p + 1][k];
        if (tile + PF * G < ntiles) tile_load4(in, (long long)(tile + PF * G) * kTreeTile, n, q[PF - 1]);
        const float r = block_reduce<4>(acc, lds, OpAdd());
        if (threadIdx.x == 0) tsum[tile] = r;
    }
    if (!counter) return;  // block-uniform
    __threadfence();       // this block's tile sums, device-wide, before its arrival
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(counter, 1u) == (unsigned)G - 1u ? 1u : 0u;
    lds_bcast_sync();
    if (!s_last) return;
    __threadfence();  // every other block's tile sums
    // exclusive scan of the ntiles sums in place: 16 per thread per round
    constexpr int kPer = 16, kRound = 256 * kPer;
    __shared__ float stage[tpad(kRound)];
    __shared__ float wl[4];
    const int t = threadIdx.x;
    float carry = 0.f;
    for (int base = 0; base < ntiles; base += kRound) {
#pragma unroll
        for (int k = 0; k < kPer / 4; ++k) {
            const int e = (k * 256 + t) * 4;
            const Vec4<float> v = load_v4(tsum, (long long)base + e, ntiles, 0.f);
            stage[tpad(e)] = v.x;
            stage[tpad(e + 1)] = v.y;
            stage[tpad(e + 2)] = v.z;
            stage[tpad(e + 3)] = v.w;
        }
        __syncthreads();
        float v[kPer], acc = 0.f;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            v[k] = stage[tpad(t * kPer + k)];
            acc = acc + v[k];
        }
        float tot;
        float run = carry + block_exclusive_scan<4>(acc, wl, tot, OpAdd());
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            stage[tpad(t * kPer + k)] = run;
            run = run + v[k];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kPer / 4; ++k) {
            const int e = (k * 256 + t) * 4;
            store_v4(tsum, (long long)base + e, ntiles,
                     Vec4<float>{stage[tpad(e)], stage[tpad(e + 1)], stage[tpad(e + 2)], stage[tpad(e + 3)]});
        }
        __syncthreads();
        carry = carry + tot;
    }
    if (t == 0) *counter = 0u;  // ready for the next call on this workspace
}
}  // namespace

CME_EXPORT int cme_scan_tree_tune(const float* in, float* out, long long n, int arm, void* ws, void* stream) {
    hipStream_t s = as_stream(stream);
    if (n <= 0) return 0;
    const long long tiles = (n + kTreeTile - 1) / kTreeTile;
    if (tiles >= (1ll << 31)) return (int)hipErrorInvalidValue;
    const int nt = (int)tiles;
    if (arm == 0) return launch_tree_rts<float>(in, out, n, 0, 1, ws, s);
    float* part = (float*)ws;
    unsigned* counter = (arm == 6 || arm == 7) ? (unsigned*)((char*)ws + ((size_t)nt * 4 + 255) / 256 * 256) : nullptr;
    const int cap = [&] { int c = nt < kRtsBlocks ? nt : kRtsBlocks; return c; }();
    int g1 = cap, g3 = cap;
    if (arm == 1) g1 = nt < 2048 ? nt : 2048;
    if (arm == 3) g1 = nt;
    if (arm == 4 || arm == 5) g3 = nt < 2048 ? nt : 2048;
    if (arm == 2 || arm == 5 || arm == 7)
        hipLaunchKernelGGL(tile_reduce_tune_kernel<2>, dim3(g1), dim3(256), 0, s, in, n, nt, part, counter);
    else
        hipLaunchKernelGGL(tile_reduce_tune_kernel<1>, dim3(g1), dim3(256), 0, s, in, n, nt, part, counter);
    if (!counter) hipLaunchKernelGGL(rts_partials_kernel<float>, dim3(1), dim3(1024), 0, s, part, nt);
    hipLaunchKernelGGL((tile_tree_scan_kernel<float, true, 0>), dim3(g3), dim3(256), 0, s, in, out, n, nt, part);
    CME_LAUNCH_STATUS();
}

// ---------------------------------------------------------------------------
// Tuning arms of the f32 sum reduction (production: scan.hip cme_reduce,
// reduce_partial_kernel + reduce_final_kernel; BASELINE config #3).
// benchmarks/tune_reduce.py times them cold.
//   arm 0 production (grid 1024, one 16-B load in flight per lane)
//   arm 1 four 16-B loads in flight per lane (grid 1024)
//   arm 2 = 1 with grid 2048
//   arm 3 = 1 with the final reduction by the last block to finish (one
//         device-scope arrival atomic per block; no second launch)
// part: >= 2048 floats, then a 256-B aligned counter word (arm 3: zero at
// the first call, left zeroed).
extern "C" int cme_reduce(const void* in, long long n, int dtype, int op, int algo, void* part, void* out,
                          void* stream);  // production (libcme213_hip.so)
namespace {
template <int U, bool LAST>
__global__ __launch_bounds__(256) void reduce_unr_kernel(const float* __restrict__ in, long long n,
                                                         float* __restrict__ part, unsigned* __restrict__ counter,
                                                         float* __restrict__ out) {
    __shared__ float lds[4];
    __shared__ unsigned s_last;
    float acc = 0.f;
    const long long stride = (long long)gridDim.x * 256 * 4;
    long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        Vec4<float> v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = load_v4(in, i + u * stride, n, 0.f);
#pragma unroll
        for (int u = 0; u < U; ++u) acc = acc + ((v[u].x + v[u].y) + (v[u].z + v[u].w));
    }
    for (; i < n; i += stride) {
        const Vec4<float> v = load_v4(in, i, n, 0.f);
        acc = acc + ((v.x + v.y) + (v.z + v.w));
    }
    const float r = block_reduce<4>(acc, lds, OpAdd());
    if (threadIdx.x == 0) part[blockIdx.x] = r;
    if constexpr (LAST) {
        __threadfence();
        __syncthreads();
        if (threadIdx.x == 0) s_last = atomicAdd(counter, 1u) == gridDim.x - 1u ? 1u : 0u;
        lds_bcast_sync();
        if (!s_last) return;
        __threadfence();
        float a = 0.f;
        for (int j = threadIdx.x; j < (int)gridDim.x; j += 256) a = a + part[j];
        const float t = block_reduce<4>(a, lds, OpAdd());
        if (threadIdx.x == 0) {
            *out = t;
            *counter = 0u;
        }
    }
}
}  // namespace

CME_EXPORT int cme_reduce_tune(const float* in, long long n, int arm, float* part, float* out, void* stream) {
    hipStream_t s = as_stream(stream);
    if (arm == 0) return cme_reduce(in, n, 0, 0, 0, part, out, stream);
    unsigned* counter = (unsigned*)((char*)part + 2048 * 4);
    const int grid = arm == 2 ? 2048 : 1024;
    if (arm == 3) {
        hipLaunchKernelGGL((reduce_unr_kernel<4, true>), dim3(grid), dim3(256), 0, s, in, n, part, counter, out);
    } else {
        hipLaunchKernelGGL((reduce_unr_kernel<4, false>), dim3(grid), dim3(256), 0, s, in, n, part, counter, out);
        hipLaunchKernelGGL((reduce_final_kernel<float, OpAdd>), dim3(1), dim3(1024), 0, s, (const float*)part, grid,
                           out, OpAdd());
    }
    CME_LAUNCH_STATUS();
}
