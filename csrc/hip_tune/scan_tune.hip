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
