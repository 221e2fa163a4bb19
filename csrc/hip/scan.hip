// Scan and reduction family (Lecture16 / Harris scan.pdf / nvr-2008-003,
// Lecture05 tree reduction), written for wave64.
//
//  * cme_scan           single-pass decoupled look-back scan (the fast one):
//                       4096-element tiles, 16 B/lane coalesced loads, DPP wave
//                       scans, one 8-B granule per tile for the hand-off.
//  * cme_scan_mlevel    multi-level scan-then-add (Harris Fig. 5) with a
//                       selectable block algorithm: Blelloch work-efficient
//                       up/down-sweep in LDS with bank-conflict-free padding, or
//                       Hillis-Steele (naive, O(n log n)).
//  * cme_reduce         two-pass block reduction (grid-stride 16-B loads, DPP
//                       wave reduce, LDS across waves) and the lecture's
//                       shared-memory tree (`s = blockDim/2; s >>= 1`) variant.
//  * cme_segscan        single-pass segmented inclusive scan with head flags.
//  * cme_spmv_scan_step fused final-project step: a[i] *= xx[i] then inclusive
//                       segmented scan of a (segment heads as a bitmask).
#include "scan_kernels.h"

// The look-back give-up word: pinned, mapped host memory (lookback.h). One per
// process; device stores reach it directly, the host reads it without a sync.
// One give-up word per device (its own 64-B line): a timed-out launch on one
// GPU does not poison look-back launches on another.
unsigned* cme::lb_host_timeout() {
    static unsigned* words = [] {
        void* p = nullptr;
        if (hipHostMalloc(&p, 64 * 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
            return (unsigned*)nullptr;
        for (int i = 0; i < 64 * 16; ++i) ((volatile unsigned*)p)[i] = 0u;
        return (unsigned*)p;
    }();
    if (!words) return nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    return words + 16 * (dev & 63);
}

// Host address of the current device's word (ops/scan.py reads / clears it).
CME_EXPORT int cme_lookback_timeout_word(void** host_word) {
    unsigned* w = lb_host_timeout();
    if (!w) return (int)hipErrorOutOfMemory;
    *host_word = w;
    return 0;
}


// Reduce-then-scan (deterministic). ws: >= 4 * 1024 bytes.
CME_EXPORT int cme_scan_rts(const void* in, void* out, long long n, int dtype, int exclusive, void* ws, void* stream) {
    hipStream_t s = as_stream(stream);
    switch (dtype) {
        case 0: return launch_rts<float>((const float*)in, (float*)out, n, exclusive, ws, s);
        case 1: return launch_rts<int>((const int*)in, (int*)out, n, exclusive, ws, s);
        case 2: return launch_rts<uint32_t>((const uint32_t*)in, (uint32_t*)out, n, exclusive, ws, s);
        default: return (int)hipErrorInvalidValue;
    }
}

// Tile-parallel reduce-then-scan with a tree block scan (scan_kernels.h
// launch_tree_rts): algo 0 Blelloch, 1 Hillis-Steele. ws: >= 4 * ceil(n / 4096)
// bytes (the tile sums, then their prefixes).
CME_EXPORT int cme_scan_tree(const void* in, void* out, long long n, int dtype, int algo, int exclusive, void* ws,
                             void* stream) {
    hipStream_t s = as_stream(stream);
    switch (dtype) {
        case 0: return launch_tree_rts<float>((const float*)in, (float*)out, n, algo, exclusive, ws, s);
        case 1: return launch_tree_rts<int>((const int*)in, (int*)out, n, algo, exclusive, ws, s);
        case 2: return launch_tree_rts<uint32_t>((const uint32_t*)in, (uint32_t*)out, n, algo, exclusive, ws, s);
        default: return (int)hipErrorInvalidValue;
    }
}

// dtype: 0 f32, 1 i32, 2 u32. ws: >= 8*ceil(n/4096) + 16 bytes.
// epoch: see launch_scan (0 = zero the workspace here)
CME_EXPORT int cme_scan(const void* in, void* out, long long n, int dtype, int exclusive, void* ws, unsigned epoch,
                        void* stream) {
    hipStream_t s = as_stream(stream);
    switch (dtype) {
        case 0: return launch_scan<float>((const float*)in, (float*)out, n, exclusive, ws, s, epoch);
        case 1: return launch_scan<int>((const int*)in, (int*)out, n, exclusive, ws, s, epoch);
        case 2: return launch_scan<uint32_t>((const uint32_t*)in, (uint32_t*)out, n, exclusive, ws, s, epoch);
        default: return (int)hipErrorInvalidValue;
    }
}

CME_EXPORT long long cme_scan_ws_bytes(long long n) { return (long long)lb2_ws_bytes((n + kScanTile - 1) / kScanTile); }


CME_EXPORT long long cme_scan_mlevel_ws_elems(long long n) {
    long long tot = 0;
    long long b = (n + kMLElems - 1) / kMLElems;
    while (b > 1) {
        tot += b;
        b = (b + kMLElems - 1) / kMLElems;
    }
    return tot + 1;
}

// algo: 0 Blelloch, 1 Hillis-Steele; dtype 0 f32, 1 i32. inclusive via add-back.
CME_EXPORT int cme_scan_mlevel(const void* in, void* out, long long n, int dtype, int algo, int exclusive, void* ws,
                               void* stream) {
    hipStream_t s = as_stream(stream);
    if (n <= 0) return 0;
    int rc;
    if (dtype == 0) rc = mlevel<float>((const float*)in, (float*)out, n, algo, (float*)ws, s);
    else if (dtype == 1) rc = mlevel<int>((const int*)in, (int*)out, n, algo, (int*)ws, s);
    else return (int)hipErrorInvalidValue;
    if (rc) return rc;
    if (!exclusive) {
        unsigned g = cdiv(n, 256);
        if (dtype == 0) hipLaunchKernelGGL(to_inclusive_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)in, (float*)out, n);
        else hipLaunchKernelGGL(to_inclusive_kernel<int>, dim3(g), dim3(256), 0, s, (const int*)in, (int*)out, n);
    }
    CME_LAUNCH_STATUS();
}

// op: 0 sum, 1 max, 2 min; dtype 0 f32, 1 i32. algo 0 = DPP/vector, 1 = LDS tree (sum only).
// part: >= 2048 elements of scratch. result written to `out` (device).
CME_EXPORT int cme_reduce(const void* in, long long n, int dtype, int op, int algo, void* part, void* out,
                          void* stream) {
    hipStream_t s = as_stream(stream);
    const int grid = 1024;
#define RED(T, OP)                                                                                              \
    hipLaunchKernelGGL((reduce_partial_kernel<T, OP>), dim3(grid), dim3(256), 0, s, (const T*)in, n, (T*)part, OP()); \
    hipLaunchKernelGGL((reduce_final_kernel<T, OP>), dim3(1), dim3(1024), 0, s, (const T*)part, grid, (T*)out, OP());
    if (algo == 1) {
        if (op != 0) return (int)hipErrorInvalidValue;
        if (dtype == 0) {
            hipLaunchKernelGGL(reduce_tree_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)in, n, (float*)part);
            hipLaunchKernelGGL((reduce_final_kernel<float, OpAdd>), dim3(1), dim3(1024), 0, s, (const float*)part,
                               grid, (float*)out, OpAdd());
        } else {
            hipLaunchKernelGGL(reduce_tree_kernel<int>, dim3(grid), dim3(256), 0, s, (const int*)in, n, (int*)part);
            hipLaunchKernelGGL((reduce_final_kernel<int, OpAdd>), dim3(1), dim3(1024), 0, s, (const int*)part, grid,
                               (int*)out, OpAdd());
        }
        CME_LAUNCH_STATUS();
    }
    if (dtype == 0) {
        if (op == 0) { RED(float, OpAdd) }
        else if (op == 1) { RED(float, OpMax) }
        else { RED(float, OpMin) }
    } else if (dtype == 1) {
        if (op == 0) { RED(int, OpAdd) }
        else if (op == 1) { RED(int, OpMax) }
        else { RED(int, OpMin) }
    } else {
        return (int)hipErrorInvalidValue;
    }
#undef RED
    CME_LAUNCH_STATUS();
}

// Segmented inclusive scan (float add). flag_mode 0: uint8 per element;
// 1: bitmask words. xmul != null fuses in[i]*xmul[i] (final-project step).
CME_EXPORT int cme_segscan(const float* in, const float* xmul, float* out, const void* flags, int flag_mode,
                           long long n, void* ws, unsigned epoch, void* stream) {
    hipStream_t s = as_stream(stream);
    if (n <= 0) return 0;
    const int tiles = (int)((n + kScanTile - 1) / kScanTile);
    static int bpc = persistent_blocks_per_cu(segscan_kernel<1, true, 4, false, true>, kScanThreads);
    const int grid = tiles < device_cu_count() * bpc ? tiles : device_cu_count() * bpc;
    unsigned* timeout = lb_host_timeout();
    if (!timeout) return (int)hipErrorOutOfMemory;
    uint64_t* desc = lb_descriptors(ws);
    if (epoch == 0) CME_TRY(hipMemsetAsync(ws, 0, lb2_ws_bytes(tiles), s));
    if (epoch >= (1u << 24)) return (int)hipErrorInvalidValue;
    const uint32_t ep = epoch ? epoch : 1u;
#define SEG(M, F)                                                                                                   \
    hipLaunchKernelGGL((segscan_kernel<M, F, 4, false, true>), dim3(grid), dim3(kScanThreads), 0, s, in, xmul, out, \
                       flags, n, desc, tiles, timeout, ep)
    if (flag_mode == 0) {
        if (xmul) SEG(0, true); else SEG(0, false);
    } else {
        if (xmul) SEG(1, true); else SEG(1, false);
    }
#undef SEG
    CME_LAUNCH_STATUS();
}


// Default: all steps in one persistent launch per 64 steps (segscan_kernel
// MULTI). CME_SPMVSCAN_MULTI=0 restores one launch per step: two-level
// look-back, 4 rows per lane, the next tile prefetched behind the look-back
// only when a block owns several tiles (a multi-round grid).
// benchmarks/tune_scan.py --spmv (profiles/spmvscan_tune_r2.log), GB/s at the
// 12 B/element model: pwtk 4821 (prefetch) / 4521, webbase-1M 4451 (no
// prefetch) / 4157, mac_econ 2273 / 2027; round 1's one-level arm: 3931 /
// 4257 / 2173.
CME_EXPORT int cme_spmv_scan_run(float* a, const float* xx, const uint32_t* flags, long long n, int iters, void* ws,
                                 void* stream) {
    if (n <= 0 || iters <= 0) return 0;
    const long long tiles = (n + 4095) / 4096;
    const bool multi = cme::tune_get(cme::kTuneSpmvScanMulti) != 0;  // 0: one launch per step (the round-2 path)
    static int bpc = persistent_blocks_per_cu(segscan_kernel<1, true, 4, true, true>, kScanThreads);
    hipStream_t s = as_stream(stream);
    if (multi) {
        // tile size and prefetch by the 4096-element tile count (tune_scan.py
        // --spmv over the 15 benchmark shapes, profiles/spmvscan_multi_r2.log):
        // short vectors want small tiles (more blocks on the look-back chain),
        // long ones 16-B x 4 rows per lane and the next tile in flight
        if (tiles <= 64) return spmv_scan_launch<1, false, true, true>(a, xx, flags, n, iters, ws, s);
        if (tiles < 400) return spmv_scan_launch<2, false, true, true>(a, xx, flags, n, iters, ws, s);
        return tiles >= 900 ? spmv_scan_launch<4, true, true, true>(a, xx, flags, n, iters, ws, s)
                            : spmv_scan_launch<4, false, true, true>(a, xx, flags, n, iters, ws, s);
    }
    const bool pf = tiles > 2LL * device_cu_count() * bpc;
    return pf ? spmv_scan_launch<4, true, true>(a, xx, flags, n, iters, ws, s)
              : spmv_scan_launch<4, false, true>(a, xx, flags, n, iters, ws, s);
}

// Workspace bytes cme_spmv_scan_run / _tune need for n elements (one 256-B
// aligned descriptor set of the finest tiling -- 1024 elements per tile -- per
// step of a launch).
CME_EXPORT int cme_spmv_scan_ws_bytes(long long n, long long* bytes) {
    const long long tiles = (n + 1023) / 1024;
    const long long set = (long long)(lb_ws_bytes(tiles) > lb2_ws_bytes(tiles) ? lb_ws_bytes(tiles) : lb2_ws_bytes(tiles));
    *bytes = kSpmvScanSteps * ((set + 255) / 256 * 256) + 256;
    return 0;
}


// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(scan_lookback_f32, 256,
                    scan_lookback_kernel<float, true, kLbRows, true, kLbMode, false, kLbPf, kLbNt>);
CME_REGISTER_KERNEL(scan_rts_reduce_f32, 256, rts_reduce_kernel<float>);
CME_REGISTER_KERNEL(scan_rts_scan_f32, 256, rts_scan_kernel<float, true>);
CME_REGISTER_KERNEL(scan_blelloch_rts_f32, 256, tile_tree_scan_kernel<float, true, 0>);
CME_REGISTER_KERNEL(segscan_bitmask_fused, 256, segscan_kernel<1, true, 4, false, true>);
