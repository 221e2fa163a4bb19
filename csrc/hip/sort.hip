// GPU sorting: LSD radix sort (8-bit digits) and merge-path merge sort.
//
// Parity: the hw4 OpenMP radix sort (hw/hw4/programming/radixsort.cpp:22-121:
// per-block histograms -> reduce -> exclusive scan -> push-down offsets ->
// per-block scatter) and merge sort (mergesort.cpp:31-144: recursive sort +
// parallel merge split at the median via upper_bound), moved to wave64.
//
// Radix pass (reduce-then-scan structure -- no in-launch hand-offs):
//   K1 upsweep  : block b histograms its contiguous chunk (LDS atomics) into
//                 counts[digit * nblocks + b]
//   K2 scan     : one block per digit scans that digit's row of counts over
//                 the blocks and writes the digit total (one small launch)
//   K3 downsweep: block b re-reads its chunk tile by tile (8192 keys); keys are
//                 ranked stably inside each wave by one returning LDS atomic
//                 per key (lanes resolve in lane order; ballot "match" on a
//                 device that fails that check), waves are combined per digit in LDS, the
//                 tile is reordered by digit in LDS and written out so that
//                 consecutive lanes store consecutive addresses of a digit run.
//                 A running per-digit base in LDS carries the chunk across tiles;
//                 the block's digit bases are the scan of the 256 digit totals
//                 (done in its prologue) plus its own row prefixes.
// int32 / float32 keys are mapped to order-preserving uint32 codes by the
// first pass's loads and back by the last pass's stores (no extra kernels).
#include "sort_kernels.h"

// blocks of the upsweep / downsweep grid: at most 1024 (4 per CU), each
// walking several 4096-key tiles -- measured on MI355X, 16M keys: 0.357 /
// 0.363 / 0.391 ms at caps 1024 / 2048 / 4096 (48M: 1.18 / 1.13 / 1.14).
// CME_RADIX_MAXBLOCKS overrides the cap (<= kMaxRadixBlocks, sweeps).
static int radix_max_blocks() {
    const long x = cme::tune_get(cme::kTuneRadixMaxBlocks);
    return x < 1 ? 1 : (x > kMaxRadixBlocks ? kMaxRadixBlocks : (int)x);
}

CME_EXPORT long long cme_radix_ws_bytes(long long n) {
    long long tiles = (n + kSortTile - 1) / kSortTile;
    long long nb = tiles < kMaxRadixBlocks ? tiles : kMaxRadixBlocks;
    return nb * kBins * 4 + kBins * 4 + 256;
}

// LSD radix sort of n keys from `in` (not modified) into `out` over bits
// [bit0, bit1), ping-ponging through `tmp` so that the last pass writes out;
// values (optional) likewise. mode: 0 uint32, 1 int32, 2 float32 keys.
// ws: cme_radix_ws_bytes(n) bytes.
// downsweep variant (CME_RADIX_DS, for A/B sweeps): bit 0 group-atomic ranks,
// bit 1 prefetch, bit 2 8192-key tiles (512 threads), bit 3 lane-order atomic
// ranks (kRankLanes; overrides bit 0). Default 14 = lane ranks + prefetch +
// 8192-key tiles (profiles/sort_r4.md, one box: 16M uint32 0.218 ms vs 0.265
// for the round-3 default 2 = ballot-match ranks + prefetch; 48M 0.684 vs
// 0.821; 16M int32 key-value 0.378 vs 0.440). With the match gone the larger
// tiles win (digit runs of ~32 keys: fewer partial lines written), where they
// lost to the barrier rounds before.
static int radix_ds_variant() { return (int)(cme::tune_get(cme::kTuneRadixDS) & 31); }

namespace {
// Lane-order check for kRankLanes: one block; every wave runs `trials`
// wave-wide returning atomics over digit patterns of 1..256 distinct values
// with masked lanes, and counts the lanes whose old value is not (running
// count + lower active lanes of the digit). Vector atomics only.
__global__ __launch_bounds__(256) void radix_lane_order_probe_kernel(int trials, unsigned* __restrict__ bad) {
    __shared__ uint32_t cnt[4][kBins];
    const int lane = lane_id(), w = threadIdx.x / kWave;
    for (int i = threadIdx.x; i < 4 * kBins; i += 256) (&cnt[0][0])[i] = 0;
    __syncthreads();
    unsigned nbad = 0;
    for (int t = 0; t < trials; ++t) {
        uint32_t h = (uint32_t)(t * 4 + w) * 0x9e3779b9u + (uint32_t)lane * 0x85ebca6bu;
        h ^= h >> 15;
        h *= 0x2c1b3c6du;
        h ^= h >> 12;
        const int ndist = 1 << (t % 9);  // 1 .. 256 distinct digits
        const uint32_t d = (h >> 8) % (uint32_t)ndist;
        const bool on = (h & 15u) != 0u;  // ~6 % masked lanes
        const uint32_t before = cnt[w][d];
        uint32_t lower = 0;
        for (int l = 0; l < kWave; ++l) {
            const uint32_t dl = (uint32_t)__shfl((int)d, l);
            const int onl = __shfl((int)on, l);
            lower += (l < lane && onl && dl == d) ? 1u : 0u;
        }
        wave_lds_sync();
        uint32_t old = 0;
        if (on) old = atomicAdd(&cnt[w][d], 1u);
        wave_lds_sync();
        nbad += (on && old != before + lower) ? 1u : 0u;
    }
    if (nbad) atomicAdd(bad, nbad);
}

std::atomic<int> g_lane_order[64];  // per device: 0 unknown, 1 lane-ordered, -1 not (or not checkable)
}  // namespace

// 1 if the device's returning LDS atomics resolve same-address lanes in lane
// order (kRankLanes is then used), 0 if not. Runs the check once per device
// (~1 ms, synchronous on a private stream); under stream capture
// an unchecked device reports 0 without checking.
CME_EXPORT int cme_radix_lane_order(int check) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    const int st = g_lane_order[dev].load();
    if (st != 0 || !check) return st > 0;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 0;
    unsigned* bad = nullptr;
    int ok = -1;
    if (hipMallocAsync((void**)&bad, 4, s) == hipSuccess) {
        unsigned hb = 1;
        if (hipMemsetAsync(bad, 0, 4, s) == hipSuccess) {
            hipLaunchKernelGGL(radix_lane_order_probe_kernel, dim3(1), dim3(256), 0, s, 9 * 48, bad);
            if (hipGetLastError() == hipSuccess &&
                hipMemcpyAsync(&hb, bad, 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
                hipStreamSynchronize(s) == hipSuccess)
                ok = hb == 0 ? 1 : -1;
        }
        (void)hipFreeAsync(bad, s);
        (void)hipStreamSynchronize(s);
    }
    (void)hipStreamDestroy(s);
    g_lane_order[dev].store(ok);
    return ok > 0;
}

CME_EXPORT int cme_radix_sort(const uint32_t* in, uint32_t* out, uint32_t* tmp, const uint32_t* vin, uint32_t* vout,
                              uint32_t* vtmp, long long n, int mode, int bit0, int bit1, void* ws, void* stream) {
    hipStream_t s = as_stream(stream);
    if (n <= 0) return 0;
    if (bit0 < 0 || bit1 > 32 || bit1 <= bit0 || mode < 0 || mode > 2 || (vin != nullptr) != (vout != nullptr) ||
        (vin && !vtmp) || n >= (1ll << 32))
        return (int)hipErrorInvalidValue;
    int dsv = radix_ds_variant();
    if (dsv & 8) {  // lane-order ranks: only on a device that passed the check
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        const bool capturing = hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
        if (!cme_radix_lane_order(capturing ? 0 : 1)) dsv &= ~8;
    }
    const bool lanes = (dsv & 8) != 0;
    const bool wide = (dsv & 4) != 0;  // 8192-key downsweep tiles
    // 16384-key tiles (bit 16: 1024 lanes, lane ranks only): digit runs of
    // ~64 keys, but one block per CU (83 KiB LDS, 82 VGPRs); measured 16M
    // 0.2195 -> 0.245-0.251 ms, 48M 0.679 -> 0.661 without prefetch
    // (raw_r6/radix_ds16k_ab_r6.jsonl) -- an arm, not the default
    const bool huge = lanes && (dsv & 16) != 0;
    const long long dtile = huge ? 4 * kSortTile : (wide ? 2 * kSortTile : kSortTile);
    const long long tiles = (n + dtile - 1) / dtile;
    const int cap = radix_max_blocks();
    int nb = tiles < cap ? (int)tiles : cap;
    const long long chunk = ((tiles + nb - 1) / nb) * dtile;
    nb = (int)((n + chunk - 1) / chunk);
    uint32_t* counts = (uint32_t*)ws;
    uint32_t* totals = counts + (size_t)nb * kBins;
    const int npass = (bit1 - bit0 + kRadixBits - 1) / kRadixBits;
    const int up_unr = (int)cme::tune_get(cme::kTuneRadixUpUnr);  // upsweep 16-B loads in flight per lane: 4, 8, 16 (-4: per-key checks)
    const uint32_t* ki = in;
    const uint32_t* vi = vin;
    for (int p = 0; p < npass; ++p) {
        const bool to_out = ((npass - 1 - p) & 1) == 0;  // the last pass lands in out
        uint32_t* ko = to_out ? out : tmp;
        uint32_t* vo = vin ? (to_out ? vout : vtmp) : nullptr;
        const int shift = bit0 + kRadixBits * p;
        const int mi = p == 0 ? mode : 0, mo = p == npass - 1 ? mode : 0;
        switch (up_unr) {
#define CME_UP(U)                                                                                                  \
    case U:                                                                                                       \
        hipLaunchKernelGGL(radix_upsweep_kernel<U>, dim3(nb), dim3(kSortThreads), 0, s, ki, n, chunk, shift, nb,     \
                           counts, mi);                                                                           \
        break;
            CME_UP(8) CME_UP(16)
#undef CME_UP
            case -4:  // the round-4 upsweep: a uniformity check per key instead of per 16-B load
                hipLaunchKernelGGL((radix_upsweep_kernel<4, false>), dim3(nb), dim3(kSortThreads), 0, s, ki, n, chunk,
                                   shift, nb, counts, mi);
                break;
            default:
                hipLaunchKernelGGL(radix_upsweep_kernel<4>, dim3(nb), dim3(kSortThreads), 0, s, ki, n, chunk, shift,
                                   nb, counts, mi);
        }
        hipLaunchKernelGGL(radix_scan_kernel, dim3(kBins), dim3(1024), 0, s, counts, nb, totals);
#define CME_DS(V, A, P)                                                                                           \
    do {                                                                                                          \
        if (huge && A == kRankLanes)                                                                              \
            hipLaunchKernelGGL((radix_downsweep_kernel<V, kRankLanes, P, 1024>), dim3(nb), dim3(1024), 0, s, ki, ko,  \
                               vi, vo, n, chunk, shift, nb, counts, totals, mi, mo);                              \
        else if (wide)                                                                                            \
            hipLaunchKernelGGL((radix_downsweep_kernel<V, A, P, 512>), dim3(nb), dim3(512), 0, s, ki, ko, vi, vo, n, \
                               chunk, shift, nb, counts, totals, mi, mo);                                         \
        else                                                                                                      \
            hipLaunchKernelGGL((radix_downsweep_kernel<V, A, P>), dim3(nb), dim3(kSortThreads), 0, s, ki, ko, vi,  \
                               vo, n, chunk, shift, nb, counts, totals, mi, mo);                                  \
    } while (0)
        // arms: 0-3 ballot-match ranks (bit 0 group atomics, bit 1 prefetch),
        // 4-5 lane ranks (without / with prefetch); `wide` picks the 512-thread
        // 8192-key tile instantiation of any arm
        const int arm = lanes ? 4 + ((dsv >> 1) & 1) : (dsv & 3);
        if (vin) {
            if (arm == 0) CME_DS(true, kRankMatch, false);
            else if (arm == 1) CME_DS(true, kRankGroup, false);
            else if (arm == 2) CME_DS(true, kRankMatch, true);
            else if (arm == 3) CME_DS(true, kRankGroup, true);
            else if (arm == 4) CME_DS(true, kRankLanes, false);
            else CME_DS(true, kRankLanes, true);
        } else {
            if (arm == 0) CME_DS(false, kRankMatch, false);
            else if (arm == 1) CME_DS(false, kRankGroup, false);
            else if (arm == 2) CME_DS(false, kRankMatch, true);
            else if (arm == 3) CME_DS(false, kRankGroup, true);
            else if (arm == 4) CME_DS(false, kRankLanes, false);
            else CME_DS(false, kRankLanes, true);
        }
#undef CME_DS
        CME_TRY(hipGetLastError());
        ki = ko;
        vi = vo;
    }
    return 0;
}

// In-place form (sorted uint32 keys left in `keys`; keys_alt / vals_alt scratch).
CME_EXPORT int cme_radix_sort_u32(uint32_t* keys, uint32_t* keys_alt, uint32_t* vals, uint32_t* vals_alt, long long n,
                                  int bit0, int bit1, void* ws, void* stream) {
    if (n <= 1) return 0;
    const int npass = (bit1 - bit0 + kRadixBits - 1) / kRadixBits;
    if (npass & 1) {  // odd: sort into keys_alt, copy back
        int rc = cme_radix_sort(keys, keys_alt, keys, vals, vals ? vals_alt : nullptr, vals, n, 0, bit0, bit1, ws,
                                stream);
        if (rc) return rc;
        CME_TRY(hipMemcpyAsync(keys, keys_alt, n * 4, hipMemcpyDeviceToDevice, as_stream(stream)));
        if (vals) CME_TRY(hipMemcpyAsync(vals, vals_alt, n * 4, hipMemcpyDeviceToDevice, as_stream(stream)));
        return 0;
    }
    return cme_radix_sort(keys, keys, keys_alt, vals, vals, vals_alt, n, 0, bit0, bit1, ws, stream);
}

// Stable merge sort of n keys from `in` into `out` (ping-pong through `tmp`;
// `in` may equal `out`; values optional, likewise). mode: 0 uint32, 1 int32,
// 2 float32 keys. The schedule is ms_sort_host in sort_kernels.h (the
// tuning library instantiates it with its 4-way pass arm).
CME_EXPORT long long cme_merge_ws_bytes(long long n) { return ms_ws_bytes(n); }

CME_EXPORT int cme_merge_sort_ws(const uint32_t* in, uint32_t* out, uint32_t* tmp, const uint32_t* vin,
                                 uint32_t* vout, uint32_t* vtmp, long long n, int mode, void* ws, void* stream) {
    return ms_sort_host<MsTwoWayOnly>(in, out, tmp, vin, vout, vtmp, n, mode, ws, stream);
}

CME_EXPORT int cme_merge_sort(const uint32_t* in, uint32_t* out, uint32_t* tmp, const uint32_t* vin, uint32_t* vout,
                              uint32_t* vtmp, long long n, int mode, void* stream) {
    return cme_merge_sort_ws(in, out, tmp, vin, vout, vtmp, n, mode, nullptr, stream);
}

// In-place form (keys sorted into `keys`; keys_alt / vals_alt scratch).
CME_EXPORT int cme_merge_sort_u32(uint32_t* keys, uint32_t* keys_alt, uint32_t* vals, uint32_t* vals_alt, long long n,
                                  void* stream) {
    return cme_merge_sort(keys, keys, keys_alt, vals, vals, vals_alt, n, 0, stream);
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(radix_upsweep, 256, radix_upsweep_kernel<4>);
CME_REGISTER_KERNEL(radix_downsweep_kv, 256, radix_downsweep_kernel<true>);
CME_REGISTER_KERNEL(ms_block_sort, 512, ms_block_sort_kernel<false>);
CME_REGISTER_KERNEL(ms_merge_pass, 256, ms_merge_pass_kernel<false>);
CME_REGISTER_KERNEL(ms_block_radix, 1024, ms_block_radix_kernel<kRankLanes>);
