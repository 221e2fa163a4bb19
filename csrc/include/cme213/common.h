// cme213x native runtime: shared definitions for the HIP (gfx950) library.
//
// Replaces the reference's per-assignment `mp1-util.h` launch checking
// (hw/hw1/programming/mp1-util.h:8-18: sync + cudaGetLastError + exit) with a
// non-fatal, graph-capturable contract: every exported launcher returns the
// hipError_t as an int and never synchronises, so the Python layer can raise a
// RuntimeError and callers can capture launches into hipGraphs.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define CME_EXPORT extern "C" __attribute__((visibility("default")))

// Kernel registry (for the occupancy / resource report, cme_kernel_query):
// every translation unit registers its main kernels with the block size it
// launches them with. Defined in runtime.hip.
namespace cme {
void register_kernel(const char* name, const void* fn, int block);
}
#define CME_REGISTER_KERNEL(tag, block, ...) \
    static const int cme_reg_##tag = (::cme::register_kernel(#tag, reinterpret_cast<const void*>(&__VA_ARGS__), block), 0)

// Wave64 is the CDNA execution quantum; never assume 32.
constexpr int kWave = 64;
// MI355X: 256 CUs in 8 XCDs.
constexpr int kNumCU = 256;
constexpr int kNumXCD = 8;

#define CME_TRY(expr)                                  \
    do {                                               \
        hipError_t _e = (expr);                        \
        if (_e != hipSuccess) return (int)_e;          \
    } while (0)

// Return the launch status without synchronising (check_launch replacement).
#define CME_LAUNCH_STATUS() return (int)hipGetLastError()

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline unsigned cdiv(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

// Grid size for grid-stride memory-bound kernels: enough blocks to fill all
// 256 CUs several times over, capped so the tail stays short.
static inline unsigned stream_grid(size_t work_items, unsigned block, unsigned blocks_per_cu = 8) {
    size_t want = (work_items + block - 1) / block;
    size_t cap = (size_t)kNumCU * blocks_per_cu;
    if (want > cap) want = cap;
    if (want < 1) want = 1;
    return (unsigned)want;
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 "XCD swizzle must
// be bijective"): blocks b and b+8 share an XCD under round-robin dispatch, so
// give each XCD group a contiguous range of logical tiles. Speed only, never
// correctness.
__device__ __forceinline__ unsigned xcd_remap(unsigned bid, unsigned nwg) {
    const unsigned xcd = bid % kNumXCD;
    const unsigned q = nwg / kNumXCD, r = nwg % kNumXCD;
    const unsigned base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + bid / kNumXCD;
}

// CUs of the CURRENT device, cached per device: a partitioned MI355X
// (CPX/DPX modes) or another gfx950 part exposes fewer than 256, so grids
// that must be co-resident are sized from this, never from kNumCU.
static inline int device_cu_count() {
    static int cached[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return kNumCU;
    int& c = cached[dev & 63];
    if (c == 0) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = kNumCU;
        c = v;
    }
    return c;
}

// Waves of `kernel` (launched with `threads` per block) the device holds at
// once: occupancy-API blocks per CU x CUs x waves per block.
template <typename K>
static inline long resident_waves(K kernel, int threads) {
    int api = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&api, kernel, threads, 0) != hipSuccess || api < 1) api = 1;
    return (long)api * device_cu_count() * ((threads + kWave - 1) / kWave);
}

// Co-resident grid for a persistent kernel: min(occupancy API - 1, cap)
// blocks per CU (the API can over-report by one block per CU on gfx950 for
// SGPR-heavy kernels -- MI355X_MICROARCH.md "Residency"), at least 1.
template <typename K>
static inline int persistent_blocks_per_cu(K kernel, int threads, int cap = 4) {
    int api = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&api, kernel, threads, 0) != hipSuccess) api = 2;
    int b = api - 1;
    if (b > cap) b = cap;
    if (b < 1) b = 1;
    return b;
}

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & (kWave - 1)); }
