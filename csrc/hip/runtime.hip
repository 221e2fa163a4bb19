// Runtime helpers exported by libcme213_hip.so: error strings, device query,
// and a hipEvent-based timer pair (the reference's event_pair/start_timer/
// stop_timer, hw/hw1/programming/mp1-util.h:1-39, as a non-printing C ABI; the
// Python layer prints the "<name> took X ms" line).
#include "cme213/common.h"

CME_EXPORT const char* cme_hip_error_string(int e) { return hipGetErrorString((hipError_t)e); }

CME_EXPORT int cme_device_info(int dev, int* cus, int* lds_per_block, int* wave, long long* gmem) {
    hipDeviceProp_t p;
    CME_TRY(hipGetDeviceProperties(&p, dev));
    *cus = p.multiProcessorCount;
    *lds_per_block = (int)p.sharedMemPerBlock;
    *wave = p.warpSize;
    *gmem = (long long)p.totalGlobalMem;
    return 0;
}

CME_EXPORT int cme_sync(void* stream) { return (int)hipStreamSynchronize(as_stream(stream)); }

// Device-wide barrier + sticky-error check (CME_SYNC_CHECK debug mode).
CME_EXPORT int cme_device_sync() {
    CME_TRY(hipDeviceSynchronize());
    return (int)hipGetLastError();
}

// -------------------------------------------------------------- registry
// Resource / occupancy report for the registered kernels: the MI355X answer
// to the reference's CUDA Occupancy Calculator spreadsheet and `ptxas -v`
// (refs/CUDA_Occupancy_Calculator.xls; slides/Lecture08 slides 7-9).
#include <cstring>
#include <vector>

namespace cme {
struct KernelInfo {
    const char* name;
    const void* fn;
    int block;
};
static std::vector<KernelInfo>& kernel_registry() {
    static std::vector<KernelInfo> v;
    return v;
}
void register_kernel(const char* name, const void* fn, int block) { kernel_registry().push_back({name, fn, block}); }
}  // namespace cme

CME_EXPORT int cme_kernel_count() { return (int)cme::kernel_registry().size(); }

// out[0..7] = block, VGPRs (numRegs), static LDS bytes, scratch bytes/lane,
// max threads/block, resident blocks per CU (occupancy API), resident waves
// per SIMD, max dynamic LDS bytes.
CME_EXPORT int cme_kernel_query(int i, char* name, int name_len, int* out) {
    auto& r = cme::kernel_registry();
    if (i < 0 || i >= (int)r.size()) return (int)hipErrorInvalidValue;
    const auto& k = r[i];
    std::strncpy(name, k.name, name_len - 1);
    name[name_len - 1] = 0;
    hipFuncAttributes a;
    CME_TRY(hipFuncGetAttributes(&a, k.fn));
    int blocks = 0;
    CME_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k.fn, k.block, 0));
    out[0] = k.block;
    out[1] = a.numRegs;
    out[2] = (int)a.sharedSizeBytes;
    out[3] = (int)a.localSizeBytes;
    out[4] = a.maxThreadsPerBlock;
    out[5] = blocks;
    out[6] = blocks * (k.block / kWave) / 4;
    out[7] = a.maxDynamicSharedSizeBytes;
    return 0;
}

// ------------------------------------------------------------ tuning table
// (cme213/tuning.h). Names are the environment variables without "CME_",
// lower-cased: "pipe_vw", "dist_schedule", ...
#include <atomic>
#include <cctype>
#include <cstdlib>

#include "cme213/tuning.h"

namespace {
struct TuneEntry {
    const char* env;
    long dflt;
};
// order = cme::TuneKey
const TuneEntry kTuneTable[cme::kTuneCount] = {
    {"CME_PIPE_VW", 0},          {"CME_PIPE_CHUNK", 0},         {"CME_PIPE_PER_CU", 0},
    {"CME_PIPE_THIN_MIN", 64},   {"CME_DIST_SCHEDULE", 2},      {"CME_DIST_EVENT_SCOPE", 0},
    {"CME_DIST_VERBOSE", 0},     {"CME_DIST_GATE_SPINS", 1L << 24}, {"CME_DIST_FAKE_XCHG_US", 0},
    {"CME_RADIX_MAXBLOCKS", 1024}, {"CME_RADIX_DS", 14},          {"CME_STREAM2_CHUNK", 0},
    {"CME_STREAMN_CHUNK", 0},    {"CME_STREAMN_ROUNDS", 0},     {"CME_STREAMN_MINCHUNK", 0},
    {"CME_STREAMN_THIN_WAVES", 1024}, {"CME_STREAMN_CAPPCT", 100}, {"CME_SPMVSCAN_MULTI", 1},
    {"CME_SPMV_NT", 2},          {"CME_SPMV_DIA1", 0},          {"CME_PIPE_TAPER", 0},
    {"CME_RADIX_UP_UNR", 4},     {"CME_RADIX_OS_LANES", 1},
    {"CME_FLOW_PER_CU", 0},      {"CME_FLOW_SPINS", 1L << 22},  {"CME_FLOW_MODE", 0},
    {"CME_SPMV_STREAM_ROWS", 0},
    {"CME_TILE_RES_MINR", 1},    {"CME_SPMV_SHORT_RPT", 1},     {"CME_MERGE_PART", -1},
    {"CME_MERGE_TILE", 4096},    {"CME_MERGE_BLOCK", 0},        {"CME_MERGE_SAMPLES", 1},
    {"CME_MERGE_BLOCK_SORT", 1},
};
std::atomic<long> g_tune_val[cme::kTuneCount];
std::atomic<int> g_tune_state[cme::kTuneCount];  // 0 not loaded, 1 from env / default, 2 set

long tune_env(int k) {
    const char* e = getenv(kTuneTable[k].env);
    if (!e || !*e) return kTuneTable[k].dflt;
    if (k == cme::kTuneDistEventScope) return strcmp(e, "device") == 0 ? 1 : atol(e);
    if (k == cme::kTuneDistVerbose) return 1;
    return atol(e);
}

int tune_key(const char* name) {
    for (int k = 0; k < cme::kTuneCount; ++k) {
        const char* env = kTuneTable[k].env + 4;  // skip "CME_"
        int i = 0;
        while (env[i] && name[i] && tolower((unsigned char)env[i]) == name[i]) ++i;
        if (!env[i] && !name[i]) return k;
    }
    return -1;
}
}  // namespace

long cme::tune_get(cme::TuneKey k) {
    if (g_tune_state[k].load(std::memory_order_acquire) == 0) {
        g_tune_val[k].store(tune_env(k), std::memory_order_relaxed);
        int expect = 0;
        g_tune_state[k].compare_exchange_strong(expect, 1, std::memory_order_acq_rel);
    }
    return g_tune_val[k].load(std::memory_order_relaxed);
}

// Set a knob for this process (overrides its environment variable).
CME_EXPORT int cme_tune_set(const char* name, long long value) {
    const int k = tune_key(name);
    if (k < 0) return (int)hipErrorInvalidValue;
    g_tune_val[k].store((long)value, std::memory_order_relaxed);
    g_tune_state[k].store(2, std::memory_order_release);
    return 0;
}

// Back to the environment variable / default.
CME_EXPORT int cme_tune_reset(const char* name) {
    const int k = tune_key(name);
    if (k < 0) return (int)hipErrorInvalidValue;
    g_tune_state[k].store(0, std::memory_order_release);
    return 0;
}

// Current value; *is_set = 1 if set through cme_tune_set.
CME_EXPORT int cme_tune_get(const char* name, long long* value, int* is_set) {
    const int k = tune_key(name);
    if (k < 0) return (int)hipErrorInvalidValue;
    *value = cme::tune_get((cme::TuneKey)k);
    *is_set = g_tune_state[k].load(std::memory_order_acquire) == 2;
    return 0;
}

// Number of knobs and the i-th knob's name (for listing).
CME_EXPORT int cme_tune_name(int i, char* out, int len) {
    if (i < 0 || i >= cme::kTuneCount || len < 2) return (int)hipErrorInvalidValue;
    const char* env = kTuneTable[i].env + 4;
    int j = 0;
    for (; env[j] && j < len - 1; ++j) out[j] = (char)tolower((unsigned char)env[j]);
    out[j] = 0;
    return 0;
}
CME_EXPORT int cme_tune_count() { return cme::kTuneCount; }
