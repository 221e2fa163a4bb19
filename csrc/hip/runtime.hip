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
