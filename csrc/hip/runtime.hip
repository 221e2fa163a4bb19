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
