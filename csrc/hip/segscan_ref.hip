// The final project's own SpMV-scan algorithms, as comparison variants of the
// single-pass look-back segmented scan (scan.hip: cme_spmv_scan_run):
//
//  serial : one lane per segment, sequential scan -- fp_old.cu:28-58 (1/32
//           lanes busy in the reference; here 1 lane of 64 per segment, but
//           all lanes of a wave work on different segments).
//  wave   : one wave per segment, windows of 64 elements scanned with DPP
//           (wave_inclusive_scan) plus a carried running sum -- the
//           algorithm of fp.cu:28-59 (warp per segment, Hillis-Steele over
//           32-element windows advancing 31). The reference relies on
//           warp-synchronous global-memory writes without volatile or
//           barriers (a race outside Fermi lock-step); the DPP scan keeps
//           the window in registers so no such hazard exists.
//
// Both fuse the a *= x[k] product (xx = x[k], pre-gathered) and run `iters`
// iterations in place.
#include "cme213/common.h"
#include "cme213/wave.h"

using namespace cme;

namespace {

__global__ __launch_bounds__(256) void segscan_serial_kernel(float* __restrict__ a, const float* __restrict__ xx,
                                                             const int* __restrict__ s, int nseg) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nseg) return;
    float acc = 0.f;
    for (int l = s[i]; l < s[i + 1]; ++l) {
        acc += a[l] * xx[l];
        a[l] = acc;
    }
}

__global__ __launch_bounds__(256) void segscan_wave_kernel(float* __restrict__ a, const float* __restrict__ xx,
                                                           const int* __restrict__ s, int nseg) {
    const int lane = lane_id();
    const int wave = (blockIdx.x * 256 + threadIdx.x) / kWave;
    const int nwaves = gridDim.x * (256 / kWave);
    for (int sg = wave; sg < nseg; sg += nwaves) {
        const int b = s[sg], e = s[sg + 1];
        float carry = 0.f;
        for (int base = b; base < e; base += kWave) {
            const int l = base + lane;
            const float v = l < e ? a[l] * xx[l] : 0.f;
            const float incl = wave_inclusive_scan(v) + carry;
            if (l < e) a[l] = incl;
            carry = wave_readlane(incl, kWave - 1);
        }
    }
}

}  // namespace

// algo 0 serial, 1 wave. s: nseg + 1 offsets (s[0] = 0, s[nseg] = n).
CME_EXPORT int cme_segscan_offsets_run(float* a, const float* xx, const int* s, int nseg, int algo, int iters,
                                       void* stream) {
    hipStream_t st = as_stream(stream);
    for (int it = 0; it < iters; ++it) {
        if (algo == 0)
            hipLaunchKernelGGL(segscan_serial_kernel, dim3(cdiv(nseg, 256)), dim3(256), 0, st, a, xx, s, nseg);
        else
            hipLaunchKernelGGL(segscan_wave_kernel, dim3(stream_grid((size_t)nseg * kWave, 256)), dim3(256), 0, st,
                               a, xx, s, nseg);
        CME_TRY(hipGetLastError());
    }
    return 0;
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(segscan_serial, 256, segscan_serial_kernel);
CME_REGISTER_KERNEL(segscan_wave, 256, segscan_wave_kernel);
