// Native communicators + the distributed heat-stencil time loop.
//
// Replaces the reference's host-MPI halo exchange (hw/hw5/2dHeat_solution.cpp:
// 394-465, 501-628: MPI_Isend/Irecv per row -- or per grid ROW for column
// halos -- then MPI_Waitall) with one exchange PLAN per subdomain and three
// interchangeable transports that all execute it the same way:
//
//   pack   : the column / corner blocks this subdomain sends are gathered by
//            ONE kernel into the send half of a contiguous staging buffer
//            (rows are contiguous in the grid and travel straight from it);
//   move   : 0 RCCL   -- one ncclGroupStart/End batch of ncclSend/ncclRecv;
//            1 loopback -- every neighbour lives in this process: one
//              multi-segment copy kernel PULLS the neighbours' rows (grid)
//              and blocks (their staging) into our grid / staging;
//            3 IPC    -- every neighbour is another process (same GPU or a
//              peer over xGMI): its grid and staging are mapped with
//              hipIpcOpenMemHandle and the same copy kernel pulls from them,
//              ordered by epoch flags in peer-visible memory (below);
//            2 none   -- no exchange (benchmarks the compute schedule);
//   unpack : ONE kernel scatters the receive half of the staging into the
//            ghost columns / corners.
// So the loopback and IPC tests execute the exact pack / stage layout /
// unpack code the RCCL transport runs -- only the "move" differs.
//
// Schedule (dist_run): the deep-interior sweep of pass i+1 runs on the compute
// stream while the exchange of pass i is in flight on the comm stream; the
// border strips wait on an event recorded after the exchange -- no host
// synchronisation in the K-step loop, which is issued entirely from C++.
//
// torch is imported before this library is loaded, so librccl.so.1 resolves
// to the RCCL instance torch already loaded (one RCCL per process).
#include <rccl/rccl.h>
#include <string.h>

#include <map>
#include <mutex>
#include <string>

#include "cme213/common.h"
#include "cme213/tuning.h"
#include "cme213/heat_region.h"

extern "C" int cme_heat_step_f32(const float* prev, float* curr, int pitch, int gy, int xb, int xe, int yb, int ye,
                                 int order, int variant, float xcfl, float ycfl, int chunk, void* stream);
extern "C" int cme_heat_step_f64(const double* prev, double* curr, int pitch, int gy, int xb, int xe, int yb, int ye,
                                 int order, int variant, double xcfl, double ycfl, int chunk, void* stream);
extern "C" int cme_heat_stepn_f32(const float* prev, float* curr, int pitch, int gy, const int* out, int nout,
                                  const int* ext, int order, int nsteps, float xcfl, float ycfl, int chunk, int fma,
                                  void* stream);
extern "C" int cme_heat_pipe_f32(const float* prev, float* curr, int pitch, int gy, const int* out, int nout,
                                 const int* ext, int order, int nsteps, float xcfl, float ycfl, int chunk, int fma,
                                 void* stream);
extern "C" int cme_heat_pipe_gated_f32(const float* prev, float* curr, int pitch, int gy, const int* out, int nout,
                                       const int* ext, int order, int nsteps, float xcfl, float ycfl, int fma,
                                       int wait_from, const unsigned* flag, unsigned value, unsigned* timeout,
                                       void* stream);
extern "C" int cme_heat_pipe_f64(const double* prev, double* curr, int pitch, int gy, const int* out, int nout,
                                 const int* ext, int order, int nsteps, double xcfl, double ycfl, int chunk, int fma,
                                 void* stream);
extern "C" int cme_heat_pipe_gated_f64(const double* prev, double* curr, int pitch, int gy, const int* out, int nout,
                                       const int* ext, int order, int nsteps, double xcfl, double ycfl, int fma,
                                       int wait_from, const unsigned* flag, unsigned value, unsigned* timeout,
                                       void* stream);
extern "C" int cme_heat_stepn_f64(const double* prev, double* curr, int pitch, int gy, const int* out, int nout,
                                  const int* ext, int order, int nsteps, double xcfl, double ycfl, int chunk, int fma,
                                  void* stream);
// heat_fast.hip: reassociated arithmetic (fp32, order 8 for the passes)
extern "C" int cme_heat_step_fast_f32(const float* prev, float* curr, int pitch, int gy, int xb, int xe, int yb,
                                      int ye, int order, float xcfl, float ycfl, void* stream);
extern "C" int cme_heat_pipe_fast_f32(const float* prev, float* curr, int pitch, int gy, const int* out, int nout,
                                      const int* ext, int order, int nsteps, float xcfl, float ycfl, int chunk,
                                      int wait_from, const unsigned* flag, unsigned value, unsigned* timeout,
                                      void* stream);

#define CME_TRY_INT(expr)                 \
    do {                                  \
        int _ri = (expr);                 \
        if (_ri) return _ri;              \
    } while (0)

// RCCL status codes are returned as 10000 + ncclResult_t so the Python layer
// can tell them from hipError_t (decoded with cme_rccl_error_string).
#define NCCL_TRY(expr)                                        \
    do {                                                      \
        ncclResult_t _r = (expr);                             \
        if (_r != ncclSuccess) return 10000 + (int)_r;        \
    } while (0)

CME_EXPORT int cme_rccl_unique_id(char* out128) {
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    static_assert(sizeof(id) == 128, "ncclUniqueId size");
    for (int i = 0; i < 128; ++i) out128[i] = id.internal[i];
    return 0;
}

CME_EXPORT int cme_rccl_init(void** comm, int nranks, const void* id128, int rank) {
    ncclUniqueId id;
    for (int i = 0; i < 128; ++i) id.internal[i] = ((const char*)id128)[i];
    ncclComm_t c;
    NCCL_TRY(ncclCommInitRank(&c, nranks, id, rank));
    *comm = (void*)c;
    return 0;
}

// Failure detection: poll the communicator's asynchronous error state (a
// peer died, a network/xGMI error) and abort it so pending collectives return
// instead of hanging (SURVEY §5 "communicator-abort path").
CME_EXPORT int cme_rccl_async_error(void* comm, int* err) {
    ncclResult_t r;
    NCCL_TRY(ncclCommGetAsyncError((ncclComm_t)comm, &r));
    *err = (int)r;
    return 0;
}

CME_EXPORT int cme_rccl_abort(void* comm) {
    NCCL_TRY(ncclCommAbort((ncclComm_t)comm));
    return 0;
}

CME_EXPORT int cme_rccl_destroy(void* comm) {
    NCCL_TRY(ncclCommDestroy((ncclComm_t)comm));
    return 0;
}

CME_EXPORT const char* cme_rccl_error_string(int code) {
    return code >= 10000 ? ncclGetErrorString((ncclResult_t)(code - 10000)) : "";
}

// dtype: 0 f32, 1 f64, 2 i32, 3 i64, 4 u8
static ncclDataType_t nccl_type(int dtype) {
    switch (dtype) {
        case 0: return ncclFloat32;
        case 1: return ncclFloat64;
        case 2: return ncclInt32;
        case 3: return ncclInt64;
        default: return ncclUint8;
    }
}

// op: 0 sum, 1 max, 2 min, 3 prod
static ncclRedOp_t nccl_op(int op) {
    switch (op) {
        case 1: return ncclMax;
        case 2: return ncclMin;
        case 3: return ncclProd;
        default: return ncclSum;
    }
}

CME_EXPORT int cme_rccl_allreduce(void* comm, const void* send, void* recv, long long count, int dtype, int op,
                                  void* stream) {
    NCCL_TRY(ncclAllReduce(send, recv, (size_t)count, nccl_type(dtype), nccl_op(op), (ncclComm_t)comm,
                           as_stream(stream)));
    return 0;
}

CME_EXPORT int cme_rccl_allgather(void* comm, const void* send, void* recv, long long count, int dtype, void* stream) {
    NCCL_TRY(ncclAllGather(send, recv, (size_t)count, nccl_type(dtype), (ncclComm_t)comm, as_stream(stream)));
    return 0;
}

// Grouped point-to-point: n entries of {peer, is_send, ptr, count}.
CME_EXPORT int cme_rccl_p2p(void* comm, int n, const int* peers, const int* is_send, void* const* ptrs,
                            const long long* counts, int dtype, void* stream) {
    NCCL_TRY(ncclGroupStart());
    for (int i = 0; i < n; ++i) {
        if (is_send[i])
            NCCL_TRY(ncclSend(ptrs[i], (size_t)counts[i], nccl_type(dtype), peers[i], (ncclComm_t)comm,
                              as_stream(stream)));
        else
            NCCL_TRY(ncclRecv(ptrs[i], (size_t)counts[i], nccl_type(dtype), peers[i], (ncclComm_t)comm,
                              as_stream(stream)));
    }
    NCCL_TRY(ncclGroupEnd());
    return 0;
}

// ------------------------------------------------------------ IPC memory
// Export / import device allocations between processes (SURVEY §2.6
// IpcPeerComm). Handles are always taken on the allocation BASE (found with
// hipMemGetAddressRange), the interior offset travels separately, so a tensor
// carved out of a caching-allocator segment maps correctly. Imports are
// reference-counted per handle: a process maps each peer segment once even
// when several tensors (grid, staging, flags) live in it.
namespace {
struct IpcImport {
    void* base = nullptr;
    int refs = 0;
};
std::mutex g_ipc_mu;
std::map<std::string, IpcImport> g_ipc_imports;
}  // namespace

CME_EXPORT int cme_ipc_export(const void* ptr, void* handle64, long long* offset) {
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    CME_TRY(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr));
    hipIpcMemHandle_t h;
    CME_TRY(hipIpcGetMemHandle(&h, (void*)base));
    memcpy(handle64, &h, sizeof(h));
    *offset = (long long)((const char*)ptr - (const char*)base);
    return 0;
}

CME_EXPORT int cme_ipc_open(const void* handle64, void** base) {
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    std::string key((const char*)handle64, sizeof(hipIpcMemHandle_t));
    IpcImport& imp = g_ipc_imports[key];
    if (imp.refs == 0) {
        hipIpcMemHandle_t h;
        memcpy(&h, handle64, sizeof(h));
        void* p = nullptr;
        hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
            g_ipc_imports.erase(key);
            return (int)e;
        }
        imp.base = p;
    }
    ++imp.refs;
    *base = imp.base;
    return 0;
}

CME_EXPORT int cme_ipc_close(void* base) {
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    for (auto it = g_ipc_imports.begin(); it != g_ipc_imports.end(); ++it) {
        if (it->second.base != base) continue;
        if (--it->second.refs == 0) {
            void* p = it->second.base;
            g_ipc_imports.erase(it);
            CME_TRY(hipIpcCloseMemHandle(p));
        }
        return 0;
    }
    return (int)hipErrorInvalidValue;
}

namespace {

// ------------------------------------------------------------ exchange kernels
constexpr int kMaxPieces = 8;  // column halos (2) + corner blocks (4) per subdomain
constexpr int kMaxSegs = 16;   // rows (2) + blocks (6) per pull

// A list of staged rectangular blocks: piece p is rows[p] x width[p]
// elements at (x[p], y[p]) of the grid <-> stage + off[p].
struct BlkList {
    int x[kMaxPieces], y[kMaxPieces], rows[kMaxPieces], width[kMaxPieces];
    long long off[kMaxPieces];
    int n;
};

// One launch packs (grid -> stage) or unpacks (stage -> grid) every piece:
// blockIdx.y = piece, grid-stride over its elements.
template <typename T, bool kPack>
__global__ __launch_bounds__(256) void blocks_kernel(T* __restrict__ g, int pitch, T* __restrict__ stage,
                                                     BlkList l) {
    const int p = blockIdx.y;
    if (p >= l.n) return;
    const int w = l.width[p], cnt = l.rows[p] * w;
    T* st = stage + l.off[p];
    for (int i = blockIdx.x * 256 + threadIdx.x; i < cnt; i += gridDim.x * 256) {
        const int r = i / w, c = i - r * w;
        T* gp = g + (size_t)(l.y[p] + r) * pitch + l.x[p] + c;
        if (kPack)
            st[i] = *gp;
        else
            *gp = st[i];
    }
}

// Multi-segment device copy (the "move" of the loopback and IPC transports):
// blockIdx.y = segment; 16-B lanes when the segment allows, 4-B otherwise
// (every element type is 4- or 8-B, so 4-B granules always tile a segment).
struct CopyList {
    const void* src[kMaxSegs];
    void* dst[kMaxSegs];
    long long bytes[kMaxSegs];
    int n;
};

template <bool kSysAcquire>
__global__ __launch_bounds__(256) void multi_copy_kernel(CopyList l) {
    const int s = blockIdx.y;
    if (s >= l.n) return;
    if constexpr (kSysAcquire) {
        // IPC pull: peer memory (over xGMI) may sit in this XCD's L2 from an
        // earlier pass; a system-scope acquire drops those lines before the
        // loads (one lane fences, the barrier holds the block behind it).
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
    }
    const char* src = (const char*)l.src[s];
    char* dst = (char*)l.dst[s];
    const long long nb = l.bytes[s];
    const long long tid = (long long)blockIdx.x * 256 + threadIdx.x, stride = (long long)gridDim.x * 256;
    if ((((uintptr_t)src | (uintptr_t)dst | (uintptr_t)nb) & 15) == 0) {
        const uint4* s4 = (const uint4*)src;
        uint4* d4 = (uint4*)dst;
        for (long long i = tid; i < nb / 16; i += stride) d4[i] = s4[i];
    } else {
        const unsigned* s1 = (const unsigned*)src;
        unsigned* d1 = (unsigned*)dst;
        for (long long i = tid; i < nb / 4; i += stride) d1[i] = s1[i];
    }
}

int launch_copies(const CopyList& l, hipStream_t s, bool sys_acquire = false) {
    if (l.n == 0) return 0;
    long long mx = 0;
    for (int i = 0; i < l.n; ++i) mx = l.bytes[i] > mx ? l.bytes[i] : mx;
    unsigned gx = cdiv((size_t)(mx / 16 + 1), 256);
    if (gx > 64) gx = 64;
    if (sys_acquire)
        hipLaunchKernelGGL(multi_copy_kernel<true>, dim3(gx, l.n), dim3(256), 0, s, l);
    else
        hipLaunchKernelGGL(multi_copy_kernel<false>, dim3(gx, l.n), dim3(256), 0, s, l);
    CME_TRY(hipGetLastError());
    return 0;
}

// ---------------------------------------------------- cross-process epochs
// Pass e of the IPC transport is ordered across processes by 32-bit epoch
// words in device memory every peer maps:
//   flags[0]      = e   : "my blocks of pass e are packed, my rows written"
//   flags[1 + j]  = e   : "neighbour j has pulled pass e from me"
// A signal kernel stores them (system-scope atomic stores, written through to
// memory: a plain store behind a fence is never seen by another XCD -- see
// cdna_hip_programming.md §6 G16); a one-wave wait kernel polls them with
// relaxed system-scope loads and s_sleep, bounded: a peer that never signals
// sets the sticky timeout word instead of hanging the GPU, and every later
// wait returns at once. Payload visibility needs no in-kernel fences: the
// producing kernels have ENDED (end-of-kernel release) before the signal
// kernel runs, and the consuming copy kernel starts (dispatch acquire) after
// the wait kernel has seen the epoch.
constexpr int kMaxPeers = 8;
constexpr unsigned kSpinLimit = 1u << 23;  // x (poll + ~0.2 us sleep): seconds, not forever

struct FlagList {
    unsigned* f[kMaxPeers + 1];
    int n;
};

__global__ __launch_bounds__(64) void ipc_signal_kernel(FlagList l, unsigned value) {
    const int i = threadIdx.x;
    if (i < l.n) __hip_atomic_store(l.f[i], value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void ipc_wait_kernel(FlagList l, unsigned value, unsigned* timeout) {
    const int i = threadIdx.x;
    if (i >= l.n) return;
    if (__hip_atomic_load(timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return;  // sticky
    for (unsigned spins = 0;; ++spins) {
        const unsigned v = __hip_atomic_load(l.f[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((int)(v - value) >= 0) break;  // wrap-safe "v >= value"
        if (spins >= kSpinLimit) {
            __hip_atomic_store(timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
        __builtin_amdgcn_s_sleep(16);
    }
}

// Rehearsal only (transport 2 with CME_DIST_FAKE_XCHG_US > 0): stands in for
// the network part of an exchange on the comm stream -- one wave that holds
// the stream for a fixed wall-clock time, between the real pack and unpack
// kernels -- so the border -> exchange -> border chain of an N-GPU run can be
// timed on one GPU (benchmarks/bench_dist_rank.py --fake-xchg-us).
__global__ __launch_bounds__(64) void delay_kernel(unsigned long long ticks) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

int launch_delay_us(int us, hipStream_t s) {
    static const long long khz = [] {
        int dev = 0, rate = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, dev) != hipSuccess || rate <= 0)
            rate = 100000;  // 100 MHz
        return (long long)rate;
    }();
    hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, s, (unsigned long long)(khz * us / 1000));
    CME_TRY(hipGetLastError());
    return 0;
}

int launch_signal(const FlagList& l, unsigned v, hipStream_t s) {
    if (l.n == 0) return 0;
    hipLaunchKernelGGL(ipc_signal_kernel, dim3(1), dim3(64), 0, s, l, v);
    CME_TRY(hipGetLastError());
    return 0;
}

int launch_wait(const FlagList& l, unsigned v, unsigned* timeout, hipStream_t s) {
    if (l.n == 0) return 0;
    hipLaunchKernelGGL(ipc_wait_kernel, dim3(1), dim3(64), 0, s, l, v, timeout);
    CME_TRY(hipGetLastError());
    return 0;
}

// bit 3 of the flags word: reassociated ("fast") arithmetic, fp32 order 8
// (heat_fast.hip: the wide-lane pipelined pass with FMA arm 5 for 2-4 step
// passes, a plain kernel for single steps)
constexpr int kArithFast = 8;

// single step: streaming kernel, exact (variant 2) or FMA (variant 6), or the
// reassociated kernel
template <typename T>
int step_region(const T* p, T* c, int pitch, int gy, const int* r, int order, T xcfl, T ycfl, int fma,
                hipStream_t s);

template <>
int step_region<float>(const float* p, float* c, int pitch, int gy, const int* r, int order, float xcfl, float ycfl,
                       int fma, hipStream_t s) {
    if (fma & kArithFast)
        return cme_heat_step_fast_f32(p, c, pitch, gy, r[0], r[1], r[2], r[3], order, xcfl, ycfl, (void*)s);
    return cme_heat_step_f32(p, c, pitch, gy, r[0], r[1], r[2], r[3], order, (fma & 1) ? 6 : 2, xcfl, ycfl, 0,
                             (void*)s);
}
template <>
int step_region<double>(const double* p, double* c, int pitch, int gy, const int* r, int order, double xcfl,
                        double ycfl, int fma, hipStream_t s) {
    return cme_heat_step_f64(p, c, pitch, gy, r[0], r[1], r[2], r[3], order, (fma & 1) ? 6 : 2, xcfl, ycfl, 0,
                             (void*)s);
}

// ns-step pass (ns = 2..4) over n (<= 4) regions in one launch. `fma` bit 0:
// FMA-contracted stencil; bit 1 (kKernelPipe): 3-4 step fp32 passes run the
// wave-pipelined kernel (heat_pipe.hip) instead of streamN -- same bits.
constexpr int kKernelPipe = 2;
// bit 2 of the same flags word (cme_heat_dist_run only): never use the fused
// schedule in this call (schedule 0 instead) -- the caller's fallback
constexpr int kNoFused = 4;
template <typename T>
int stepn_regions(const T* p, T* c, int pitch, int gy, const int* r, int n, const int* ext, int order, int ns,
                  T xcfl, T ycfl, int fma, hipStream_t s);

template <>
int stepn_regions<float>(const float* p, float* c, int pitch, int gy, const int* r, int n, const int* ext, int order,
                         int ns, float xcfl, float ycfl, int fma, hipStream_t s) {
    if (fma & kArithFast)
        return cme_heat_pipe_fast_f32(p, c, pitch, gy, r, n, ext, order, ns, xcfl, ycfl, 0, 0, nullptr, 0u, nullptr,
                                      (void*)s);
    if ((fma & kKernelPipe) && ns >= 3)
        return cme_heat_pipe_f32(p, c, pitch, gy, r, n, ext, order, ns, xcfl, ycfl, 0, fma & 1, (void*)s);
    return cme_heat_stepn_f32(p, c, pitch, gy, r, n, ext, order, ns, xcfl, ycfl, 0, fma & 1, (void*)s);
}
template <>
int stepn_regions<double>(const double* p, double* c, int pitch, int gy, const int* r, int n, const int* ext,
                          int order, int ns, double xcfl, double ycfl, int fma, hipStream_t s) {
    if ((fma & kKernelPipe) && ns >= 3)
        return cme_heat_pipe_f64(p, c, pitch, gy, r, n, ext, order, ns, xcfl, ycfl, 0, fma & 1, (void*)s);
    return cme_heat_stepn_f64(p, c, pitch, gy, r, n, ext, order, ns, xcfl, ycfl, 0, fma & 1, (void*)s);
}

// fused-schedule pass: every region in one pipelined launch, regions
// [wait_from, n) gated on *flag >= value
template <typename T>
int gated_pass(const T* p, T* c, int pitch, int gy, const int* r, int n, const int* ext, int order, int ns, T xcfl,
               T ycfl, int fma, int wait_from, const unsigned* flag, unsigned value, unsigned* timeout,
               hipStream_t s) {
    if constexpr (sizeof(T) == 4) {
        if (fma & kArithFast)
            return cme_heat_pipe_fast_f32(p, c, pitch, gy, r, n, ext, order, ns, xcfl, ycfl, 0, wait_from, flag, value,
                                          timeout, (void*)s);
        return cme_heat_pipe_gated_f32(p, c, pitch, gy, r, n, ext, order, ns, xcfl, ycfl, fma & 1, wait_from, flag,
                                       value, timeout, (void*)s);
    }
    else
        return cme_heat_pipe_gated_f64(p, c, pitch, gy, r, n, ext, order, ns, xcfl, ycfl, fma & 1, wait_from, flag,
                                       value, timeout, (void*)s);
}

// Queue-independence probe of the fused schedule. Its border workgroups spin
// INSIDE the compute stream's kernel until the comm stream's signal kernel
// runs; that is only safe if the two streams sit on different hardware
// queues (with GPU_MAX_HW_QUEUES or a stream count that makes HIP share a
// queue, the signal would wait behind the spinning kernel). One wave on the
// compute stream spins (bounded: ~2 s) on a fresh device word that a signal
// kernel on the comm stream sets; it reports 1 (seen) or 2 (gave up). The
// bound is generous because other processes sharing the GPU can delay the
// signal kernel's dispatch for a time slice: a shorter bound (~0.2 s) gave a
// false "shared queue" verdict once in the 8-processes-on-one-GPU test; a
// true shared queue costs the full bound once, then the events schedule runs.
__global__ __launch_bounds__(64) void gate_probe_kernel(const unsigned* flag, unsigned value, unsigned* result) {
    if (threadIdx.x != 0) return;
    unsigned r = 2u;
    for (unsigned spins = 0; spins < (1u << 23); ++spins) {
        const unsigned v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((int)(v - value) >= 0) {
            r = 1u;
            break;
        }
        __builtin_amdgcn_s_sleep(8);
    }
    __hip_atomic_store(result, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------- distributed loop
// IPC view of one neighbouring process (layout mirrored by IpcPeerDesc in
// models/heat2d_dist.py).
struct IpcPeerDesc {
    void* buf[2];     // its grid states, mapped into this process
    void* stage;      // its staging buffer (the send half is what we pull)
    unsigned* flags;  // its epoch words
    int rank;         // its global rank
    int slot;         // our index among ITS neighbours (its flags[1 + slot])
};

struct IpcPlan {
    unsigned* flags;          // ours: [0] ready epoch, [1 + j] consumed by our neighbour j
    unsigned* timeout;        // ours: sticky give-up word of the wait kernels
    long long* epoch;         // host: passes exchanged so far (persists across calls)
    const long long* row_src; // per rows[i]: the peer's send offset (elements of its grid state)
    const long long* blk_src; // per blks[i]: the peer's staging offset of the block it sends us
    int npeer;
    IpcPeerDesc peer[kMaxPeers];
};

// One descriptor per subdomain owned by this process (1 with RCCL / IPC; any
// number with the loopback transport, where every neighbour lives in this
// process). Layout must match SubDesc in models/heat2d_dist.py.
struct SubDesc {
    void* buf[2];
    int pitch, gy;
    const int* interior;  // n_int x {xb, xe, yb, ye}
    int n_int;
    const int* border;    // n_b x {xb, xe, yb, ye}
    int n_b;
    const int* ext;       // {xb, xe, yb, ye} intermediate-step region of multi-step passes
    const long long* rows;  // n_rows x {peer, send_off, recv_off, count} (elements)
    int n_rows;
    const int* blks;      // n_blks x {peer, send_x, send_y, recv_x, recv_y, rows, width}
    int n_blks;
    void* stage;          // 2 * sum(rows*width) elements: send half, then receive half
    int rank;             // global rank of this subdomain
    const IpcPlan* ipc;   // transport 3 only
};

constexpr int kBlk = 7;
constexpr int kMaxSubs = 64;

// staging offsets of the blocks (send half; the receive half adds `total`)
long long stage_layout(const SubDesc& d, long long* off) {
    long long t = 0;
    for (int i = 0; i < d.n_blks; ++i) {
        off[i] = t;
        t += (long long)d.blks[i * kBlk + 5] * d.blks[i * kBlk + 6];
    }
    return t;
}

template <typename T>
int pack_blocks(const SubDesc& d, T* g, hipStream_t s) {
    if (d.n_blks == 0) return 0;
    if (d.n_blks > kMaxPieces) return (int)hipErrorInvalidValue;
    BlkList l;
    l.n = d.n_blks;
    long long off[kMaxPieces];
    stage_layout(d, off);
    int mx = 0;
    for (int i = 0; i < d.n_blks; ++i) {
        const int* c = d.blks + i * kBlk;
        l.x[i] = c[1], l.y[i] = c[2], l.rows[i] = c[5], l.width[i] = c[6], l.off[i] = off[i];
        mx = c[5] * c[6] > mx ? c[5] * c[6] : mx;
    }
    hipLaunchKernelGGL((blocks_kernel<T, true>), dim3(cdiv(mx, 256) < 32 ? cdiv(mx, 256) : 32, l.n), dim3(256), 0,
                       s, g, d.pitch, (T*)d.stage, l);
    CME_TRY(hipGetLastError());
    return 0;
}

template <typename T>
int unpack_blocks(const SubDesc& d, T* g, hipStream_t s) {
    if (d.n_blks == 0) return 0;
    if (d.n_blks > kMaxPieces) return (int)hipErrorInvalidValue;
    BlkList l;
    l.n = d.n_blks;
    long long off[kMaxPieces];
    const long long total = stage_layout(d, off);
    int mx = 0;
    for (int i = 0; i < d.n_blks; ++i) {
        const int* c = d.blks + i * kBlk;
        l.x[i] = c[3], l.y[i] = c[4], l.rows[i] = c[5], l.width[i] = c[6], l.off[i] = total + off[i];
        mx = c[5] * c[6] > mx ? c[5] * c[6] : mx;
    }
    hipLaunchKernelGGL((blocks_kernel<T, false>), dim3(cdiv(mx, 256) < 32 ? cdiv(mx, 256) : 32, l.n), dim3(256), 0,
                       s, g, d.pitch, (T*)d.stage, l);
    CME_TRY(hipGetLastError());
    return 0;
}

// Per-subdomain streams and events. Events for border / interior completion
// are double-buffered by pass parity so that a pass can wait on the PREVIOUS
// pass's record while this pass's record is already enqueued.
struct SubCtx {
    hipStream_t compute = nullptr, border = nullptr, comm = nullptr;
    hipEvent_t ev_border[2] = {nullptr, nullptr}, ev_int[2] = {nullptr, nullptr}, ev_comm = nullptr;
    hipEvent_t ev_start = nullptr, ev_pack = nullptr;
    // fused schedule: the comm stream signals xflag = ++xposted after each
    // exchange; the next pass's border workgroups wait for it in-kernel
    unsigned* xflag = nullptr;     // device word
    unsigned xposted = 0;          // last value signalled (host mirror)
    unsigned* xtimeout = nullptr;  // pinned host word: a gated wait gave up
    // queue-independence probe (gate_probe_kernel): 0 not run, 1 passed,
    // -1 failed (compute and comm share a hardware queue: no fused schedule)
    int probe = 0;
    unsigned* probe_word = nullptr;    // device word the comm stream signals
    unsigned* probe_result = nullptr;  // pinned host word the probe writes
};

struct DistCtx {
    int dev = -1;
    int nsub = 0;
    int last_schedule = -1;  // schedule the last dist_run used (cme_heat_dist_info)
    SubCtx sub[kMaxSubs];
};

int get_ctx(int nsub, DistCtx** out) {
    static DistCtx ctx[16];
    int dev;
    CME_TRY(hipGetDevice(&dev));
    DistCtx& c = ctx[dev & 15];
    if (c.dev != dev) {
        c.dev = dev;
        c.nsub = 0;
    }
    for (int i = c.nsub; i < nsub; ++i) {  // grow lazily, never shrink
        SubCtx& u = c.sub[i];
        // border strips and the exchange are on the critical path: their
        // workgroups are dispatched ahead of the (long) interior kernel's
        int least = 0, greatest = 0;
        CME_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
        CME_TRY(hipStreamCreateWithFlags(&u.compute, hipStreamNonBlocking));
        CME_TRY(hipStreamCreateWithPriority(&u.border, hipStreamNonBlocking, greatest));
        CME_TRY(hipStreamCreateWithPriority(&u.comm, hipStreamNonBlocking, greatest));
        // The events only order streams of THIS device, so a device-scope
        // release would do; measured on one N=8 subdomain (profiles/
        // dist_rank_r2.md) the default system-scope record is no slower
        // (0.0321-0.0322 vs 0.0334-0.0338 ms/step), so it stays the default.
        // CME_DIST_EVENT_SCOPE=device selects hipEventReleaseToDevice.
        const unsigned evf = cme::tune_get(cme::kTuneDistEventScope) == 1
                                 ? (unsigned)(hipEventDisableTiming | hipEventReleaseToDevice)
                                 : (unsigned)hipEventDisableTiming;
        for (int k = 0; k < 2; ++k) {
            CME_TRY(hipEventCreateWithFlags(&u.ev_border[k], evf));
            CME_TRY(hipEventCreateWithFlags(&u.ev_int[k], evf));
        }
        CME_TRY(hipEventCreateWithFlags(&u.ev_comm, evf));
        CME_TRY(hipEventCreateWithFlags(&u.ev_start, evf));
        CME_TRY(hipEventCreateWithFlags(&u.ev_pack, evf));
        CME_TRY(hipMalloc(&u.xflag, sizeof(unsigned)));
        CME_TRY(hipMemset(u.xflag, 0, sizeof(unsigned)));
        CME_TRY(hipHostMalloc(&u.xtimeout, sizeof(unsigned), hipHostMallocMapped));
        *u.xtimeout = 0u;
        u.xposted = 0;
        CME_TRY(hipMalloc(&u.probe_word, sizeof(unsigned)));
        CME_TRY(hipMemset(u.probe_word, 0, sizeof(unsigned)));
        CME_TRY(hipHostMalloc(&u.probe_result, sizeof(unsigned), hipHostMallocMapped));
        *u.probe_result = 0u;
    }
    if (nsub > c.nsub) c.nsub = nsub;
    *out = &c;
    return 0;
}

// RCCL transport: pack -> one grouped send/recv batch -> unpack, all on the
// sub's comm stream.
template <typename T>
int post_exchange_rccl(ncclComm_t comm, const SubDesc& d, T* g, ncclDataType_t dt, hipStream_t cs) {
    T* stage = (T*)d.stage;
    long long off[kMaxPieces];
    if (d.n_blks > kMaxPieces) return (int)hipErrorInvalidValue;
    const long long total = stage_layout(d, off);
    CME_TRY_INT(pack_blocks<T>(d, g, cs));
    // Sends in plan order, receives in REVERSE plan order (rows, then
    // blocks). The plan lists rows top, bottom and blocks left, corners,
    // right -- piece i and piece n-1-i of a group face opposite ways -- so a
    // peer's k-th send to us meets our k-th receive from it even when one
    // peer sits on several sides (periodic grids; with one block per axis
    // that peer is this rank itself, and RCCL moves the bytes as self-sends).
    NCCL_TRY(ncclGroupStart());
    for (int i = 0; i < d.n_rows; ++i) {
        const long long* r = d.rows + i * 4;
        NCCL_TRY(ncclSend(g + r[1], (size_t)r[3], dt, (int)r[0], comm, cs));
    }
    for (int i = 0; i < d.n_blks; ++i) {
        const int* c = d.blks + i * kBlk;
        NCCL_TRY(ncclSend(stage + off[i], (size_t)((long long)c[5] * c[6]), dt, c[0], comm, cs));
    }
    for (int i = d.n_rows - 1; i >= 0; --i) {
        const long long* r = d.rows + i * 4;
        NCCL_TRY(ncclRecv(g + r[2], (size_t)r[3], dt, (int)r[0], comm, cs));
    }
    for (int i = d.n_blks - 1; i >= 0; --i) {
        const int* c = d.blks + i * kBlk;
        NCCL_TRY(ncclRecv(stage + total + off[i], (size_t)((long long)c[5] * c[6]), dt, c[0], comm, cs));
    }
    NCCL_TRY(ncclGroupEnd());
    return unpack_blocks<T>(d, g, cs);
}

int find_sub(const SubDesc* subs, int nsub, int rank) {
    for (int i = 0; i < nsub; ++i)
        if (subs[i].rank == rank) return i;
    return -1;
}

// The RCCL transport's matching, for the transports that pull: our piece i
// (of n, peer at stride*j) is the k-th receive from that peer in reverse
// order, k = pieces after i with the same peer; it reads the peer's k-th
// piece toward `me` in forward order. Returns that index, or -1.
template <typename I>
int recv_match(const I* mine, int n, int i, const I* theirs, int tn, int stride, int me) {
    const I peer = mine[i * stride];
    int k = 0;
    for (int j = i + 1; j < n; ++j) k += mine[j * stride] == peer;
    for (int j = 0; j < tn; ++j)
        if (theirs[j * stride] == (I)me && k-- == 0) return j;
    return -1;
}

// Loopback "move": pull every row of sub si (state k) straight from the
// owning neighbour's grid and every block from the neighbour's staging (which
// that neighbour packed on its own comm stream -- the caller orders this after
// every peer's ev_pack).
template <typename T>
int pull_loopback(const SubDesc* subs, int nsub, int si, int k, hipStream_t cs) {
    const SubDesc& d = subs[si];
    T* g = (T*)d.buf[k];
    CopyList l;
    l.n = 0;
    for (int i = 0; i < d.n_rows; ++i) {
        const long long* r = d.rows + i * 4;
        const int pj = find_sub(subs, nsub, (int)r[0]);
        if (pj < 0 || l.n >= kMaxSegs) return (int)hipErrorInvalidValue;
        const SubDesc& pd = subs[pj];
        const int m = recv_match<long long>(d.rows, d.n_rows, i, pd.rows, pd.n_rows, 4, d.rank);
        if (m < 0 || pd.rows[m * 4 + 3] != r[3]) return (int)hipErrorInvalidValue;
        l.src[l.n] = (const T*)pd.buf[k] + pd.rows[m * 4 + 1];
        l.dst[l.n] = g + r[2];
        l.bytes[l.n++] = r[3] * (long long)sizeof(T);
    }
    long long off[kMaxPieces], poff[kMaxPieces];
    if (d.n_blks > kMaxPieces) return (int)hipErrorInvalidValue;
    const long long total = stage_layout(d, off);
    for (int i = 0; i < d.n_blks; ++i) {
        const int* c = d.blks + i * kBlk;
        const int pj = find_sub(subs, nsub, c[0]);
        if (pj < 0 || l.n >= kMaxSegs) return (int)hipErrorInvalidValue;
        const SubDesc& pd = subs[pj];
        if (pd.n_blks > kMaxPieces) return (int)hipErrorInvalidValue;
        stage_layout(pd, poff);
        const int m = recv_match<int>(d.blks, d.n_blks, i, pd.blks, pd.n_blks, kBlk, d.rank);
        if (m < 0 || pd.blks[m * kBlk + 5] != c[5] || pd.blks[m * kBlk + 6] != c[6]) return (int)hipErrorInvalidValue;
        l.src[l.n] = (const T*)pd.stage + poff[m];
        l.dst[l.n] = (T*)d.stage + total + off[i];
        l.bytes[l.n++] = (long long)c[5] * c[6] * (long long)sizeof(T);
    }
    return launch_copies(l, cs);
}

// IPC transport, pass epoch e, entirely on the sub's comm stream:
//   wait  our flags[1..] >= e-1  every neighbour has pulled pass e-1 (our
//                                staging may be rewritten)
//   pack  our blocks             -> staging send half
//   signal our flags[0] = e      rows (written by the border sweep the comm
//                                stream already waited for) + blocks ready
//   wait  every peer's flags[0] >= e
//   pull  rows from peers' grids, blocks from peers' staging
//   signal peer.flags[1 + slot] = e  (we are done reading them)
//   unpack
// Rows we send are re-written two passes later by our border sweep, which is
// ordered after this exchange's first wait of the NEXT pass (e+1 waits
// consumed >= e) through the border stream's wait on our ev_comm.
template <typename T>
int post_exchange_ipc(const SubDesc& d, int k, unsigned e, hipStream_t cs) {
    const IpcPlan* P = d.ipc;
    if (!P || P->npeer > kMaxPeers) return (int)hipErrorInvalidValue;
    T* g = (T*)d.buf[k];
    FlagList mine, ready, done, own_ready;
    mine.n = ready.n = done.n = 0;
    own_ready.n = 1;
    own_ready.f[0] = P->flags;
    for (int j = 0; j < P->npeer; ++j) {
        mine.f[mine.n++] = P->flags + 1 + j;
        ready.f[ready.n++] = P->peer[j].flags;
        done.f[done.n++] = P->peer[j].flags + 1 + P->peer[j].slot;
    }
    if (e > 1) CME_TRY_INT(launch_wait(mine, e - 1, P->timeout, cs));
    CME_TRY_INT(pack_blocks<T>(d, g, cs));
    CME_TRY_INT(launch_signal(own_ready, e, cs));
    CME_TRY_INT(launch_wait(ready, e, P->timeout, cs));
    auto peer_of = [&](int rank) -> int {
        for (int j = 0; j < P->npeer; ++j)
            if (P->peer[j].rank == rank) return j;
        return -1;
    };
    CopyList l;
    l.n = 0;
    for (int i = 0; i < d.n_rows; ++i) {
        const long long* r = d.rows + i * 4;
        const int j = peer_of((int)r[0]);
        if (j < 0 || l.n >= kMaxSegs) return (int)hipErrorInvalidValue;
        l.src[l.n] = (const T*)P->peer[j].buf[k] + P->row_src[i];
        l.dst[l.n] = g + r[2];
        l.bytes[l.n++] = r[3] * (long long)sizeof(T);
    }
    long long off[kMaxPieces];
    if (d.n_blks > kMaxPieces) return (int)hipErrorInvalidValue;
    const long long total = stage_layout(d, off);
    for (int i = 0; i < d.n_blks; ++i) {
        const int* c = d.blks + i * kBlk;
        const int j = peer_of(c[0]);
        if (j < 0 || l.n >= kMaxSegs) return (int)hipErrorInvalidValue;
        l.src[l.n] = (const T*)P->peer[j].stage + P->blk_src[i];
        l.dst[l.n] = (T*)d.stage + total + off[i];
        l.bytes[l.n++] = (long long)c[5] * c[6] * (long long)sizeof(T);
    }
    CME_TRY_INT(launch_copies(l, cs, true));
    CME_TRY_INT(launch_signal(done, e, cs));
    return unpack_blocks<T>(d, g, cs);
}

// peers of sub si that live in this process (loopback dependencies)
int local_peers(const SubDesc* subs, int nsub, int si, int* out) {
    int n = 0;
    const SubDesc& d = subs[si];
    for (int i = 0; i < d.n_rows; ++i) {
        const int pj = find_sub(subs, nsub, (int)d.rows[i * 4]);
        if (pj >= 0) out[n++] = pj;
    }
    for (int i = 0; i < d.n_blks; ++i) {
        const int pj = find_sub(subs, nsub, d.blks[i * kBlk]);
        if (pj >= 0) out[n++] = pj;
    }
    return n;
}

// Run the queue-independence probe once per subdomain context (synchronises
// the compute and comm streams, so it runs before this call queues anything;
// never under stream capture). Returns 0 and sets u.probe.
int run_gate_probe(SubCtx& u) {
    if (u.probe != 0) return 0;
    const bool verbose = cme::tune_get(cme::kTuneDistVerbose) != 0;
    *u.probe_result = 0u;
    CME_TRY(hipMemsetAsync(u.probe_word, 0, sizeof(unsigned), u.compute));
    CME_TRY(hipStreamSynchronize(u.compute));
    hipLaunchKernelGGL(gate_probe_kernel, dim3(1), dim3(64), 0, u.compute, (const unsigned*)u.probe_word, 1u,
                       u.probe_result);
    CME_TRY(hipGetLastError());
    FlagList fl;
    fl.n = 1;
    fl.f[0] = u.probe_word;
    CME_TRY_INT(launch_signal(fl, 1u, u.comm));
    CME_TRY(hipStreamSynchronize(u.comm));
    CME_TRY(hipStreamSynchronize(u.compute));
    u.probe = (*u.probe_result == 1u) ? 1 : -1;
    if (u.probe < 0 || verbose)
        fprintf(stderr, "cme213x dist_run: compute/comm queue probe %s%s\n", u.probe > 0 ? "passed" : "FAILED",
                u.probe > 0 ? "" : " (streams share a hardware queue): fused schedule disabled, using schedule 0");
    return 0;
}

// The time loop. Per pass i (1..tblock timesteps), for every sub:
//   border stream : wait halos of p (own comm event, + pulling neighbours'
//                   in loopback) and the previous interior; border strips;
//                   record ev_border[i&1]
//   comm stream   : wait ev_border[i&1] (+ neighbours' in loopback); post the
//                   halo exchange of c; record ev_comm
//   compute stream: wait the previous pass's ev_border; deep interior;
//                   record ev_int[i&1]
// so the interior of pass i overlaps both the border strips and the halo
// exchange of pass i. Sync mode runs everything in order on one stream.
template <typename T>
int dist_run(int transport, ncclComm_t comm, const SubDesc* subs, int nsub, int order, T xcfl, T ycfl, int iters,
             int cur, int sync, int exchange_first, int tblock, int fma, int* cur_out, hipStream_t s) {
    if (nsub < 1 || nsub > kMaxSubs) return (int)hipErrorInvalidValue;
    if ((transport == 0 || transport == 3) && nsub != 1) return (int)hipErrorInvalidValue;
    if (transport < 0 || transport > 3) return (int)hipErrorInvalidValue;
    // Stream capture is refused: the fused schedule's gate target
    // and the IPC epochs are host counters baked into kernel arguments, so a
    // replay would see stale flags as already reached; and instantiating a
    // capture of the multi-stream event schedule crashes this image's HIP
    // runtime in capture_end (profiles/dist_rank_r2.md). The loop is issued
    // from C++ with no host synchronisation, so there is little to gain.
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    CME_TRY(hipStreamIsCapturing(s, &cap));
    if (cap != hipStreamCaptureStatusNone) return (int)hipErrorStreamCaptureUnsupported;
    if (transport == 3 && (!subs[0].ipc || !subs[0].ipc->epoch)) return (int)hipErrorInvalidValue;
    if (tblock < 1 || tblock > 4 || (tblock > 3 && sizeof(T) != 4 && !(fma & kKernelPipe)))
        return (int)hipErrorInvalidValue;
    if ((fma & kArithFast) && (sizeof(T) != 4 || order != 8)) return (int)hipErrorInvalidValue;
    // 2 (default, see `fused` below) where it applies, else 0: border stream
    // || interior stream; 1: border then interior on one stream. Measured on one N=8-rank subdomain (bench_dist_rank.py,
    // null transport): 0.041 vs 0.045 ms/step -- kept as a switch for
    // re-measuring on other topologies.
    const int schedule = (int)cme::tune_get(cme::kTuneDistSchedule);
    // 2 (fused): ONE pipelined launch per pass holding the deep interior and
    // the border strips; the border workgroups (last in the grid) wait
    // in-kernel for the previous exchange's flag, so the compute queue never
    // waits on another queue (each such cross-queue wait cost ~14 us per
    // pass at N = 8, profiles/dist_fused_r2.md). Pipelined passes (fp32 or
    // fp64), one subdomain per process, and only when
    //  * the caller did not ask for schedule 0 (kNoFused bit of `fma`),
    //  * the queue-independence probe passed (run_gate_probe).
    // Other configurations use schedule 0.
    bool fused = schedule == 2 && !(fma & kNoFused) && !sync && nsub == 1 && (fma & kKernelPipe) &&
                 tblock >= 3 && subs[0].n_int + subs[0].n_b <= cme::kMaxS2Regions && subs[0].n_int >= 1;
    DistCtx* ctx;
    CME_TRY_INT(get_ctx(nsub, &ctx));
    if (fused) {
        CME_TRY_INT(run_gate_probe(ctx->sub[0]));
        fused = ctx->sub[0].probe > 0;
    }
    ctx->last_schedule = fused ? 2 : (sync ? 3 : (schedule == 1 ? 1 : 0));
    const ncclDataType_t dt = sizeof(T) == 4 ? ncclFloat32 : ncclFloat64;
    int peers[kMaxSubs][16];
    int npeer[kMaxSubs];
    for (int si = 0; si < nsub; ++si) {
        if (subs[si].n_rows + subs[si].n_blks > 16) return (int)hipErrorInvalidValue;
        npeer[si] = local_peers(subs, nsub, si, peers[si]);
        if (transport == 1 && npeer[si] != subs[si].n_rows + subs[si].n_blks) return (int)hipErrorInvalidValue;
    }
    long long epoch = (transport == 3) ? *subs[0].ipc->epoch : 0;
    // CME_DIST_FAKE_XCHG_US (read per call): transport 2 stands a delay in
    // for the network between real pack / unpack kernels (rehearsal timing,
    // benchmarks/bench_dist_rank.py); the other transports hold their comm
    // stream that long before each exchange (a test forces the fused gate's
    // timeout path this way)
    const int fake_us = (int)cme::tune_get(cme::kTuneDistFakeXchgUs);
    // Exchange the halos of state k for every sub. The caller has made each
    // comm stream wait for what the exchange reads; ev_comm is recorded after.
    auto exchange_all = [&](int k) -> int {
        if (transport != 2 && fake_us > 0)
            for (int si = 0; si < nsub; ++si) CME_TRY_INT(launch_delay_us(fake_us, ctx->sub[si].comm));
        if (transport == 0)
            return post_exchange_rccl<T>(comm, subs[0], (T*)subs[0].buf[k], dt, ctx->sub[0].comm);
        if (transport == 3) return post_exchange_ipc<T>(subs[0], k, (unsigned)(++epoch), ctx->sub[0].comm);
        if (transport == 2) {
            if (fake_us <= 0) return 0;
            for (int si = 0; si < nsub; ++si) {  // pack -> "network" -> unpack, as transport 0
                SubCtx& u = ctx->sub[si];
                CME_TRY_INT(pack_blocks<T>(subs[si], (T*)subs[si].buf[k], u.comm));
                CME_TRY_INT(launch_delay_us(fake_us, u.comm));
                CME_TRY_INT(unpack_blocks<T>(subs[si], (T*)subs[si].buf[k], u.comm));
            }
            return 0;
        }
        for (int si = 0; si < nsub; ++si) {  // loopback: pack everything, then pull
            CME_TRY_INT(pack_blocks<T>(subs[si], (T*)subs[si].buf[k], ctx->sub[si].comm));
            CME_TRY(hipEventRecord(ctx->sub[si].ev_pack, ctx->sub[si].comm));
        }
        for (int si = 0; si < nsub; ++si) {
            SubCtx& u = ctx->sub[si];
            for (int j = 0; j < npeer[si]; ++j)
                CME_TRY(hipStreamWaitEvent(u.comm, ctx->sub[peers[si][j]].ev_pack, 0));
            CME_TRY_INT(pull_loopback<T>(subs, nsub, si, k, u.comm));
            CME_TRY_INT(unpack_blocks<T>(subs[si], (T*)subs[si].buf[k], u.comm));
        }
        return 0;
    };
    auto sweep = [&](int si, const int* regs, int n, int k, int ns, hipStream_t st) -> int {
        const SubDesc& d = subs[si];
        const T* p = (const T*)d.buf[k];
        T* c = (T*)d.buf[k ^ 1];
        if (n == 0) return 0;
        if (ns > 1)  // all regions (e.g. the 2-4 border strips) in ONE launch
            return stepn_regions<T>(p, c, d.pitch, d.gy, regs, n, d.ext, order, ns, xcfl, ycfl, fma, st);
        for (int i = 0; i < n; ++i) {
            int rc = step_region<T>(p, c, d.pitch, d.gy, regs + 4 * i, order, xcfl, ycfl, fma, st);
            if (rc) return rc;
        }
        return 0;
    };
    // all work starts after what is already queued on the caller's stream
    for (int si = 0; si < nsub; ++si) {
        SubCtx& u = ctx->sub[si];
        CME_TRY(hipEventRecord(u.ev_start, s));
        CME_TRY(hipStreamWaitEvent(u.compute, u.ev_start, 0));
        CME_TRY(hipStreamWaitEvent(u.border, u.ev_start, 0));
        CME_TRY(hipStreamWaitEvent(u.comm, u.ev_start, 0));
    }
    // Events recorded by THIS call. Everything an earlier call queued is
    // already ordered before ev_start (the caller's stream joined all of it),
    // so waits on events of earlier calls are skipped as redundant.
    bool comm_rec = false, int_rec[2] = {false, false}, border_rec[2] = {false, false};
    auto wait_if = [&](hipStream_t st, hipEvent_t ev, bool rec) -> int {
        if (rec) CME_TRY(hipStreamWaitEvent(st, ev, 0));
        return 0;
    };
    if (exchange_first) {  // make the halos of the current state valid
        CME_TRY_INT(exchange_all(cur));
        for (int si = 0; si < nsub; ++si) CME_TRY(hipEventRecord(ctx->sub[si].ev_comm, ctx->sub[si].comm));
        comm_rec = true;
        for (int si = 0; si < nsub; ++si)
            for (int j = 0; j < nsub; ++j) CME_TRY(hipStreamWaitEvent(ctx->sub[si].compute, ctx->sub[j].ev_comm, 0));
    }
    // comm streams wait this pass's border strips (own + local neighbours'),
    // then the exchange of the state those strips completed
    auto post_comm = [&](int par, int k) -> int {
        for (int si = 0; si < nsub; ++si) {
            SubCtx& u = ctx->sub[si];
            CME_TRY(hipStreamWaitEvent(u.comm, u.ev_border[par], 0));
            for (int j = 0; j < npeer[si]; ++j)
                CME_TRY(hipStreamWaitEvent(u.comm, ctx->sub[peers[si][j]].ev_border[par], 0));
        }
        CME_TRY_INT(exchange_all(k));
        for (int si = 0; si < nsub; ++si) CME_TRY(hipEventRecord(ctx->sub[si].ev_comm, ctx->sub[si].comm));
        comm_rec = true;
        return 0;
    };
    int pass = 0;
    for (int it = 0; it < iters; ++pass) {
        // timesteps in this pass: tblock, or what is left (a tail pass of
        // fewer steps reuses the tblock*B-deep halos and regions)
        const int ns = (iters - it) < tblock ? (iters - it) : tblock;
        const int par = pass & 1;
        if (fused) {
            SubCtx& u = ctx->sub[0];
            const SubDesc& d = subs[0];
            if (ns >= 3) {  // deep interior first (no wait), border strips gated on the last exchange
                int regs[4 * cme::kMaxS2Regions];
                for (int i = 0; i < 4 * d.n_int; ++i) regs[i] = d.interior[i];
                for (int i = 0; i < 4 * d.n_b; ++i) regs[4 * d.n_int + i] = d.border[i];
                CME_TRY_INT(gated_pass<T>((const T*)d.buf[cur], (T*)d.buf[cur ^ 1], d.pitch, d.gy, regs,
                                          d.n_int + d.n_b, d.ext, order, ns, xcfl, ycfl, fma, d.n_int, u.xflag,
                                          u.xposted, u.xtimeout, u.compute));
            } else {  // tail pass on the non-pipelined kernels: plain stream order
                CME_TRY_INT(wait_if(u.compute, u.ev_comm, comm_rec));
                CME_TRY_INT(sweep(0, d.interior, d.n_int, cur, ns, u.compute));
                CME_TRY_INT(sweep(0, d.border, d.n_b, cur, ns, u.compute));
            }
            CME_TRY(hipEventRecord(u.ev_int[par], u.compute));
            int_rec[par] = true;
            CME_TRY(hipStreamWaitEvent(u.comm, u.ev_int[par], 0));
            CME_TRY_INT(exchange_all(cur ^ 1));
            FlagList fl;
            fl.n = 1;
            fl.f[0] = u.xflag;
            CME_TRY_INT(launch_signal(fl, ++u.xposted, u.comm));
            CME_TRY(hipEventRecord(u.ev_comm, u.comm));
            comm_rec = true;
        } else if (sync) {
            for (int si = 0; si < nsub; ++si) {
                SubCtx& u = ctx->sub[si];
                CME_TRY_INT(sweep(si, subs[si].interior, subs[si].n_int, cur, ns, u.compute));
                CME_TRY_INT(sweep(si, subs[si].border, subs[si].n_b, cur, ns, u.compute));
                CME_TRY(hipEventRecord(u.ev_border[par], u.compute));
            }
            border_rec[par] = true;
            CME_TRY_INT(post_comm(par, cur ^ 1));
            for (int si = 0; si < nsub; ++si) {
                SubCtx& u = ctx->sub[si];
                CME_TRY(hipStreamWaitEvent(u.compute, u.ev_comm, 0));
                for (int j = 0; j < npeer[si]; ++j)
                    CME_TRY(hipStreamWaitEvent(u.compute, ctx->sub[peers[si][j]].ev_comm, 0));
            }
        } else if (schedule == 1) {
            // single compute stream: [halos of p] -> border strips -> interior;
            // the exchange of the new borders overlaps the interior
            for (int si = 0; si < nsub; ++si) {
                SubCtx& u = ctx->sub[si];
                CME_TRY_INT(wait_if(u.compute, u.ev_comm, comm_rec));
                for (int j = 0; j < npeer[si]; ++j)
                    CME_TRY_INT(wait_if(u.compute, ctx->sub[peers[si][j]].ev_comm, comm_rec));
                CME_TRY_INT(sweep(si, subs[si].border, subs[si].n_b, cur, ns, u.compute));
                CME_TRY(hipEventRecord(u.ev_border[par], u.compute));
            }
            border_rec[par] = true;
            CME_TRY_INT(post_comm(par, cur ^ 1));
            for (int si = 0; si < nsub; ++si) {
                SubCtx& u = ctx->sub[si];
                CME_TRY_INT(sweep(si, subs[si].interior, subs[si].n_int, cur, ns, u.compute));
                CME_TRY(hipEventRecord(u.ev_int[par], u.compute));
            }
            int_rec[par] = true;
        } else {
            for (int si = 0; si < nsub; ++si) {  // border strips of pass i
                SubCtx& u = ctx->sub[si];
                CME_TRY_INT(wait_if(u.border, u.ev_comm, comm_rec));
                for (int j = 0; j < npeer[si]; ++j)
                    CME_TRY_INT(wait_if(u.border, ctx->sub[peers[si][j]].ev_comm, comm_rec));
                CME_TRY_INT(wait_if(u.border, u.ev_int[par ^ 1], int_rec[par ^ 1]));
                CME_TRY_INT(sweep(si, subs[si].border, subs[si].n_b, cur, ns, u.border));
                CME_TRY(hipEventRecord(u.ev_border[par], u.border));
            }
            border_rec[par] = true;
            CME_TRY_INT(post_comm(par, cur ^ 1));  // halo exchange of the new state
            for (int si = 0; si < nsub; ++si) {  // deep interior, overlapping both
                SubCtx& u = ctx->sub[si];
                CME_TRY_INT(wait_if(u.compute, u.ev_border[par ^ 1], border_rec[par ^ 1]));
                CME_TRY_INT(sweep(si, subs[si].interior, subs[si].n_int, cur, ns, u.compute));
                CME_TRY(hipEventRecord(u.ev_int[par], u.compute));
            }
            int_rec[par] = true;
        }
        cur ^= 1;
        it += ns;
    }
    // the caller's stream resumes after every stream of every sub
    for (int si = 0; si < nsub; ++si) {
        SubCtx& u = ctx->sub[si];
        CME_TRY(hipEventRecord(u.ev_int[0], u.compute));
        CME_TRY(hipEventRecord(u.ev_border[0], u.border));
        CME_TRY(hipStreamWaitEvent(s, u.ev_int[0], 0));
        CME_TRY(hipStreamWaitEvent(s, u.ev_border[0], 0));
        if (!comm_rec) CME_TRY(hipEventRecord(u.ev_comm, u.comm));  // join the comm stream in any case
        CME_TRY(hipStreamWaitEvent(s, u.ev_comm, 0));
    }
    if (transport == 3) *subs[0].ipc->epoch = epoch;
    *cur_out = cur;
    return 0;
}

}  // namespace

// The distributed heat loop (see dist_run). transport 0 = RCCL (`comm`, one
// sub), 1 = loopback (every neighbour is one of `subs`), 2 = none (halos are
// not exchanged; benchmarks/bench_dist_rank.py), 3 = IPC (one sub per
// process, neighbours' memory mapped through SubDesc.ipc). dtype 0 f32, 1 f64.
// tblock n (1-4): n steps per exchange (nB-deep halos, `interior` shrunk by
// nB on neighbour sides, `ext` = owned region grown by (n-1)B on neighbour
// sides; 4 fp32 only). fma bit 0: FMA-contracted stencil; bit 1: 3-4 step
// fp32 passes on the wave-pipelined kernel (kKernelPipe).
CME_EXPORT int cme_heat_dist_run(int transport, void* comm, const void* subs, int nsub, int dtype, int order,
                                 double xcfl, double ycfl, int iters, int cur, int sync, int exchange_first,
                                 int tblock, int fma, int* cur_out, void* stream) {
    const SubDesc* sd = (const SubDesc*)subs;
    if (dtype == 0)
        return dist_run<float>(transport, (ncclComm_t)comm, sd, nsub, order, (float)xcfl, (float)ycfl, iters, cur,
                               sync, exchange_first, tblock, fma, cur_out, as_stream(stream));
    return dist_run<double>(transport, (ncclComm_t)comm, sd, nsub, order, xcfl, ycfl, iters, cur, sync,
                            exchange_first, tblock, fma, cur_out, as_stream(stream));
}

// Which schedule the last cme_heat_dist_run on this device used: 0 streams +
// events, 1 one compute stream, 2 fused (gated one-launch passes), 3 sync;
// -1 before any run. probe: the fused schedule's queue-independence probe of
// subdomain 0 (0 not run, 1 passed, -1 failed).
CME_EXPORT int cme_heat_dist_info(int* schedule, int* probe) {
    DistCtx* ctx;
    CME_TRY_INT(get_ctx(0, &ctx));
    *schedule = ctx->last_schedule;
    *probe = ctx->nsub > 0 ? ctx->sub[0].probe : 0;
    return 0;
}

// Fused-schedule health: *timed_out = 1 if a gated border wait of the native
// loop on this device gave up since the last call (the state is then
// invalid); clears the words. Synchronises the device first.
CME_EXPORT int cme_heat_dist_gate_status(int* timed_out) {
    *timed_out = 0;
    DistCtx* ctx;
    CME_TRY_INT(get_ctx(0, &ctx));
    CME_TRY(hipDeviceSynchronize());
    for (int i = 0; i < ctx->nsub; ++i) {
        if (ctx->sub[i].xtimeout && *ctx->sub[i].xtimeout) *timed_out = 1;
        if (ctx->sub[i].xtimeout) *ctx->sub[i].xtimeout = 0u;
    }
    return 0;
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(halo_pack_f32, 256, blocks_kernel<float, true>);
CME_REGISTER_KERNEL(halo_copy, 256, multi_copy_kernel<false>);
CME_REGISTER_KERNEL(ipc_wait, 64, ipc_wait_kernel);

// ABI check for the ctypes mirrors in models/heat2d_dist.py (tests/test_protos.py):
// {sizeof SubDesc, offsetof SubDesc.ipc, sizeof IpcPeerDesc, sizeof IpcPlan, offsetof IpcPlan.peer}
CME_EXPORT int cme_dist_abi(long long* out) {
    out[0] = (long long)sizeof(SubDesc);
    out[1] = (long long)offsetof(SubDesc, ipc);
    out[2] = (long long)sizeof(IpcPeerDesc);
    out[3] = (long long)sizeof(IpcPlan);
    out[4] = (long long)offsetof(IpcPlan, peer);
    return 0;
}
