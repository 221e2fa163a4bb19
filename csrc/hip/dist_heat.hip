// Native RCCL communicator + the distributed heat-stencil time loop.
//
// Replaces the reference's host-MPI halo exchange (hw/hw5/2dHeat_solution.cpp:
// 394-465, 501-628: MPI_Isend/Irecv per row -- or per grid ROW for column
// halos -- then MPI_Waitall) with:
//   * one ncclGroupStart/End batch of ncclSend/ncclRecv per exchange on a
//     dedicated communication stream (rows go straight out of / into the grid;
//     column halos are packed by a kernel into a contiguous staging buffer);
//   * the deep-interior sweep of step t+1 running on the compute stream while
//     the exchange of step t is in flight; the border strips wait on an event
//     recorded after the exchange -- no host synchronisation in the loop;
//   * the whole K-step loop issued from C++ (no per-step Python), RCCL
//     bootstrapped from a unique id broadcast by torch.distributed.
// torch is imported before this library is loaded, so librccl.so.1 resolves
// to the RCCL instance torch already loaded (one RCCL per process).
#include <rccl/rccl.h>

#include "cme213/common.h"

extern "C" int cme_heat_step_f32(const float* prev, float* curr, int pitch, int gy, int xb, int xe, int yb, int ye,
                                 int order, int variant, float xcfl, float ycfl, int chunk, void* stream);
extern "C" int cme_heat_step_f64(const double* prev, double* curr, int pitch, int gy, int xb, int xe, int yb, int ye,
                                 int order, int variant, double xcfl, double ycfl, int chunk, void* stream);
extern "C" int cme_heat_step2_f32(const float* prev, float* curr, int pitch, int gy, const int* out, const int* ext,
                                  int order, float xcfl, float ycfl, int chunk, int fma, void* stream);
extern "C" int cme_heat_step2_f64(const double* prev, double* curr, int pitch, int gy, const int* out, const int* ext,
                                  int order, double xcfl, double ycfl, int chunk, int fma, void* stream);

#define CME_TRY_INT(expr)                 \
    do {                                  \
        int _ri = (expr);                 \
        if (_ri) return _ri;              \
    } while (0)

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

namespace {

// Staged rectangular blocks (column halos, corner halos): rows x w elements
// at (x0, y0) <-> contiguous staging.
template <typename T>
__global__ __launch_bounds__(256) void pack_block_kernel(const T* __restrict__ g, int pitch, int x0, int y0, int ny,
                                                         int w, T* __restrict__ stage) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= ny * w) return;
    const int r = i / w, c = i % w;
    stage[i] = g[(size_t)(y0 + r) * pitch + x0 + c];
}

template <typename T>
__global__ __launch_bounds__(256) void unpack_block_kernel(T* __restrict__ g, int pitch, int x0, int y0, int ny, int w,
                                                           const T* __restrict__ stage) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= ny * w) return;
    const int r = i / w, c = i % w;
    g[(size_t)(y0 + r) * pitch + x0 + c] = stage[i];
}

struct DistCtx {
    int dev = -1;
    hipStream_t comm_stream = nullptr;
    hipEvent_t ev_compute = nullptr, ev_comm = nullptr;
};

int get_ctx(DistCtx** out) {
    static DistCtx ctx[16];
    int dev;
    CME_TRY(hipGetDevice(&dev));
    DistCtx& c = ctx[dev & 15];
    if (c.dev != dev) {
        CME_TRY(hipStreamCreateWithFlags(&c.comm_stream, hipStreamNonBlocking));
        CME_TRY(hipEventCreateWithFlags(&c.ev_compute, hipEventDisableTiming));
        CME_TRY(hipEventCreateWithFlags(&c.ev_comm, hipEventDisableTiming));
        c.dev = dev;
    }
    *out = &c;
    return 0;
}

// single step: streaming kernel, exact (variant 2) or FMA (variant 6)
template <typename T>
int step_region(const T* p, T* c, int pitch, int gy, const int* r, int order, T xcfl, T ycfl, int fma,
                hipStream_t s);

template <>
int step_region<float>(const float* p, float* c, int pitch, int gy, const int* r, int order, float xcfl, float ycfl,
                       int fma, hipStream_t s) {
    return cme_heat_step_f32(p, c, pitch, gy, r[0], r[1], r[2], r[3], order, fma ? 6 : 2, xcfl, ycfl, 0, (void*)s);
}
template <>
int step_region<double>(const double* p, double* c, int pitch, int gy, const int* r, int order, double xcfl,
                        double ycfl, int fma, hipStream_t s) {
    return cme_heat_step_f64(p, c, pitch, gy, r[0], r[1], r[2], r[3], order, fma ? 6 : 2, xcfl, ycfl, 0, (void*)s);
}

template <typename T>
int step2_region(const T* p, T* c, int pitch, int gy, const int* r, const int* ext, int order, T xcfl, T ycfl,
                 int fma, hipStream_t s);

template <>
int step2_region<float>(const float* p, float* c, int pitch, int gy, const int* r, const int* ext, int order,
                        float xcfl, float ycfl, int fma, hipStream_t s) {
    return cme_heat_step2_f32(p, c, pitch, gy, r, ext, order, xcfl, ycfl, 0, fma, (void*)s);
}
template <>
int step2_region<double>(const double* p, double* c, int pitch, int gy, const int* r, const int* ext, int order,
                         double xcfl, double ycfl, int fma, hipStream_t s) {
    return cme_heat_step2_f64(p, c, pitch, gy, r, ext, order, xcfl, ycfl, 0, fma, (void*)s);
}

// Exchange plan for buffer `g`:
//   rows[i*4 + 0..3]  = {peer, send_off, recv_off, count}  (element offsets;
//                       full pitched rows go straight out of / into the grid)
//   blks[i*7 + 0..6]  = {peer, send_x, send_y, recv_x, recv_y, rows, width}
//                       (column halos and, for 2B-deep halos, the corners
//                       to/from the diagonal peers)
//   stage: 2 * sum(rows*width) elements (send halves first, then recv halves)
constexpr int kBlk = 7;

template <typename T>
int post_exchange(ncclComm_t comm, T* g, int pitch, const long long* rows, int n_rows, const int* blks, int n_blks,
                  T* stage, ncclDataType_t dt, hipStream_t cs) {
    long long total = 0;
    for (int i = 0; i < n_blks; ++i) total += (long long)blks[i * kBlk + 5] * blks[i * kBlk + 6];
    long long off = 0;
    for (int i = 0; i < n_blks; ++i) {
        const int* c = blks + i * kBlk;
        const int cnt = c[5] * c[6];
        hipLaunchKernelGGL(pack_block_kernel<T>, dim3(cdiv(cnt, 256)), dim3(256), 0, cs, g, pitch, c[1], c[2], c[5],
                           c[6], stage + off);
        off += cnt;
    }
    CME_TRY(hipGetLastError());
    NCCL_TRY(ncclGroupStart());
    for (int i = 0; i < n_rows; ++i) {
        const long long* r = rows + i * 4;
        NCCL_TRY(ncclSend(g + r[1], (size_t)r[3], dt, (int)r[0], comm, cs));
        NCCL_TRY(ncclRecv(g + r[2], (size_t)r[3], dt, (int)r[0], comm, cs));
    }
    off = 0;
    for (int i = 0; i < n_blks; ++i) {
        const int* c = blks + i * kBlk;
        const long long cnt = (long long)c[5] * c[6];
        NCCL_TRY(ncclSend(stage + off, (size_t)cnt, dt, c[0], comm, cs));
        NCCL_TRY(ncclRecv(stage + total + off, (size_t)cnt, dt, c[0], comm, cs));
        off += cnt;
    }
    NCCL_TRY(ncclGroupEnd());
    off = 0;
    for (int i = 0; i < n_blks; ++i) {
        const int* c = blks + i * kBlk;
        const int cnt = c[5] * c[6];
        hipLaunchKernelGGL(unpack_block_kernel<T>, dim3(cdiv(cnt, 256)), dim3(256), 0, cs, g, pitch, c[3], c[4], c[5],
                           c[6], stage + total + off);
        off += cnt;
    }
    CME_TRY(hipGetLastError());
    return 0;
}

template <typename T>
int dist_run(ncclComm_t comm, T* buf0, T* buf1, int pitch, int gy, const int* interior, int n_int, const int* border,
             int n_b, const int* ext, int tblock, int fma, const long long* rows, int n_rows, const int* cols, int n_cols, T* stage, int order, T xcfl,
             T ycfl, int iters, int cur, int sync, int exchange_first, int* cur_out, hipStream_t s) {
    DistCtx* ctx;
    CME_TRY_INT(get_ctx(&ctx));
    const ncclDataType_t dt = sizeof(T) == 4 ? ncclFloat32 : ncclFloat64;
    T* bufs[2] = {buf0, buf1};
    hipStream_t cs = ctx->comm_stream;
    if (exchange_first) {  // make halos of the current state valid
        CME_TRY(hipEventRecord(ctx->ev_compute, s));
        CME_TRY(hipStreamWaitEvent(cs, ctx->ev_compute, 0));
        int rc = post_exchange<T>(comm, bufs[cur], pitch, rows, n_rows, cols, n_cols, stage, dt, cs);
        if (rc) return rc;
        CME_TRY(hipEventRecord(ctx->ev_comm, cs));
        CME_TRY(hipStreamWaitEvent(s, ctx->ev_comm, 0));
    }
    // tblock == 2: halos are 2B deep, each exchange feeds TWO timesteps computed
    // in one pass (stream2, intermediate step on region `ext`); odd tails
    // take one single step (the 2B halo over-satisfies it).
    for (int it = 0; it < iters;) {
        const T* p = bufs[cur];
        T* c = bufs[cur ^ 1];
        const bool two = tblock == 2 && it + 1 < iters;
        auto sweep = [&](const int* regs, int n) -> int {
            for (int i = 0; i < n; ++i) {
                int rc = two ? step2_region<T>(p, c, pitch, gy, regs + 4 * i, ext, order, xcfl, ycfl, fma, s)
                             : step_region<T>(p, c, pitch, gy, regs + 4 * i, order, xcfl, ycfl, fma, s);
                if (rc) return rc;
            }
            return 0;
        };
        if (sync) {
            CME_TRY_INT(sweep(interior, n_int));
            CME_TRY_INT(sweep(border, n_b));
            CME_TRY(hipEventRecord(ctx->ev_compute, s));
            CME_TRY(hipStreamWaitEvent(cs, ctx->ev_compute, 0));
            int rc = post_exchange<T>(comm, c, pitch, rows, n_rows, cols, n_cols, stage, dt, cs);
            if (rc) return rc;
            CME_TRY(hipEventRecord(ctx->ev_comm, cs));
            CME_TRY(hipStreamWaitEvent(s, ctx->ev_comm, 0));
        } else {
            // deep interior needs no ghost cells: overlaps the previous exchange
            CME_TRY_INT(sweep(interior, n_int));
            CME_TRY(hipStreamWaitEvent(s, ctx->ev_comm, 0));  // halos of p have arrived
            CME_TRY_INT(sweep(border, n_b));
            CME_TRY(hipEventRecord(ctx->ev_compute, s));
            CME_TRY(hipStreamWaitEvent(cs, ctx->ev_compute, 0));
            int rc = post_exchange<T>(comm, c, pitch, rows, n_rows, cols, n_cols, stage, dt, cs);
            if (rc) return rc;
            CME_TRY(hipEventRecord(ctx->ev_comm, cs));
        }
        cur ^= 1;
        it += two ? 2 : 1;
    }
    // leave the compute stream ordered after the last exchange
    CME_TRY(hipStreamWaitEvent(s, ctx->ev_comm, 0));
    *cur_out = cur;
    return 0;
}

}  // namespace

// The distributed heat loop (see dist_run). dtype 0 = f32, 1 = f64.
// tblock 1: one step per exchange; 2: two steps per exchange (needs 2B-deep
// halos, `interior` shrunk by 2B on neighbour sides, `ext` = owned region
// grown by B on neighbour sides). fma: FMA-contracted stencil.
CME_EXPORT int cme_heat_dist_run(void* comm, void* buf0, void* buf1, int pitch, int gy, const int* interior, int n_int,
                                 const int* border, int n_b, const int* ext, int tblock, int fma,
                                 const long long* rows, int n_rows, const int* cols,
                                 int n_cols, void* stage, int dtype, int order, double xcfl, double ycfl, int iters,
                                 int cur, int sync, int exchange_first, int* cur_out, void* stream) {
    if (dtype == 0)
        return dist_run<float>((ncclComm_t)comm, (float*)buf0, (float*)buf1, pitch, gy, interior, n_int, border, n_b,
                               ext, tblock, fma, rows, n_rows, cols, n_cols, (float*)stage, order, (float)xcfl, (float)ycfl, iters, cur,
                               sync, exchange_first, cur_out, as_stream(stream));
    return dist_run<double>((ncclComm_t)comm, (double*)buf0, (double*)buf1, pitch, gy, interior, n_int, border, n_b,
                            ext, tblock, fma, rows, n_rows, cols, n_cols, (double*)stage, order, xcfl, ycfl, iters, cur, sync,
                            exchange_first, cur_out, as_stream(stream));
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(halo_pack_f32, 256, pack_block_kernel<float>);
