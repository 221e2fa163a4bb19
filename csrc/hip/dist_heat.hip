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
extern "C" int cme_heat_stepn_f32(const float* prev, float* curr, int pitch, int gy, const int* out, int nout,
                                  const int* ext, int order, int nsteps, float xcfl, float ycfl, int chunk, int fma,
                                  void* stream);
extern "C" int cme_heat_stepn_f64(const double* prev, double* curr, int pitch, int gy, const int* out, int nout,
                                  const int* ext, int order, int nsteps, double xcfl, double ycfl, int chunk, int fma,
                                  void* stream);

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

// ns-step pass (ns = 2..4) over n (<= 4) regions in one launch
template <typename T>
int stepn_regions(const T* p, T* c, int pitch, int gy, const int* r, int n, const int* ext, int order, int ns,
                  T xcfl, T ycfl, int fma, hipStream_t s);

template <>
int stepn_regions<float>(const float* p, float* c, int pitch, int gy, const int* r, int n, const int* ext, int order,
                         int ns, float xcfl, float ycfl, int fma, hipStream_t s) {
    return cme_heat_stepn_f32(p, c, pitch, gy, r, n, ext, order, ns, xcfl, ycfl, 0, fma, (void*)s);
}
template <>
int stepn_regions<double>(const double* p, double* c, int pitch, int gy, const int* r, int n, const int* ext,
                          int order, int ns, double xcfl, double ycfl, int fma, hipStream_t s) {
    return cme_heat_stepn_f64(p, c, pitch, gy, r, n, ext, order, ns, xcfl, ycfl, 0, fma, (void*)s);
}

// ------------------------------------------------------------- distributed loop
// One descriptor per subdomain owned by this process (1 with RCCL; any number
// with the loopback transport, where every neighbour lives in this process).
// Layout must match SubDesc in models/heat2d_dist.py.
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
    void* stage;          // RCCL transport: 2 * sum(rows*width) elements
    int rank;             // global rank of this subdomain
};

constexpr int kBlk = 7;
constexpr int kMaxSubs = 64;

// Per-subdomain streams and events. Events for border / interior completion
// are double-buffered by pass parity so that a pass can wait on the PREVIOUS
// pass's record while this pass's record is already enqueued.
struct SubCtx {
    hipStream_t compute = nullptr, border = nullptr, comm = nullptr;
    hipEvent_t ev_border[2] = {nullptr, nullptr}, ev_int[2] = {nullptr, nullptr}, ev_comm = nullptr;
    hipEvent_t ev_start = nullptr;
};

struct DistCtx {
    int dev = -1;
    int nsub = 0;
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
        for (int k = 0; k < 2; ++k) {
            CME_TRY(hipEventCreateWithFlags(&u.ev_border[k], hipEventDisableTiming));
            CME_TRY(hipEventCreateWithFlags(&u.ev_int[k], hipEventDisableTiming));
        }
        CME_TRY(hipEventCreateWithFlags(&u.ev_comm, hipEventDisableTiming));
        CME_TRY(hipEventCreateWithFlags(&u.ev_start, hipEventDisableTiming));
    }
    if (nsub > c.nsub) c.nsub = nsub;
    *out = &c;
    return 0;
}

// RCCL transport: one grouped send/recv batch on the sub's comm stream.
// Staged blocks are packed into `stage` first and unpacked after the group.
template <typename T>
int post_exchange_rccl(ncclComm_t comm, const SubDesc& d, T* g, ncclDataType_t dt, hipStream_t cs) {
    T* stage = (T*)d.stage;
    long long total = 0;
    for (int i = 0; i < d.n_blks; ++i) total += (long long)d.blks[i * kBlk + 5] * d.blks[i * kBlk + 6];
    long long off = 0;
    for (int i = 0; i < d.n_blks; ++i) {
        const int* c = d.blks + i * kBlk;
        const int cnt = c[5] * c[6];
        hipLaunchKernelGGL(pack_block_kernel<T>, dim3(cdiv(cnt, 256)), dim3(256), 0, cs, g, d.pitch, c[1], c[2], c[5],
                           c[6], stage + off);
        off += cnt;
    }
    CME_TRY(hipGetLastError());
    NCCL_TRY(ncclGroupStart());
    for (int i = 0; i < d.n_rows; ++i) {
        const long long* r = d.rows + i * 4;
        NCCL_TRY(ncclSend(g + r[1], (size_t)r[3], dt, (int)r[0], comm, cs));
        NCCL_TRY(ncclRecv(g + r[2], (size_t)r[3], dt, (int)r[0], comm, cs));
    }
    off = 0;
    for (int i = 0; i < d.n_blks; ++i) {
        const int* c = d.blks + i * kBlk;
        const long long cnt = (long long)c[5] * c[6];
        NCCL_TRY(ncclSend(stage + off, (size_t)cnt, dt, c[0], comm, cs));
        NCCL_TRY(ncclRecv(stage + total + off, (size_t)cnt, dt, c[0], comm, cs));
        off += cnt;
    }
    NCCL_TRY(ncclGroupEnd());
    off = 0;
    for (int i = 0; i < d.n_blks; ++i) {
        const int* c = d.blks + i * kBlk;
        const int cnt = c[5] * c[6];
        hipLaunchKernelGGL(unpack_block_kernel<T>, dim3(cdiv(cnt, 256)), dim3(256), 0, cs, g, d.pitch, c[3], c[4], c[5],
                           c[6], stage + total + off);
        off += cnt;
    }
    CME_TRY(hipGetLastError());
    return 0;
}

int find_sub(const SubDesc* subs, int nsub, int rank) {
    for (int i = 0; i < nsub; ++i)
        if (subs[i].rank == rank) return i;
    return -1;
}

// Loopback transport: PULL every halo of sub `si` (state k) from the owning
// neighbour's matching send region with device copies on si's comm stream.
template <typename T>
int post_exchange_loopback(const SubDesc* subs, int nsub, int si, int k, hipStream_t cs) {
    const SubDesc& d = subs[si];
    T* g = (T*)d.buf[k];
    for (int i = 0; i < d.n_rows; ++i) {
        const long long* r = d.rows + i * 4;
        const int pj = find_sub(subs, nsub, (int)r[0]);
        if (pj < 0) return (int)hipErrorInvalidValue;
        const SubDesc& pd = subs[pj];
        long long src_off = -1;
        for (int j = 0; j < pd.n_rows; ++j)
            if (pd.rows[j * 4] == d.rank) src_off = pd.rows[j * 4 + 1];
        if (src_off < 0) return (int)hipErrorInvalidValue;
        CME_TRY(hipMemcpyAsync(g + r[2], (T*)pd.buf[k] + src_off, (size_t)r[3] * sizeof(T), hipMemcpyDeviceToDevice,
                               cs));
    }
    for (int i = 0; i < d.n_blks; ++i) {
        const int* c = d.blks + i * kBlk;
        const int pj = find_sub(subs, nsub, c[0]);
        if (pj < 0) return (int)hipErrorInvalidValue;
        const SubDesc& pd = subs[pj];
        const int* m = nullptr;
        for (int j = 0; j < pd.n_blks; ++j)
            if (pd.blks[j * kBlk] == d.rank) m = pd.blks + j * kBlk;
        if (!m || m[5] != c[5] || m[6] != c[6]) return (int)hipErrorInvalidValue;
        const T* src = (const T*)pd.buf[k] + (size_t)m[2] * pd.pitch + m[1];
        T* dst = g + (size_t)c[4] * d.pitch + c[3];
        CME_TRY(hipMemcpy2DAsync(dst, (size_t)d.pitch * sizeof(T), src, (size_t)pd.pitch * sizeof(T),
                                 (size_t)c[6] * sizeof(T), (size_t)c[5], hipMemcpyDeviceToDevice, cs));
    }
    return 0;
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
    if (transport == 0 && nsub != 1) return (int)hipErrorInvalidValue;
    if (tblock < 1 || tblock > 4 || (tblock > 2 && sizeof(T) != 4)) return (int)hipErrorInvalidValue;
    // 0 (default): border stream || interior stream; 1: border then interior
    // on one stream. Measured on one N=8-rank subdomain (bench_dist_rank.py,
    // null transport): 0.041 vs 0.045 ms/step -- kept as a switch for
    // re-measuring on other topologies.
    static const int schedule = [] {
        const char* e = getenv("CME_DIST_SCHEDULE");
        return e ? atoi(e) : 0;
    }();
    DistCtx* ctx;
    CME_TRY_INT(get_ctx(nsub, &ctx));
    const ncclDataType_t dt = sizeof(T) == 4 ? ncclFloat32 : ncclFloat64;
    int peers[kMaxSubs][16];
    int npeer[kMaxSubs];
    for (int si = 0; si < nsub; ++si) {
        npeer[si] = local_peers(subs, nsub, si, peers[si]);
        if (transport == 1 && npeer[si] != subs[si].n_rows + subs[si].n_blks) return (int)hipErrorInvalidValue;
    }
    auto exchange = [&](int si, int k) -> int {
        if (transport == 0) return post_exchange_rccl<T>(comm, subs[si], (T*)subs[si].buf[k], dt, ctx->sub[si].comm);
        if (transport == 1) return post_exchange_loopback<T>(subs, nsub, si, k, ctx->sub[si].comm);
        return 0;  // transport 2: no exchange (benchmarking the compute schedule)
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
    if (exchange_first) {  // make the halos of the current state valid
        for (int si = 0; si < nsub; ++si) CME_TRY_INT(exchange(si, cur));
        for (int si = 0; si < nsub; ++si) CME_TRY(hipEventRecord(ctx->sub[si].ev_comm, ctx->sub[si].comm));
        for (int si = 0; si < nsub; ++si)
            for (int j = 0; j < nsub; ++j) CME_TRY(hipStreamWaitEvent(ctx->sub[si].compute, ctx->sub[j].ev_comm, 0));
    }
    int pass = 0;
    for (int it = 0; it < iters; ++pass) {
        // timesteps in this pass: tblock, or what is left (a tail pass of
        // fewer steps reuses the tblock*B-deep halos and regions)
        const int ns = (iters - it) < tblock ? (iters - it) : tblock;
        const int par = pass & 1;
        if (sync) {
            for (int si = 0; si < nsub; ++si) {
                SubCtx& u = ctx->sub[si];
                CME_TRY_INT(sweep(si, subs[si].interior, subs[si].n_int, cur, ns, u.compute));
                CME_TRY_INT(sweep(si, subs[si].border, subs[si].n_b, cur, ns, u.compute));
                CME_TRY(hipEventRecord(u.ev_border[par], u.compute));
            }
            for (int si = 0; si < nsub; ++si) {
                SubCtx& u = ctx->sub[si];
                CME_TRY(hipStreamWaitEvent(u.comm, u.ev_border[par], 0));
                for (int j = 0; j < npeer[si]; ++j)
                    CME_TRY(hipStreamWaitEvent(u.comm, ctx->sub[peers[si][j]].ev_border[par], 0));
                CME_TRY_INT(exchange(si, cur ^ 1));
                CME_TRY(hipEventRecord(u.ev_comm, u.comm));
            }
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
                CME_TRY(hipStreamWaitEvent(u.compute, u.ev_comm, 0));
                for (int j = 0; j < npeer[si]; ++j)
                    CME_TRY(hipStreamWaitEvent(u.compute, ctx->sub[peers[si][j]].ev_comm, 0));
                CME_TRY_INT(sweep(si, subs[si].border, subs[si].n_b, cur, ns, u.compute));
                CME_TRY(hipEventRecord(u.ev_border[par], u.compute));
            }
            for (int si = 0; si < nsub; ++si) {
                SubCtx& u = ctx->sub[si];
                CME_TRY(hipStreamWaitEvent(u.comm, u.ev_border[par], 0));
                for (int j = 0; j < npeer[si]; ++j)
                    CME_TRY(hipStreamWaitEvent(u.comm, ctx->sub[peers[si][j]].ev_border[par], 0));
                CME_TRY_INT(exchange(si, cur ^ 1));
                CME_TRY(hipEventRecord(u.ev_comm, u.comm));
            }
            for (int si = 0; si < nsub; ++si) {
                SubCtx& u = ctx->sub[si];
                CME_TRY_INT(sweep(si, subs[si].interior, subs[si].n_int, cur, ns, u.compute));
                CME_TRY(hipEventRecord(u.ev_int[par], u.compute));
            }
        } else {
            for (int si = 0; si < nsub; ++si) {  // border strips of pass i
                SubCtx& u = ctx->sub[si];
                CME_TRY(hipStreamWaitEvent(u.border, u.ev_comm, 0));
                for (int j = 0; j < npeer[si]; ++j)
                    CME_TRY(hipStreamWaitEvent(u.border, ctx->sub[peers[si][j]].ev_comm, 0));
                CME_TRY(hipStreamWaitEvent(u.border, u.ev_int[par ^ 1], 0));
                CME_TRY_INT(sweep(si, subs[si].border, subs[si].n_b, cur, ns, u.border));
                CME_TRY(hipEventRecord(u.ev_border[par], u.border));
            }
            for (int si = 0; si < nsub; ++si) {  // halo exchange of the new state
                SubCtx& u = ctx->sub[si];
                CME_TRY(hipStreamWaitEvent(u.comm, u.ev_border[par], 0));
                for (int j = 0; j < npeer[si]; ++j)
                    CME_TRY(hipStreamWaitEvent(u.comm, ctx->sub[peers[si][j]].ev_border[par], 0));
                CME_TRY_INT(exchange(si, cur ^ 1));
                CME_TRY(hipEventRecord(u.ev_comm, u.comm));
            }
            for (int si = 0; si < nsub; ++si) {  // deep interior, overlapping both
                SubCtx& u = ctx->sub[si];
                CME_TRY(hipStreamWaitEvent(u.compute, u.ev_border[par ^ 1], 0));
                CME_TRY_INT(sweep(si, subs[si].interior, subs[si].n_int, cur, ns, u.compute));
                CME_TRY(hipEventRecord(u.ev_int[par], u.compute));
            }
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
        CME_TRY(hipStreamWaitEvent(s, u.ev_comm, 0));
    }
    *cur_out = cur;
    return 0;
}

}  // namespace

// The distributed heat loop (see dist_run). transport 0 = RCCL (`comm`, one
// sub), 1 = loopback (every neighbour is one of `subs`), 2 = none (halos are
// not exchanged; benchmarks/bench_dist_rank.py). dtype 0 f32, 1 f64.
// tblock n (1-4): n steps per exchange (nB-deep halos, `interior` shrunk by
// nB on neighbour sides, `ext` = owned region grown by (n-1)B on neighbour
// sides; 3 and 4 fp32 only). fma: FMA-contracted stencil.
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

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(halo_pack_f32, 256, pack_block_kernel<float>);
