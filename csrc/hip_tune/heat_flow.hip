// Cross-pass dataflow schedule of the wave-pipelined heat pass (gfx950).
//
// The multi-pass driver (heat_run: the reference's time loop,
// hw/hw2/solution/2dHeat_solution.cu:537-573, and the overlap idea of the
// async hw5 loop, hw/hw5/2dHeat_solution.cpp:537-628) launched one kernel per
// NS-step pass, so every pass ended with its slowest CU: the per-task trace of
// the 16384^2 pass has 15 % of the workgroup slots idle while the last round
// of tasks drains, plus a ~3 us kernel boundary (profiles/
// dist_rank_trace_r4.md, profiles/heat_flow_r5.md). Here ONE persistent
// launch runs all P passes:
//
//  * XCD bands: the grid's chunk rows are cut into 8 bands, band x handled by
//    the workgroups of XCD x (HW_REG_XCC_ID; dispatch is round-robin over the
//    8 XCDs, so each holds 1/8 of the grid). Each band has its own ticket
//    word and hands out (pass, chunk, strip) tasks pass-major, so every task
//    a ticket depends on was handed out earlier -- within a band by the same
//    queue, across a band edge by a queue whose lower passes are all handed
//    out (no deadlock while every XCD holds a workgroup);
//  * task (p, s, c) of pass p > 0 waits until the 3 x 3 neighbourhood of
//    tasks (p - 1, s +- 1, c +- 1) has finished (per-task completion words
//    holding 1 + the last finished pass). A task reads rows y0 - NS*B ..
//    y1 + NS*B and columns xs - 16 .. xs + OUT + 16 of its input and writes
//    [y0, y1) x [xs, xs + OUT) of its output, so with chunks of >= NS*B rows
//    and strips of >= 16 columns that neighbourhood covers the read-after-
//    write on the new input AND the write-after-read on the buffer this pass
//    overwrites (the previous pass's input);
//  * hand-off without an L2 write-back: producer and consumer of every edge
//    inside a band share the XCD's L2, so the producer only drains its
//    stores (vmcnt(0)) before its completion word and the consumer only
//    invalidates its L1 (one agent-scope acquire). The rows another band
//    reads -- the NS*B rows next to a band edge -- are stored write-through
//    (sc1) instead of non-temporally, so they are in memory when the flag
//    is (cdna_hip_programming.md §6 Guideline 16, R1). Measured
//    alternatives (profiles/heat_flow_r5.md): one global queue with a
//    release fence (buffer_wbl2) after every task ran 7 % slower than
//    per-pass launches; every output row write-through 35 % slower.
//
// The tail of pass p overlaps the head of pass p + 1; only the last pass
// drains. Each task's arithmetic is heat_pipe.h's pipe_task, so the result is
// that of P one-pass launches, bit for bit (tests/test_heat_flow.py).
//
// Bounded waits: a completion word not reached within `spins` polls sets a
// per-call abort word (every workgroup stops at its next ticket or poll) and
// the sticky pinned timeout word that cme_heat_flow_status reports -- the
// grid always drains.
//
// LDS hazard found on the way: lane 0's LDS write of the next ticket needs
// an explicit s_waitcnt lgkmcnt(0) before the barrier the other waves read it
// behind -- hipcc drops the one __syncthreads() carries when the barrier heads
// the loop and the write ends the body (profiles/lds_broadcast_isa_r6.md) --
// and waves then ran the previous ticket (two tasks wrong in ~1 run of 5 at
// 4096^2). cme::lds_bcast_sync (wave.h) is the wait + barrier.
#include "../hip/heat_pipe.h"
#include "cme213/persist_ws.h"
#include "cme213/wave.h"

using namespace cme;

namespace {

constexpr int kBands = 8;      // one per XCD
constexpr int kCtlStride = 32;  // ticket words 128 B apart

struct FlowArgs {
    unsigned* ctl;       // [0] abort, [1] give-up records, [3] tasks per pass; ticket of band x at [32 (x + 1)]
    unsigned* done;      // [tasks per pass]: 1 + the last pass that task slot finished (zeroed per call)
    unsigned* timeout;   // pinned host word: set when a wait gives up (sticky)
    unsigned spins;      // polls per wait before giving up
    int npass;
    int chunk;           // rows per chunk
    // diagnostics (CME_FLOW_MODE): 1 an agent-scope release fence after every
    // task, 4096 one global queue (no bands) with every output row stored
    // non-temporally and a release fence after every task, 2048 the first
    // task never publishes (the timeout / drain test)
    int mode;
    unsigned long long* trace;  // profiling: per ticket {ticket time, start, end, HW_ID | XCC_ID << 32}
};

// OST: output stores of the pipelined task, 0 non-temporal (every task then
// needs a release fence), 2 non-temporal except the band-edge rows (write-
// through)
template <typename T, int ORDER, int RB, int NS, int FMA, int PD, bool NT, int WPR, int VW, int OCC, int OST>
__global__ __launch_bounds__(NS * WPR * 64, (OCC > 0 ? 4 * OCC / NS : 1)) void heat_flow_kernel(
    T* a, T* b, int pitch, int gy, S2Regions R, int xb1, int xe1, int yb1, int ye1, T xcfl, T ycfl, FlowArgs f) {
    constexpr int NSLOT = PipeN<T, ORDER, RB, NS, FMA, false, PD, NT, WPR, VW, false>::NSLOT;
    constexpr int B = HeatOrder<ORDER>::B;
    __shared__ V4<T> ring[NS - 1][NSLOT][RB][VW / 4][64 * WPR];
    __shared__ V4<T> edge[WPR > 1 ? NS : 1][3][RB][WPR][2];
    __shared__ int s_ticket, s_stop;
    const int lane = lane_id();
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
    const int k = wv / WPR, sub = wv % WPR;
    const int tpp = R.wave_end[0];
    const int strips = R.strips[0];
    const int nch = tpp / strips;
    // this workgroup's band: its XCD's chunk rows [c_lo, c_hi) (OST 0: the
    // whole grid, one queue)
    const int band = OST == 2 ? (int)(__builtin_amdgcn_s_getreg(20 | (31 << 11)) & 7) : 0;  // HW_REG_XCC_ID
    const int c_lo = OST == 2 ? band * nch / kBands : 0;
    const int c_hi = OST == 2 ? (band + 1) * nch / kBands : nch;
    const int btasks = (c_hi - c_lo) * strips;
    const int total = btasks * f.npass;
    unsigned* ticket = f.ctl + kCtlStride * (band + 1);
    // rows other bands read: the NS*B next to each interior band edge
    const int wt_lo = (OST == 2 && band > 0) ? R.yb[0] + c_lo * f.chunk + NS * B : INT_MIN;
    const int wt_hi = (OST == 2 && band < kBands - 1) ? R.yb[0] + c_hi * f.chunk - NS * B : INT_MAX;
    if (blockIdx.x == 0 && threadIdx.x == 0) f.ctl[3] = (unsigned)tpp;  // diagnostics (cme_heat_flow_debug)
    // ONE lane fetches the next ticket, at the END of the previous task's
    // divergent publish block (and once before the loop): a second lane-0
    // block at the top of the loop body was merged with the publish block
    // across the back edge by the compiler, which then treated the loop exit
    // as divergent
    unsigned long long t_tk = 0;
    auto fetch = [&]() {
        int tk = btasks > 0 ? (int)__hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                            : total;
        if (__hip_atomic_load(f.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) tk = total;
        s_ticket = tk;
        s_stop = 0;
        if (f.trace) t_tk = wall_clock64();
    };
    if (threadIdx.x == 0) fetch();
    for (;;) {
        lds_bcast_sync();  // lane 0's ticket write (wave.h: the loop-head barrier case)
        const int t = __builtin_amdgcn_readfirstlane(s_ticket);
        if (t >= total) break;
        const int pass = t / btasks, local = t - pass * btasks;
        const int strip = local % strips, ck = c_lo + local / strips;
        const int task = ck * strips + strip;
        if (pass > 0) {
            if (wv == 0) {
                // lanes 0..8 watch one neighbour task each (lane = 3 * dc + ds)
                const unsigned* w = nullptr;
                if (lane < 9) {
                    const int s2 = strip + lane % 3 - 1, c2 = ck + lane / 3 - 1;
                    if (s2 >= 0 && s2 < strips && c2 >= 0 && c2 < nch) w = f.done + c2 * strips + s2;
                }
                bool give_up = false;
                for (unsigned spins = 0;; ++spins) {
                    const bool mine =
                        w == nullptr ||
                        (int)(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - (unsigned)pass) >= 0;
                    if (__all(mine)) break;
                    if (spins >= f.spins) {
                        // diagnostics: up to 64 give-up records of 16 words
                        // {ticket, pass, strip, chunk, value seen by lanes 0..8}
                        unsigned slot = 0;
                        if (lane == 0) {
                            __hip_atomic_store(f.ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            __hip_atomic_store(f.timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                            slot = __hip_atomic_fetch_add(f.ctl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        }
                        slot = __shfl(slot, 0, 64);
                        if (slot < 64) {
                            unsigned* rec = f.done + tpp + 16 * slot;
                            if (lane == 0) {
                                rec[0] = (unsigned)t;
                                rec[1] = (unsigned)pass;
                                rec[2] = (unsigned)strip;
                                rec[3] = (unsigned)ck;
                            }
                            if (lane < 9)
                                rec[4 + lane] = w ? __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                  : 0xffffffffu;
                        }
                        give_up = true;
                        break;
                    }
                    if ((spins & 255u) == 255u &&
                        __builtin_amdgcn_readfirstlane(
                            __hip_atomic_load(f.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0u) {
                        give_up = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                // ONE acquire after the match (this CU's L1); its wait holds
                // the barrier below until the invalidate has completed
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (give_up && lane == 0) s_stop = 1;
            }
            lds_bcast_sync();
            if (__builtin_amdgcn_readfirstlane(s_stop)) break;
        }
        unsigned long long t_start = 0;
        if (f.trace && threadIdx.x == 0) t_start = wall_clock64();
        T* src = (pass & 1) ? b : a;
        T* dst = (pass & 1) ? a : b;
        pipe_task<T, ORDER, RB, NS, FMA, PD, NT, WPR, VW, false, NSLOT, OST>(
            ring, edge, R, 0, task, src, dst, pitch, gy, xb1, xe1, yb1, ye1, xcfl, ycfl, k, sub, lane, wt_lo, wt_hi);
        // publish: every wave drains its stores (and its last loads of the
        // input this pass's successors overwrite), barrier, one lane stores
        // the completion word
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            if (OST == 0 || (f.mode & 1)) {  // non-temporal band-crossing rows: write the L2 back first
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            const unsigned long long t_end = f.trace ? wall_clock64() : 0ull;  // before the flag
            if (!((f.mode & 2048) && t == 0))
                __hip_atomic_store(f.done + task, (unsigned)(pass + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (f.trace) {  // profiling only (vector stores)
                const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_REG_HW_ID
                const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // HW_REG_XCC_ID
                unsigned long long* tr = f.trace + 4ull * (pass * tpp + task);
                tr[0] = t_tk;
                tr[1] = t_start;
                tr[2] = t_end;
                tr[3] = ((unsigned long long)(xcc & 0xff) << 32) | hw;
            }
            fetch();
        }
    }
}

// per-call control words + completion words + give-up records
// (cme213/persist_ws.h), zeroed by one memset node
PersistWs& flow_ws() { return persist_ws_for<0>(); }

// The XCD bands assume workgroups on all 8 XCDs with XCC_ID 0..7 (the full
// MI355X in SPX mode): band x is served only by XCD x's workgroups. A probe
// launch records the XCC_IDs the dispatcher actually uses (vector atomics);
// any other set -- a CPX / DPX compute partition, a part with fewer XCDs --
// makes the launcher take the single-queue schedule (OST = 0), which needs
// no band. Cached per device.
__global__ void xcc_probe_kernel(unsigned* mask) {
    if (threadIdx.x == 0) atomicOr(mask, 1u << (__builtin_amdgcn_s_getreg(20 | (31 << 11)) & 31));  // HW_REG_XCC_ID
}

int xcd_bands_ok(bool* ok) {
    static int cached[64];  // 0 unknown, 1 all 8 bands served, 2 not
    int dev = 0;
    CME_TRY(hipGetDevice(&dev));
    int& c = cached[dev & 63];
    if (c == 0) {
        unsigned* m = nullptr;
        CME_TRY(hipMalloc(&m, 4));
        CME_TRY(hipMemset(m, 0, 4));
        hipLaunchKernelGGL(xcc_probe_kernel, dim3(64 * device_cu_count()), dim3(64), 0, nullptr, m);
        CME_TRY(hipGetLastError());
        unsigned h = 0;
        CME_TRY(hipMemcpy(&h, m, 4, hipMemcpyDeviceToHost));
        CME_TRY(hipFree(m));
        c = h == 0xffu ? 1 : 2;
    }
    *ok = c == 1;
    return 0;
}

constexpr size_t kCtlWords = kCtlStride * (kBands + 1);

template <typename T, int ORDER, int NS, int FMA, int RB, int PD, bool NT, int WPR, int VW, int OCC, int OST>
int launch_flow(T* a, T* b, int pitch, int gy, Region g, T xcfl, T ycfl, int npass, hipStream_t s,
                unsigned long long* trace, int* ntasks_out) {
    constexpr int B = HeatOrder<ORDER>::B;
    constexpr int kOut = PipeOut<NS, WPR, VW, B>::kOut;
    static_assert(kOut >= 16, "flow: the strip neighbourhood must cover the pass's column reach");
    if (npass < 1) return 0;
    if ((pitch & 63) != 0) return (int)hipErrorInvalidValue;
    if ((size_t)gy * pitch * sizeof(T) >= (1ull << 31)) return (int)hipErrorInvalidValue;  // 32-bit store offsets
    static const long resident = [] {
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &per_cu, heat_flow_kernel<T, ORDER, RB, NS, FMA, PD, NT, WPR, VW, OCC, OST>, NS * WPR * 64, 0) !=
                hipSuccess ||
            per_cu < 1)
            per_cu = 1;
        return (long)per_cu * device_cu_count();
    }();
    const int H = g.ye - g.yb;
    if (H <= 0 || g.xe <= g.xb) return 0;
    const int strips = (int)cdiv(g.xe - (g.xb & ~(VW - 1)), kOut);
    const int per_cu = (int)cme::tune_get(cme::kTuneFlowPerCU);
    int chunk = pipe_chunk<NS, RB, VW>(strips, H, 0, per_cu, resident, false);
    // the 3 x 3 neighbourhood covers a task's row reach only for chunks of
    // at least NS*B rows (a whole-height chunk has no row neighbours at all);
    // a band edge's write-through rows need two of them
    if (chunk < 2 * NS * B) chunk = ((2 * NS * B + RB - 1) / RB) * RB;
    // a whole number of chunk rows per band (the bands' XCDs then carry equal
    // work: 58 chunk rows at 16384^2 gave bands of 7 and 8, and the 8-row
    // bands' neighbours waited on them)
    {
        int n = (int)cdiv(H, chunk);
        n = n < kBands ? n : ((n + kBands - 1) / kBands) * kBands;
        const int c2 = (((int)cdiv(H, n) + RB - 1) / RB) * RB;
        if (c2 >= 2 * NS * B) chunk = c2;
    }
    const int nch = (int)cdiv(H, chunk);
    const long tpp = (long)strips * nch;
    if (tpp * npass >= (1l << 31) || chunk >= 65536) return (int)hipErrorInvalidValue;
    PersistWs* w = &flow_ws();
    {
        const int rc = w->reserve(kCtlWords + (size_t)tpp + 16 * 64);  // + 64 give-up records
        if (rc) return rc;
    }
    CME_TRY(hipMemsetAsync(w->dev, 0, w->words * 4, s));
    S2Regions R{};
    R.n = 1;
    R.xb[0] = g.xb, R.xe[0] = g.xe, R.yb[0] = g.yb, R.ye[0] = g.ye;
    R.strips[0] = strips;
    R.chunk[0] = chunk;  // no taper: every chunk of a strip is `chunk` rows (the last one shorter)
    R.wave_end[0] = (int)tpp;
    FlowArgs f;
    f.ctl = w->dev;
    f.done = w->dev + kCtlWords;
    f.timeout = w->timeout;
    const long sp = cme::tune_get(cme::kTuneFlowSpins);
    f.spins = sp > 0 ? (unsigned)sp : (1u << 22);
    f.npass = npass;
    f.chunk = chunk;
    f.mode = (int)cme::tune_get(cme::kTuneFlowMode);
    f.trace = trace;
    // every resident workgroup (a band's queue drains into its XCD's share of
    // them; fewer workgroups than the resident count would idle CUs)
    const long grid = resident;
    if (ntasks_out) *ntasks_out = (int)tpp;
    hipLaunchKernelGGL((heat_flow_kernel<T, ORDER, RB, NS, FMA, PD, NT, WPR, VW, OCC, OST>), dim3((unsigned)grid),
                       dim3(NS * WPR * 64), 0, s, a, b, pitch, gy, R, g.xb, g.xe, g.yb, g.ye, xcfl, ycfl, f);
    CME_LAUNCH_STATUS();
}

// the production pass of each arithmetic (fp32, order 8, wide lanes, RB = 2,
// non-temporal stores; heat_pipe.hip / heat_fast.hip): exact (FMA arm 0),
// FMA-contracted with term-major chains (4), reassociated with its terms
// interleaved across the lane's points (5); registers capped for 3 waves per
// SIMD
template <int FMA>
int flow_arith(float* a, float* b, int pitch, int gy, Region g, float xcfl, float ycfl, int npass, hipStream_t s,
               unsigned long long* trace, int* ntasks) {
    bool bands = false;
    {
        const int rc = xcd_bands_ok(&bands);
        if (rc) return rc;
    }
    // diagnostics (mode 4096), or not the 8 XCC_IDs the bands need: one
    // queue, a release fence per task
    if (!bands || (cme::tune_get(cme::kTuneFlowMode) & 4096))
        return launch_flow<float, 8, 4, FMA, 2, 1, true, 1, 8, 3, 0>(a, b, pitch, gy, g, xcfl, ycfl, npass, s, trace,
                                                                    ntasks);
    return launch_flow<float, 8, 4, FMA, 2, 1, true, 1, 8, 3, 2>(a, b, pitch, gy, g, xcfl, ycfl, npass, s, trace,
                                                                ntasks);
}

int flow_f32(float* a, float* b, int pitch, int gy, Region g, int arith, int ns, float xcfl, float ycfl, int npass,
             hipStream_t s, unsigned long long* trace, int* ntasks) {
    if (ns != 4) return (int)hipErrorInvalidValue;
    switch (arith) {
        case 0: return flow_arith<0>(a, b, pitch, gy, g, xcfl, ycfl, npass, s, trace, ntasks);
        case 1: return flow_arith<4>(a, b, pitch, gy, g, xcfl, ycfl, npass, s, trace, ntasks);
        case 2: return flow_arith<5>(a, b, pitch, gy, g, xcfl, ycfl, npass, s, trace, ntasks);
        default: return (int)hipErrorInvalidValue;
    }
}

}  // namespace

// npass passes of ns (4) timesteps of the whole region [xb, xe) x [yb, ye),
// fp32 order 8, in ONE persistent launch; pass 0 reads a, pass p reads
// (p & 1 ? b : a). arith: 0 exact, 1 FMA-contracted, 2 reassociated. The
// result lands in (npass & 1 ? b : a). Every cell outside the region holds
// the same fixed value in a and b (Dirichlet boundary).
CME_EXPORT int cme_heat_flow_f32(float* a, float* b, int pitch, int gy, int xb, int xe, int yb, int ye, int order,
                                 int arith, int ns, float xcfl, float ycfl, int npass, void* stream) {
    if (order != 8) return (int)hipErrorInvalidValue;
    return flow_f32(a, b, pitch, gy, Region{xb, xe, yb, ye}, arith, ns, xcfl, ycfl, npass, as_stream(stream), nullptr,
                    nullptr);
}

// profiling: the same launch recording every task's ticket / start / end
// wall clock (100 MHz) and HW_ID / XCC_ID into trace[4 * tasks_per_pass *
// npass] (index pass * tasks_per_pass + chunk * strips + strip;
// benchmarks/trace_flow.py); *ntasks = tasks per pass.
CME_EXPORT int cme_heat_flow_trace_f32(float* a, float* b, int pitch, int gy, int xb, int xe, int yb, int ye,
                                       int order, int arith, int ns, float xcfl, float ycfl, int npass,
                                       unsigned long long* trace, int* ntasks, void* stream) {
    if (order != 8 || !trace || !ntasks) return (int)hipErrorInvalidValue;
    return flow_f32(a, b, pitch, gy, Region{xb, xe, yb, ye}, arith, ns, xcfl, ycfl, npass, as_stream(stream), trace,
                    ntasks);
}

// Diagnostics: copies the first `nwords` words of the last launch's control
// block (abort, give-up count, 0, tasks per pass, ..., band tickets at
// 32 (x + 1), completion words from word 288, then the give-up records) to
// host memory (synchronous).
CME_EXPORT int cme_heat_flow_debug(unsigned* host, int nwords) {
    PersistWs& w = flow_ws();
    if (!w.dev || nwords < 0) return (int)hipErrorInvalidValue;
    if ((size_t)nwords > w.words) nwords = (int)w.words;
    return (int)hipMemcpy(host, w.dev, (size_t)nwords * 4, hipMemcpyDeviceToHost);
}

// Sticky give-up flag of the flow launches (pinned host word; read after the
// stream is synchronised). reset != 0 clears it.
CME_EXPORT int cme_heat_flow_status(unsigned* timed_out, int reset) {
    *timed_out = flow_ws().take_timeout(reset != 0);
    return 0;
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(heat_flow4_fma_f32_o8, 256, heat_flow_kernel<float, 8, 2, 4, 4, 1, true, 1, 8, 3, 2>);
CME_REGISTER_KERNEL(heat_flow4_fast_f32_o8, 256, heat_flow_kernel<float, 8, 2, 4, 5, 1, true, 1, 8, 3, 2>);
