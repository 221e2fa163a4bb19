// Tuning arm of the merge sort (libcme213_tune.so only, `make TUNE=1`): the
// 4-way merge-path pass, built and measured slower than two 2-way passes on
// MI355X (profiles/sort_r6.md: 48M int32 1.88 vs 1.44 ms). Production entry
// points are in csrc/hip/sort.hip; the schedule is the shared ms_sort_host.
#include "../hip/sort_kernels.h"

namespace {
// Stage 1 of a 4-way tile (ms_merge4_pass_kernel): the tile's slices of runs
// A, B, C, D sit in LDS as X = [A | C] (C from index xa on) and Y = [B | D]
// (D from y0 + yb on). Ordered by (pair, key) -- A and B pair 0, C and D
// pair 1 -- X and Y are each sorted, and one merge path over them yields
// [merge(A, B) | merge(C, D)], both stable (X first on ties). The pair bit
// rides above the 32-bit key, so the exhausted-run sentinel ~0 sorts after
// every real key and the step needs no bounds test. Same cursor discipline
// as ms_merge16.
__device__ __forceinline__ uint64_t ms_pair_key(const uint32_t* sk, int p, int e, int p1) {
    const uint32_t x = sk[lp(p)];
    return p < e ? ((uint64_t)(p >= p1 ? 1u : 0u) << 32) | x : ~0ull;
}

template <bool HAS_VALUES, int CAP>
__device__ __forceinline__ void ms_merge16_pairs(const uint32_t* sk, const uint32_t* sv, int lx, int xa, int y0, int ly,
                                                 int yb, int i, int j, uint32_t (&k)[kMsItems],
                                                 uint32_t (&v)[kMsItems]) {
    int pa = i, pb = y0 + j;
    const int ea = lx, eb = y0 + ly, sa = xa, sb = y0 + yb;
    uint64_t ka = ms_pair_key(sk, pa, ea, sa), kb = ms_pair_key(sk, pb, eb, sb);
#pragma unroll
    for (int q = 0; q < kMsItems; ++q) {
        const bool take_a = ka <= kb;
        k[q] = (uint32_t)(take_a ? ka : kb);
        if constexpr (HAS_VALUES) {
            const int x = take_a ? pa : pb;
            v[q] = sv[lp(x < CAP ? x : CAP - 1)];
        }
        pa += take_a ? 1 : 0;
        pb += take_a ? 0 : 1;
        const int np = take_a ? pa : pb;  // one LDS load per step
        const uint64_t nv = ms_pair_key(sk, np, take_a ? ea : eb, take_a ? sa : sb);
        ka = take_a ? nv : ka;
        kb = take_a ? kb : nv;
    }
}

// Exact 4-way splits of every output tile boundary of a 4-way pass (runs of
// L merged four at a time into runs of 4L; one wave per boundary). The tile's
// output is merge(AB, CD) with AB = merge(A, B) and CD = merge(C, D), neither
// materialised. Per boundary at diagonal d of its group this finds
//   x  = the AB keys among the first d outputs (outer merge path of AB / CD),
//   sA = the A keys among the first x keys of AB, sC = the C keys among the
//        first d - x keys of CD,
// and writes (x, sA, sC) to b4[3 t ..]. Inputs from the launch before
// (ms_partition_kernel at run length L with vfirst / vlast):
//   split2 -- the A / B (C / D) split at every tile multiple of each pair, so
//             any AB[m] lies in a window of one tile: the split of diagonal m
//             is bracketed by split2 at the tile multiples around m;
//   vfirst / vlast -- first / last key of every tile of AB and CD, which
//             narrow the outer search to one tile's width first, as the run
//             samples do for a 2-way pass.
// Then 8 outer candidates x 8 lanes: each outer round evaluates AB[m] and
// CD[d - 1 - m] for 8 candidates m by 8-ary inner searches in their
// one-tile windows (two searches per lane group, loads in flight together).
__global__ __launch_bounds__(256) void ms_partition4_kernel(const uint32_t* __restrict__ ki, long long n, long long L,
                                                            long long tile, long long ntiles,
                                                            const long long* __restrict__ split2,
                                                            const uint32_t* __restrict__ vfirst,
                                                            const uint32_t* __restrict__ vlast,
                                                            long long* __restrict__ b4) {
    const long long t = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= ntiles) return;  // wave-uniform: one wave per boundary, no barriers
    const int lane = lane_id(), c = lane >> 3, s = lane & 7;
    const long long o0 = t * tile, g0 = o0 & ~(4 * L - 1), d = o0 - g0;
    auto run = [&](long long off) { return off <= 0 ? 0ll : (off < L ? off : L); };
    const long long la = run(n - g0), lb = run(n - g0 - L), lc = run(n - g0 - 2 * L), ld = run(n - g0 - 3 * L);
    const long long lab = la + lb, lcd = lc + ld;
    const uint32_t* A = ki + g0;
    const uint32_t* B = A + la;
    const uint32_t* C = ki + g0 + lab;
    const uint32_t* D = C + lc;
    const long long pab = g0 / tile, pcd = (g0 + lab) / tile;  // first tile of each pair (lab % tile == 0 if lcd > 0)
    // the merge-path range of diagonal m in a pair, narrowed by split2
    auto bounds = [&](long long m, long long lx, long long ly, long long p, long long& lo, long long& hi) {
        lo = m - ly > 0 ? m - ly : 0;
        hi = m < lx ? m : lx;
        if (m > 0) {
            const long long j = (m + tile - 1) / tile;  // m in ((j - 1) tile, j tile]
            const long long slo = split2[p + j - 1];
            const long long shi = j * tile >= lx + ly ? lx : split2[p + j];
            lo = slo > lo ? slo : lo;
            hi = shi < hi ? shi : hi;
        }
    };
    const int gsh = lane & ~7;
    // two 8-ary merge-path searches per lane group at once: (A, B) at m1, (C, D) at m2
    auto search2 = [&](long long m1, long long& lo1, long long& hi1, long long m2, long long& lo2, long long& hi2) {
        while (__ballot(lo1 < hi1 || lo2 < hi2)) {
            const long long st1 = (hi1 - lo1 + 7) / 8, st2 = (hi2 - lo2 + 7) / 8;
            const long long q1 = lo1 + s * st1, q2 = lo2 + s * st2;
            const bool p1 = lo1 < hi1 && q1 < hi1 && A[q1] <= B[m1 - 1 - q1];
            const bool p2 = lo2 < hi2 && q2 < hi2 && C[q2] <= D[m2 - 1 - q2];
            const uint64_t f1m = (__ballot(!p1) >> gsh) & 0xffull, f2m = (__ballot(!p2) >> gsh) & 0xffull;
            const int f1 = f1m ? __builtin_ctzll(f1m) : 8, f2 = f2m ? __builtin_ctzll(f2m) : 8;
            if (lo1 < hi1) {
                const long long nlo = f1 == 0 ? lo1 : lo1 + (long long)(f1 - 1) * st1 + 1, mf = lo1 + f1 * st1;
                hi1 = f1 == 8 ? hi1 : (mf < hi1 ? mf : hi1);
                lo1 = nlo;
            }
            if (lo2 < hi2) {
                const long long nlo = f2 == 0 ? lo2 : lo2 + (long long)(f2 - 1) * st2 + 1, mf = lo2 + f2 * st2;
                hi2 = f2 == 8 ? hi2 : (mf < hi2 ? mf : hi2);
                lo2 = nlo;
            }
        }
    };
    long long lo = d - lcd > 0 ? d - lcd : 0, hi = d < lab ? d : lab;
    if (lo < hi) {  // wave-uniform; narrow x to one tile of AB on the samples: Q(j tile) over 64 candidates
        const long long j0 = (lo + tile - 1) / tile, j1 = (hi + tile - 1) / tile;
        long long jlo = j0, jhi = j1;
        const long long gb = (g0 + lab + d) / tile - 1;  // CD[d - 1 - j tile] ends tile gb - j
        while (jlo < jhi) {
            const long long st = (jhi - jlo + 63) / 64, j = jlo + lane * st;
            const bool q = j < jhi && vfirst[pab + j] <= vlast[gb - j];
            const uint64_t fails = __ballot(!q);
            const int f = fails ? __builtin_ctzll(fails) : 64;
            const long long nlo = f == 0 ? jlo : jlo + (long long)(f - 1) * st + 1, jf = jlo + f * st;
            jhi = f == 64 ? jhi : (jf < jhi ? jf : jhi);
            jlo = nlo;
        }
        if (jlo < j1 && jlo * tile < hi) hi = jlo * tile;
        if (jlo > j0 && (jlo - 1) * tile + 1 > lo) lo = (jlo - 1) * tile + 1;
    }
    while (lo < hi) {  // wave-uniform outer search: Q(m) = AB[m] <= CD[d - 1 - m]
        const long long st = (hi - lo + 7) / 8, m = lo + c * st;
        const bool act = m < hi;
        long long lo1 = 0, hi1 = 0, lo2 = 0, hi2 = 0;
        if (act) {
            bounds(m, la, lb, pab, lo1, hi1);
            bounds(d - 1 - m, lc, ld, pcd, lo2, hi2);
        }
        search2(m, lo1, hi1, d - 1 - m, lo2, hi2);
        bool q = false;
        if (act) {  // AB[m] and CD[d - 1 - m] from their splits (X first on ties)
            const long long m2 = d - 1 - m, jb = m - lo1, jd = m2 - lo2;
            const uint32_t ab = lo1 < la && (jb >= lb || A[lo1] <= B[jb]) ? A[lo1] : B[jb];
            const uint32_t cd = lo2 < lc && (jd >= ld || C[lo2] <= D[jd]) ? C[lo2] : D[jd];
            q = ab <= cd;
        }
        const uint64_t fails = __ballot(!q);  // the 8 lanes of a candidate agree
        const int f = fails ? __builtin_ctzll(fails) >> 3 : 8;
        const long long nlo = f == 0 ? lo : lo + (long long)(f - 1) * st + 1, mf = lo + f * st;
        hi = f == 8 ? hi : (mf < hi ? mf : hi);
        lo = nlo;
    }
    const long long x = lo;
    long long lo1, hi1, lo2, hi2;
    bounds(x, la, lb, pab, lo1, hi1);
    bounds(d - x, lc, ld, pcd, lo2, hi2);
    search2(x, lo1, hi1, d - x, lo2, hi2);
    if (lane == 0) {
        b4[3 * t] = x;
        b4[3 * t + 1] = lo1;
        b4[3 * t + 2] = lo2;
    }
}

// One output tile of a 4-way pass (runs of L -> 4L): half the HBM passes of
// the 2-way form for two LDS merge stages per tile. b4 holds every
// boundary's (x, sA, sC) from ms_partition4_kernel, so the block loads
// exactly its 4096 keys: the slices of A, B, C and D, laid out as X = [A | C],
// Y = [B | D]. Stage 1 merges X and Y on (pair, key) into
// [merge(A, B) | merge(C, D)] (ms_merge16_pairs); stage 2 merges those two.
template <bool HAS_VALUES>
__global__ __launch_bounds__(kMsThreads) void ms_merge4_pass_kernel(const uint32_t* __restrict__ ki,
                                                                    uint32_t* __restrict__ ko,
                                                                    const uint32_t* __restrict__ vi,
                                                                    uint32_t* __restrict__ vo, long long n, long long L,
                                                                    int mode_out, const long long* __restrict__ b4,
                                                                    MsSamples smp) {
    constexpr int NT = kMsThreads, TILE = kMsTile;
    __shared__ uint32_t sk[lp_size(TILE) + 1];
    __shared__ uint32_t sv[HAS_VALUES ? lp_size(TILE) : 1];
    const int t = threadIdx.x;
    const long long tile = xcd_remap(blockIdx.x, gridDim.x);
    const long long o0 = tile * TILE;
    const long long o1 = o0 + TILE < n ? o0 + TILE : n;
    const long long g0 = o0 & ~(4 * L - 1);
    auto run = [&](long long off) { return off <= 0 ? 0ll : (off < L ? off : L); };
    const long long la = run(n - g0), lb = run(n - g0 - L), lc = run(n - g0 - 2 * L), ld = run(n - g0 - 3 * L);
    const long long lab = la + lb, lcd = lc + ld;
    const long long d0 = o0 - g0, d1 = o1 - g0;
    const long long x0 = b4[3 * tile], a0 = b4[3 * tile + 1], c0 = b4[3 * tile + 2];
    long long x1 = lab, a1 = la, c1 = lc;  // a tile ending its group takes the rest of all four runs
    if (d1 != lab + lcd) {
        x1 = b4[3 * tile + 3];
        a1 = b4[3 * tile + 4];
        c1 = b4[3 * tile + 5];
    }
    const long long bb0 = x0 - a0, bb1 = x1 - a1, dd0 = (d0 - x0) - c0, dd1 = (d1 - x1) - c1;
    int na = (int)(a1 - a0), nb = (int)(bb1 - bb0), nc = (int)(c1 - c0), nd = (int)(dd1 - dd0);
    if (na < 0 || nb < 0 || nc < 0 || nd < 0 || na + nb + nc + nd != d1 - d0 || a0 < 0 || bb0 < 0 || c0 < 0 ||
        dd0 < 0 || a1 > la || bb1 > lb || c1 > lc || dd1 > ld)
        na = nb = nc = nd = 0;  // never out of range
    const long long ga = g0 + a0, gb = g0 + la + bb0, gc = g0 + lab + c0, gd = g0 + lab + lc + dd0;
    const int nx = na + nc, cnt = nx + nb + nd;
    for (int x = t; x < cnt; x += NT) {
        const long long g = x < na ? ga + x : (x < nx ? gc + (x - na) : (x < nx + nb ? gb + (x - nx) : gd + (x - nx - nb)));
        sk[lp(x)] = ki[g];
        if constexpr (HAS_VALUES) sv[lp(x)] = vi[g];
    }
    __syncthreads();
    const int p0 = kMsItems * t < cnt ? kMsItems * t : cnt;
    uint32_t k[kMsItems], v[kMsItems];
    {  // stage 1
        const int i = ms_split([&](int x) { return ((uint64_t)(x >= na ? 1u : 0u) << 32) | sk[lp(x)]; },
                               [&](int y) { return ((uint64_t)(y >= nb ? 1u : 0u) << 32) | sk[lp(nx + y)]; }, nx,
                               nb + nd, p0);
        ms_merge16_pairs<HAS_VALUES, TILE>(sk, sv, nx, na, nx, nb + nd, nb, i, p0 - i, k, v);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kMsItems; ++q) {
        sk[lp(kMsItems * t + q)] = k[q];
        if constexpr (HAS_VALUES) sv[lp(kMsItems * t + q)] = v[q];
    }
    __syncthreads();
    const int nab = na + nb;  // stage 2: merge(A, B) = [0, nab) with merge(C, D) = [nab, cnt)
    const int i = ms_split([&](int x) { return sk[lp(x)]; }, [&](int y) { return sk[lp(nab + y)]; }, nab, cnt - nab,
                           p0);
    ms_merge16<HAS_VALUES, TILE>(sk, sv, 0, nab, nab, cnt - nab, i, p0 - i, k, v);
    ms_store_tile<HAS_VALUES, NT>(sk, sv, k, v, ko, vo, o0, cnt, mode_out, smp);
}

struct MsFourWay {
    static constexpr bool kOn = true;
    static hipError_t pass(hipStream_t s, const uint32_t* ki, uint32_t* ko, const uint32_t* vi, uint32_t* vo, long long n,
                    long long L, long long mtile, long long tiles, const long long* split, const uint32_t* vfirst,
                    const uint32_t* vlast, long long* b4, int mo, MsSamples so) {
        hipLaunchKernelGGL(ms_partition4_kernel, dim3(cdiv(tiles, 4)), dim3(256), 0, s, ki, n, L, mtile, tiles, split,
                           vfirst, vlast, b4);
        if (vi)
            hipLaunchKernelGGL(ms_merge4_pass_kernel<true>, dim3(tiles), dim3(kMsThreads), 0, s, ki, ko, vi, vo, n, L,
                               mo, b4, so);
        else
            hipLaunchKernelGGL(ms_merge4_pass_kernel<false>, dim3(tiles), dim3(kMsThreads), 0, s, ki, ko, vi, vo, n,
                               L, mo, b4, so);
        return hipGetLastError();
    }
};
}  // namespace

// The merge sort with 4-way passes (cme_merge_sort_ws's arguments; ws of
// cme_merge_ws_bytes(n) bytes, required: the 4-way passes need the
// partition launches).
CME_EXPORT int cme_merge_sort4_tune(const uint32_t* in, uint32_t* out, uint32_t* tmp, const uint32_t* vin,
                                    uint32_t* vout, uint32_t* vtmp, long long n, int mode, void* ws, void* stream) {
    if (!ws) return (int)hipErrorInvalidValue;
    return ms_sort_host<MsFourWay>(in, out, tmp, vin, vout, vtmp, n, mode, ws, stream);
}
