// Data-parallel algorithm layer: the Thrust algorithms the reference calls
// (hw3 create/solve_cipher, hw1 cipher_solution, fp.cu) and the scan
// applications of slides/Lecture16 (stream compaction, dedup, split), as
// native wave64 kernels.
//
//  select      : copy_if / remove_copy_if / unique / stable_partition /
//                nonzero-indices, deterministic and stable. Reduce-then-scan:
//                (1) per-4096-tile selected counts from the predicate,
//                (2) exclusive scan of tile counts (cme_scan_rts),
//                (3) per-tile block scan, selected items compacted in LDS,
//                    then written as one contiguous coalesced run per tile.
//                Alternative for values / indices: ONE pass with the tile's
//                output offset from a two-level decoupled look-back over the
//                selected counts (select_lookback_kernel; slower, see
//                select_impl).
//                Predicates: flags[i] != 0, x[i] != value, i == 0 ||
//                x[i] != x[i-1] (head of a run: unique / reduce_by_key keys);
//                optionally inverted. Output: the values, or their indices.
//  search      : vectorised lower_bound / upper_bound (one lane per query;
//                the top levels of every search share cache lines in L2).
//  seg_reduce  : reduce_by_key values given segment offsets, one wave per
//                segment (DPP wave reduction), sum / max / min.
//  arg_reduce  : max_element / min_element (first index on ties), two-pass.
//  inner       : inner_product with (plus, multiplies) in fp32 with a fp64
//                per-lane accumulator, or (plus, equal_to) counting matches.
#include "cme213/common.h"
#include "cme213/lookback.h"
#include "cme213/wave.h"

using namespace cme;

extern "C" int cme_scan_rts(const void* in, void* out, long long n, int dtype, int exclusive, void* ws, void* stream);

namespace {

constexpr int kThreads = 256;
constexpr int kItems = 16;
constexpr int kTile = kThreads * kItems;

// predicate codes
enum : int { kPredFlags = 0, kPredNeq = 1, kPredHead = 2 };
constexpr int kSelectLookback = 8;  // cme_select mode bit: single-pass look-back (modes 0 / 1)

template <typename U>
__device__ __forceinline__ bool pred_at(const U* __restrict__ x, const uint8_t* __restrict__ flags, long long i, int pred,
                                        U value, int invert) {
    bool s;
    if (pred == kPredFlags)
        s = flags[i] != 0;
    else if (pred == kPredNeq)
        s = x[i] != value;
    else
        s = (i == 0) || (x[i] != x[i - 1]);
    return s != (invert != 0);
}

// This thread's 16 consecutive items + selection mask. Full tiles of an
// aligned input use 16-B vector loads (1/4/8 of them for 1/4/8-byte items);
// the last (partial) tile and unaligned inputs take the guarded scalar path.
template <typename U>
__device__ __forceinline__ uint32_t load_items(const U* __restrict__ x, const uint8_t* __restrict__ flags, long long n,
                                               long long base, int pred, U value, int invert, bool vec, U (&v)[kItems]) {
    uint32_t mask = 0;
    if (vec) {
        const uint4* px = reinterpret_cast<const uint4*>(x + base);
#pragma unroll
        for (int k = 0; k < (int)(kItems * sizeof(U) / 16); ++k) {
            const uint4 w = px[k];
            __builtin_memcpy(reinterpret_cast<char*>(v) + 16 * k, &w, 16);
        }
        if (pred == kPredFlags) {
            const uint4 fw = *reinterpret_cast<const uint4*>(flags + base);
            uint8_t f[kItems];
            __builtin_memcpy(f, &fw, 16);
#pragma unroll
            for (int j = 0; j < kItems; ++j) mask |= (uint32_t)(f[j] != 0) << j;
        } else if (pred == kPredNeq) {
#pragma unroll
            for (int j = 0; j < kItems; ++j) mask |= (uint32_t)(v[j] != value) << j;
        } else {
            const U prev0 = base > 0 ? x[base - 1] : U(0);
            mask |= (uint32_t)(base == 0 || v[0] != prev0);
#pragma unroll
            for (int j = 1; j < kItems; ++j) mask |= (uint32_t)(v[j] != v[j - 1]) << j;
        }
        if (invert) mask = ~mask & 0xffffu;
    } else {
#pragma unroll
        for (int j = 0; j < kItems; ++j) {
            const long long i = base + j;
            if (i < n) {
                v[j] = x[i];
                if (pred_at<U>(x, flags, i, pred, value, invert)) mask |= 1u << j;
            }
        }
    }
    return mask;
}

__device__ __forceinline__ bool tile_vec_ok(const void* x, const void* flags, long long n, long long tile0) {
    return tile0 + kTile <= n && ((uintptr_t)x & 15) == 0 && (flags == nullptr || ((uintptr_t)flags & 15) == 0);
}

template <typename U>
__global__ __launch_bounds__(kThreads) void select_count_kernel(const U* __restrict__ x,
                                                                const uint8_t* __restrict__ flags, long long n,
                                                                int pred, U value, int invert,
                                                                int* __restrict__ tile_counts) {
    __shared__ int red[kThreads / kWave];
    const long long tile0 = (long long)blockIdx.x * kTile;
    const long long base = tile0 + (long long)threadIdx.x * kItems;
    const bool vec = tile_vec_ok(x, pred == kPredFlags ? flags : nullptr, n, tile0);
    int c;
    if (vec && pred == kPredFlags) {  // flags only: one 16-B load
        const uint4 fw = *reinterpret_cast<const uint4*>(flags + base);
        uint8_t f[kItems];
        __builtin_memcpy(f, &fw, 16);
        c = 0;
#pragma unroll
        for (int j = 0; j < kItems; ++j) c += f[j] != 0;
        if (invert) c = kItems - c;
    } else {
        U v[kItems];
        c = __builtin_popcount(load_items<U>(x, flags, n, base, pred, value, invert, vec, v));
    }
    c = block_reduce<kThreads / kWave>(c, red);
    if (threadIdx.x == 0) tile_counts[blockIdx.x] = c;
}

// mode 0: write selected values; 1: selected indices (int64);
// 2: stable partition (selected first, then the rest, values).
template <typename U, int MODE>
__global__ __launch_bounds__(kThreads) void select_scatter_kernel(const U* __restrict__ x,
                                                                  const uint8_t* __restrict__ flags, long long n,
                                                                  int pred, U value, int invert,
                                                                  const int* __restrict__ tile_counts,
                                                                  const int* __restrict__ tile_offsets, int ntiles,
                                                                  void* __restrict__ out,
                                                                  long long* __restrict__ count_out) {
    using O = typename std::conditional<MODE == 1, long long, U>::type;
    __shared__ O stage[kTile];
    __shared__ int red[kThreads / kWave];
    const long long tile0 = (long long)blockIdx.x * kTile;
    const long long base = tile0 + (long long)threadIdx.x * kItems;
    const bool vec = tile_vec_ok(x, pred == kPredFlags ? flags : nullptr, n, tile0);
    U v[kItems];
    const uint32_t mask = load_items<U>(x, flags, n, base, pred, value, invert, vec, v);
    const int c = __builtin_popcount(mask);
    int tile_sel;
    const int off = block_exclusive_scan<kThreads / kWave>(c, red, tile_sel);
    const int tile_len = (int)min((long long)kTile, n - tile0);
    // selected items to stage[0, tile_sel); (partition) the rest after them
    int ks = off, ku = tile_sel + ((int)threadIdx.x * kItems - off);
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const long long i = base + j;
        if (i >= n) break;
        if (mask >> j & 1u) {
            if constexpr (MODE == 1)
                stage[ks++] = (O)i;
            else
                stage[ks++] = v[j];
        } else if constexpr (MODE == 2) {
            stage[ku++] = v[j];
        }
    }
    __syncthreads();
    const long long sel_off = tile_offsets[blockIdx.x];
    const long long last = ntiles - 1;
    const long long total_sel = (long long)tile_offsets[last] + tile_counts[last];
    O* o = reinterpret_cast<O*>(out);
    for (int k = threadIdx.x; k < tile_sel; k += kThreads) o[sel_off + k] = stage[k];
    if constexpr (MODE == 2) {
        const long long uns_off = total_sel + (tile0 - sel_off);
        for (int k = tile_sel + threadIdx.x; k < tile_len; k += kThreads) o[uns_off + (k - tile_sel)] = stage[k];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *count_out = total_sel;
}

// Single-pass select (modes 0 values / 1 indices): block b compacts tiles b,
// b+G, ... in order; the tile's output offset is the exclusive prefix of the
// selected counts, resolved by the two-level decoupled look-back (wave 0,
// lookback.h lb2_lookback) while the other waves stage the selected items in
// LDS. The next tile's raw items (full aligned tiles) are loaded before the
// look-back wait, so a block keeps two tiles of loads in flight. Reads the
// input once (the reduce-then-scan path reads it twice).
template <typename U>
struct RawTile {
    U v[kItems];
    uint4 fw;  // kPredFlags: the 16 flag bytes
    U prev;    // kPredHead: the item before this thread's first
};

template <typename U>
__device__ __forceinline__ void raw_load(const U* __restrict__ x, const uint8_t* __restrict__ flags, long long base,
                                         int pred, RawTile<U>& r) {
    const uint4* px = reinterpret_cast<const uint4*>(x + base);
#pragma unroll
    for (int k = 0; k < (int)(kItems * sizeof(U) / 16); ++k) {
        const uint4 w = px[k];
        __builtin_memcpy(reinterpret_cast<char*>(r.v) + 16 * k, &w, 16);
    }
    if (pred == kPredFlags) r.fw = *reinterpret_cast<const uint4*>(flags + base);
    if (pred == kPredHead) r.prev = base > 0 ? x[base - 1] : U(0);
}

template <typename U>
__device__ __forceinline__ uint32_t raw_mask(const RawTile<U>& r, long long base, int pred, U value, int invert) {
    uint32_t mask = 0;
    if (pred == kPredFlags) {
        uint8_t f[kItems];
        __builtin_memcpy(f, &r.fw, 16);
#pragma unroll
        for (int j = 0; j < kItems; ++j) mask |= (uint32_t)(f[j] != 0) << j;
    } else if (pred == kPredNeq) {
#pragma unroll
        for (int j = 0; j < kItems; ++j) mask |= (uint32_t)(r.v[j] != value) << j;
    } else {
        mask |= (uint32_t)(base == 0 || r.v[0] != r.prev);
#pragma unroll
        for (int j = 1; j < kItems; ++j) mask |= (uint32_t)(r.v[j] != r.v[j - 1]) << j;
    }
    return invert ? (~mask & 0xffffu) : mask;
}

template <typename U, int MODE>
__global__ __launch_bounds__(kThreads) void select_lookback_kernel(const U* __restrict__ x,
                                                                   const uint8_t* __restrict__ flags, long long n,
                                                                   int pred, U value, int invert, int ntiles,
                                                                   uint64_t* desc, unsigned* timeout,
                                                                   void* __restrict__ out,
                                                                   long long* __restrict__ count_out) {
    using O = typename std::conditional<MODE == 1, long long, U>::type;
    __shared__ O stage[kTile];
    __shared__ int red[kThreads / kWave];
    __shared__ int s_pre;
    const int lane = lane_id();
    const int wid = threadIdx.x / kWave;
    const Lb2 lbv = lb2_views(desc, ntiles);
    O* o = reinterpret_cast<O*>(out);
    const void* fl_chk = pred == kPredFlags ? (const void*)flags : nullptr;
    RawTile<U> cur, nxt;
    int tile = blockIdx.x;
    if (tile < ntiles && tile_vec_ok(x, fl_chk, n, (long long)tile * kTile))
        raw_load<U>(x, flags, (long long)tile * kTile + (long long)threadIdx.x * kItems, pred, cur);
    for (; tile < ntiles; tile += gridDim.x) {
        const long long tile0 = (long long)tile * kTile;
        const long long base = tile0 + (long long)threadIdx.x * kItems;
        uint32_t mask;
        if (tile_vec_ok(x, fl_chk, n, tile0)) {
            mask = raw_mask<U>(cur, base, pred, value, invert);
        } else {
            mask = load_items<U>(x, flags, n, base, pred, value, invert, false, cur.v);
        }
        int tile_sel;
        const int off = block_exclusive_scan<kThreads / kWave>(__builtin_popcount(mask), red, tile_sel);
        if (threadIdx.x == 0) lb2_put(lbv.agg + tile, tile_sel);
        int ks = off;
#pragma unroll
        for (int j = 0; j < kItems; ++j) {
            if (mask >> j & 1u) {
                if constexpr (MODE == 1)
                    stage[ks++] = (O)(base + j);
                else
                    stage[ks++] = cur.v[j];
            }
        }
        const int next = tile + gridDim.x;
        if (next < ntiles && tile_vec_ok(x, fl_chk, n, (long long)next * kTile))
            raw_load<U>(x, flags, (long long)next * kTile + (long long)threadIdx.x * kItems, pred, nxt);
        if (wid == 0) {
            const int pre = lb2_lookback<int>(lbv, tile, ntiles, tile_sel, 0u, timeout);
            if (lane == 0) s_pre = pre;
        }
        lds_bcast_sync();
        const long long sel_off = s_pre;
        for (int k = threadIdx.x; k < tile_sel; k += kThreads) o[sel_off + k] = stage[k];
        if (tile == ntiles - 1 && threadIdx.x == 0) *count_out = sel_off + tile_sel;
        __syncthreads();  // stage and s_pre are rewritten by the next tile
        cur = nxt;
    }
}

template <typename T, bool UPPER>
__global__ __launch_bounds__(kThreads) void search_kernel(const T* __restrict__ sorted, long long n,
                                                          const T* __restrict__ q, long long m,
                                                          long long* __restrict__ out) {
    for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < m; i += (long long)gridDim.x * kThreads) {
        const T v = q[i];
        long long lo = 0, len = n;
        while (len > 0) {
            const long long half = len >> 1;
            const T s = sorted[lo + half];
            const bool go_right = UPPER ? !(v < s) : (s < v);
            if (go_right) {
                lo += half + 1;
                len -= half + 1;
            } else {
                len = half;
            }
        }
        out[i] = lo;
    }
}

// Two-level search: every block first gathers S evenly spaced splitters
// sorted[k*n/S] into LDS; a query binary-searches them there (log2 S LDS
// reads instead of the top log2 S dependent global loads), then finishes in
// the n/S-element bucket in global memory. Persistent grid: the splitter load
// is amortised over many queries per block.
template <typename T, bool UPPER, int S>
__global__ __launch_bounds__(kThreads) void search2_kernel(const T* __restrict__ sorted, long long n,
                                                           const T* __restrict__ q, long long m,
                                                           long long* __restrict__ out) {
    __shared__ T sp[S];
    for (int k = threadIdx.x; k < S; k += kThreads) sp[k] = sorted[(long long)k * n / S];
    __syncthreads();
    for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < m; i += (long long)gridDim.x * kThreads) {
        const T v = q[i];
        // c = number of splitters strictly before the answer (a prefix: sp is sorted)
        int c = 0;
#pragma unroll
        for (int half = S / 2; half > 0; half >>= 1) {
            const T s = sp[c + half - 1];
            if (UPPER ? !(v < s) : (s < v)) c += half;
        }
        if (c < S && (UPPER ? !(v < sp[c]) : (sp[c] < v))) ++c;  // S is a power of two: one more probe
        long long lo = c == 0 ? 0 : (long long)(c - 1) * n / S + 1;
        const long long hi = c == S ? n : (long long)c * n / S;
        long long len = hi - lo;
        while (len > 0) {
            const long long half = len >> 1;
            const T s = sorted[lo + half];
            if (UPPER ? !(v < s) : (s < v)) {
                lo += half + 1;
                len -= half + 1;
            } else {
                len = half;
            }
        }
        out[i] = lo;
    }
}

template <typename T, typename Op>
__global__ __launch_bounds__(kThreads) void seg_reduce_kernel(const T* __restrict__ v,
                                                              const long long* __restrict__ offsets, long long nseg,
                                                              T* __restrict__ out) {
    const int lane = lane_id();
    const long long wave = ((long long)blockIdx.x * kThreads + threadIdx.x) / kWave;
    const long long nwaves = (long long)gridDim.x * (kThreads / kWave);
    for (long long sgm = wave; sgm < nseg; sgm += nwaves) {
        const long long b = offsets[sgm], e = offsets[sgm + 1];
        T acc = Op::template identity<T>();
        for (long long i = b + lane; i < e; i += kWave) acc = Op()(acc, v[i]);
        acc = wave_reduce<Op>(acc);
        if (lane == 0) out[sgm] = acc;
    }
}

// (value, index) pairs; ties -> lower index
template <typename T, bool MAX>
struct ArgPair {
    T v;
    long long i;
};

template <typename T, bool MAX>
__device__ __forceinline__ void arg_combine(T& v, long long& i, T v2, long long i2) {
    const bool better = MAX ? (v2 > v || (v2 == v && i2 < i)) : (v2 < v || (v2 == v && i2 < i));
    if (i < 0 || (i2 >= 0 && better)) {
        v = v2;
        i = i2;
    }
}

template <typename T, bool MAX>
__device__ __forceinline__ void block_arg(T& v, long long& idx, T* sv, long long* si) {
    // wave level via shuffles (pairs of 2 words), then across 4 waves in LDS
    for (int d = kWave / 2; d >= 1; d >>= 1) {
        const T v2 = __shfl_xor(v, d);
        const long long i2 = __shfl_xor(idx, d);
        arg_combine<T, MAX>(v, idx, v2, i2);
    }
    const int w = threadIdx.x / kWave;
    if (lane_id() == 0) {
        sv[w] = v;
        si[w] = idx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < kThreads / kWave; ++k) arg_combine<T, MAX>(v, idx, sv[k], si[k]);
    }
}

template <typename T, bool MAX>
__global__ __launch_bounds__(kThreads) void arg_partial_kernel(const T* __restrict__ x, long long n,
                                                               T* __restrict__ pv, long long* __restrict__ pi) {
    __shared__ T sv[kThreads / kWave];
    __shared__ long long si[kThreads / kWave];
    T v = T(0);
    long long idx = -1;
    // 4 independent loads in flight per lane (lane-contiguous indices, so
    // the per-lane scan order is increasing and ties keep the first index)
    const long long stride = (long long)gridDim.x * kThreads;
    long long i = (long long)blockIdx.x * kThreads + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const T a0 = x[i], a1 = x[i + stride], a2 = x[i + 2 * stride], a3 = x[i + 3 * stride];
        arg_combine<T, MAX>(v, idx, a0, i);
        arg_combine<T, MAX>(v, idx, a1, i + stride);
        arg_combine<T, MAX>(v, idx, a2, i + 2 * stride);
        arg_combine<T, MAX>(v, idx, a3, i + 3 * stride);
    }
    for (; i < n; i += stride) arg_combine<T, MAX>(v, idx, x[i], i);
    block_arg<T, MAX>(v, idx, sv, si);
    if (threadIdx.x == 0) {
        pv[blockIdx.x] = v;
        pi[blockIdx.x] = idx;
    }
}

template <typename T, bool MAX>
__global__ __launch_bounds__(kThreads) void arg_final_kernel(const T* __restrict__ pv, const long long* __restrict__ pi,
                                                             int np, T* __restrict__ ov, long long* __restrict__ oi) {
    __shared__ T sv[kThreads / kWave];
    __shared__ long long si[kThreads / kWave];
    T v = T(0);
    long long idx = -1;
    for (int k = threadIdx.x; k < np; k += kThreads) arg_combine<T, MAX>(v, idx, pv[k], pi[k]);
    block_arg<T, MAX>(v, idx, sv, si);
    if (threadIdx.x == 0) {
        *ov = v;
        *oi = idx;
    }
}

constexpr int kArgBlocks = 2048;

// inner products: MODE 0 sum(a*b) (fp32 in, fp64 accumulation); MODE 1
// count(a == b) over 32-bit words
template <int MODE>
__global__ __launch_bounds__(kThreads) void inner_kernel(const void* __restrict__ a, const void* __restrict__ b,
                                                         long long n, double* __restrict__ part) {
    __shared__ double red[kThreads / kWave];
    double acc = 0.0;
    for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads) {
        if constexpr (MODE == 0)
            acc += (double)((const float*)a)[i] * (double)((const float*)b)[i];
        else
            acc += ((const uint32_t*)a)[i] == ((const uint32_t*)b)[i] ? 1.0 : 0.0;
    }
    acc = block_reduce<kThreads / kWave>(acc, red);
    if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kThreads) void sum_f64_kernel(const double* __restrict__ part, int np,
                                                           double* __restrict__ out) {
    __shared__ double red[kThreads / kWave];
    double acc = 0.0;
    for (int k = threadIdx.x; k < np; k += kThreads) acc += part[k];
    acc = block_reduce<kThreads / kWave>(acc, red);
    if (threadIdx.x == 0) *out = acc;
}

template <typename U>
int select_impl(const U* x, const uint8_t* flags, long long n, int pred, U value, int invert, int mode, void* out,
                long long* count_out, int* ws, hipStream_t s) {
    if (n <= 0) return (int)hipMemsetAsync(count_out, 0, sizeof(long long), s);
    const long long ntiles = cdiv(n, (long long)kTile);
    if (ntiles > 0x7fffffffLL) return (int)hipErrorInvalidValue;
    // mode | kSelectLookback (modes 0 / 1): the single-pass look-back kernel.
    // Measured at 2^26 (benchmarks/bench_primitives.py, profiles/
    // select_lookback_r2.jsonl): 0.209 ms vs 0.126 for reduce-then-scan --
    // 16384 tiles of 4096 items are 16 rounds of the persistent grid, and
    // each round pays the look-back hand-off; reduce-then-scan stays default.
    const bool lookback = (mode & kSelectLookback) != 0;
    mode &= ~kSelectLookback;
    if (lookback && mode == 2) return (int)hipErrorInvalidValue;
    if (lookback) {
        if (ntiles > 0x3fffffffLL) return (int)hipErrorInvalidValue;
        unsigned* timeout = lb_host_timeout();
        if (!timeout) return (int)hipErrorOutOfMemory;
        static const int bpc0 = persistent_blocks_per_cu(select_lookback_kernel<U, 0>, kThreads);
        static const int bpc1 = persistent_blocks_per_cu(select_lookback_kernel<U, 1>, kThreads);
        const long long cap = (long long)device_cu_count() * (mode == 0 ? bpc0 : bpc1);
        const int grid = (int)(ntiles < cap ? ntiles : cap);
        uint64_t* desc = lb_descriptors(ws);
        CME_TRY(hipMemsetAsync(ws, 0, lb2_ws_bytes(ntiles), s));  // cme_select_ws_bytes covers it
        if (mode == 0)
            hipLaunchKernelGGL((select_lookback_kernel<U, 0>), dim3(grid), dim3(kThreads), 0, s, x, flags, n, pred,
                               value, invert, (int)ntiles, desc, timeout, out, count_out);
        else
            hipLaunchKernelGGL((select_lookback_kernel<U, 1>), dim3(grid), dim3(kThreads), 0, s, x, flags, n, pred,
                               value, invert, (int)ntiles, desc, timeout, out, count_out);
        CME_LAUNCH_STATUS();
    }
    int* counts = ws;
    int* offsets = ws + ntiles;
    void* scan_ws = ws + 2 * ntiles;
    hipLaunchKernelGGL(select_count_kernel<U>, dim3((unsigned)ntiles), dim3(kThreads), 0, s, x, flags, n, pred, value,
                       invert, counts);
    CME_TRY(hipGetLastError());
    int rc = cme_scan_rts(counts, offsets, ntiles, 1, 1, scan_ws, (void*)s);
    if (rc) return rc;
    switch (mode) {
        case 0:
            hipLaunchKernelGGL((select_scatter_kernel<U, 0>), dim3((unsigned)ntiles), dim3(kThreads), 0, s, x, flags,
                               n, pred, value, invert, counts, offsets, (int)ntiles, out, count_out);
            break;
        case 1:
            hipLaunchKernelGGL((select_scatter_kernel<U, 1>), dim3((unsigned)ntiles), dim3(kThreads), 0, s, x, flags,
                               n, pred, value, invert, counts, offsets, (int)ntiles, out, count_out);
            break;
        case 2:
            hipLaunchKernelGGL((select_scatter_kernel<U, 2>), dim3((unsigned)ntiles), dim3(kThreads), 0, s, x, flags,
                               n, pred, value, invert, counts, offsets, (int)ntiles, out, count_out);
            break;
        default: return (int)hipErrorInvalidValue;
    }
    CME_LAUNCH_STATUS();
}

// Splitter search when the sorted array is much longer than the splitter set
// and there are enough queries per block to amortise loading it; the plain
// one-level search otherwise (and for tiny inputs).
template <typename T>
int search_impl(const T* sorted, long long n, const T* q, long long m, int upper, long long* out, hipStream_t s) {
    if (m <= 0) return 0;
    constexpr int S = sizeof(T) == 4 ? 4096 : 2048;
    if (n >= 16LL * S && m >= 64LL * S) {
        const long long blocks = (m + 16LL * kThreads - 1) / (16LL * kThreads);  // >= 16 queries per lane
        const long long cap = 4LL * device_cu_count();
        const dim3 grid((unsigned)(blocks < cap ? blocks : cap));
        if (upper)
            hipLaunchKernelGGL((search2_kernel<T, true, S>), grid, dim3(kThreads), 0, s, sorted, n, q, m, out);
        else
            hipLaunchKernelGGL((search2_kernel<T, false, S>), grid, dim3(kThreads), 0, s, sorted, n, q, m, out);
        CME_LAUNCH_STATUS();
    }
    const dim3 grid(stream_grid(m, kThreads));
    if (upper)
        hipLaunchKernelGGL((search_kernel<T, true>), grid, dim3(kThreads), 0, s, sorted, n, q, m, out);
    else
        hipLaunchKernelGGL((search_kernel<T, false>), grid, dim3(kThreads), 0, s, sorted, n, q, m, out);
    CME_LAUNCH_STATUS();
}

template <typename T>
int seg_reduce_impl(const T* v, const long long* offsets, long long nseg, int op, T* out, hipStream_t s) {
    if (nseg <= 0) return 0;
    const dim3 grid(stream_grid(nseg * kWave, kThreads));
    switch (op) {
        case 0: hipLaunchKernelGGL((seg_reduce_kernel<T, OpAdd>), grid, dim3(kThreads), 0, s, v, offsets, nseg, out); break;
        case 1: hipLaunchKernelGGL((seg_reduce_kernel<T, OpMax>), grid, dim3(kThreads), 0, s, v, offsets, nseg, out); break;
        case 2: hipLaunchKernelGGL((seg_reduce_kernel<T, OpMin>), grid, dim3(kThreads), 0, s, v, offsets, nseg, out); break;
        default: return (int)hipErrorInvalidValue;
    }
    CME_LAUNCH_STATUS();
}

template <typename T, bool MAX>
int arg_impl(const T* x, long long n, void* ws, T* ov, long long* oi, hipStream_t s) {
    T* pv = (T*)ws;
    long long* pi = (long long*)((char*)ws + kArgBlocks * 8);  // ws: 16 * kArgBlocks bytes
    const int blocks = (int)(n < (long long)kArgBlocks * kThreads ? cdiv(n, (long long)kThreads) : kArgBlocks);
    const int nb = blocks < 1 ? 1 : blocks;
    hipLaunchKernelGGL((arg_partial_kernel<T, MAX>), dim3(nb), dim3(kThreads), 0, s, x, n, pv, pi);
    CME_TRY(hipGetLastError());
    hipLaunchKernelGGL((arg_final_kernel<T, MAX>), dim3(1), dim3(kThreads), 0, s, pv, pi, nb, ov, oi);
    CME_LAUNCH_STATUS();
}

}  // namespace

// Workspace for cme_select: ints for 2 * tiles + the tile-count scan scratch,
// or the two-level look-back descriptors (lb2_ws_bytes), whichever is larger.
CME_EXPORT long long cme_select_ws_bytes(long long n) {
    const long long t = cdiv(n, (long long)kTile);
    return 16 * t + 16 * cdiv(t, 64LL) + 4096 + 64;
}

// esize: 1, 4 or 8 bytes per element (values compared bitwise).
// pred: 0 flags!=0, 1 x!=value, 2 head-of-run; mode: 0 values, 1 indices,
// 2 stable partition; + 8: single-pass look-back kernel (modes 0 / 1).
// *count_out (device) = number selected.
CME_EXPORT int cme_select(const void* x, const uint8_t* flags, long long n, int esize, int pred,
                          unsigned long long value, int invert, int mode, void* out, long long* count_out, void* ws,
                          void* stream) {
    hipStream_t s = as_stream(stream);
    switch (esize) {
        case 1: return select_impl<uint8_t>((const uint8_t*)x, flags, n, pred, (uint8_t)value, invert, mode, out, count_out, (int*)ws, s);
        case 4: return select_impl<uint32_t>((const uint32_t*)x, flags, n, pred, (uint32_t)value, invert, mode, out, count_out, (int*)ws, s);
        case 8: return select_impl<uint64_t>((const uint64_t*)x, flags, n, pred, (uint64_t)value, invert, mode, out, count_out, (int*)ws, s);
        default: return (int)hipErrorInvalidValue;
    }
}

// dtype: 0 f32, 1 i32, 2 u32, 3 i64, 4 f64
CME_EXPORT int cme_search(const void* sorted, long long n, const void* q, long long m, int dtype, int upper,
                          long long* out, void* stream) {
    hipStream_t s = as_stream(stream);
    switch (dtype) {
        case 0: return search_impl<float>((const float*)sorted, n, (const float*)q, m, upper, out, s);
        case 1: return search_impl<int>((const int*)sorted, n, (const int*)q, m, upper, out, s);
        case 2: return search_impl<uint32_t>((const uint32_t*)sorted, n, (const uint32_t*)q, m, upper, out, s);
        case 3: return search_impl<long long>((const long long*)sorted, n, (const long long*)q, m, upper, out, s);
        case 4: return search_impl<double>((const double*)sorted, n, (const double*)q, m, upper, out, s);
        default: return (int)hipErrorInvalidValue;
    }
}

// dtype: 0 f32, 1 i32, 4 f64; op: 0 sum, 1 max, 2 min
CME_EXPORT int cme_seg_reduce(const void* v, const long long* offsets, long long nseg, int dtype, int op, void* out,
                              void* stream) {
    hipStream_t s = as_stream(stream);
    switch (dtype) {
        case 0: return seg_reduce_impl<float>((const float*)v, offsets, nseg, op, (float*)out, s);
        case 1: return seg_reduce_impl<int>((const int*)v, offsets, nseg, op, (int*)out, s);
        case 4: return seg_reduce_impl<double>((const double*)v, offsets, nseg, op, (double*)out, s);
        default: return (int)hipErrorInvalidValue;
    }
}

CME_EXPORT long long cme_arg_ws_bytes() { return 16LL * kArgBlocks; }

// max_element / min_element: dtype 0 f32, 1 i32, 4 f64; is_max 1/0.
CME_EXPORT int cme_arg_reduce(const void* x, long long n, int dtype, int is_max, void* ws, void* out_val,
                              long long* out_idx, void* stream) {
    hipStream_t s = as_stream(stream);
    if (n <= 0) return (int)hipErrorInvalidValue;
#define CME_ARG(T)                                                                                      \
    return is_max ? arg_impl<T, true>((const T*)x, n, ws, (T*)out_val, out_idx, s)                      \
                  : arg_impl<T, false>((const T*)x, n, ws, (T*)out_val, out_idx, s)
    switch (dtype) {
        case 0: CME_ARG(float);
        case 1: CME_ARG(int);
        case 4: CME_ARG(double);
        default: return (int)hipErrorInvalidValue;
    }
#undef CME_ARG
}

// mode 0: sum(a*b) over fp32 (fp64 accumulation); 1: count of equal 32-bit words.
CME_EXPORT int cme_inner_product(const void* a, const void* b, long long n, int mode, double* part, double* out,
                                 void* stream) {
    hipStream_t s = as_stream(stream);
    const int blocks = (int)(n < (long long)kArgBlocks * kThreads ? (n + kThreads - 1) / kThreads : kArgBlocks);
    const int nb = blocks < 1 ? 1 : blocks;
    if (mode == 0)
        hipLaunchKernelGGL(inner_kernel<0>, dim3(nb), dim3(kThreads), 0, s, a, b, n, part);
    else
        hipLaunchKernelGGL(inner_kernel<1>, dim3(nb), dim3(kThreads), 0, s, a, b, n, part);
    CME_TRY(hipGetLastError());
    hipLaunchKernelGGL(sum_f64_kernel, dim3(1), dim3(kThreads), 0, s, part, nb, out);
    CME_LAUNCH_STATUS();
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(select_scatter_u32, 256, select_scatter_kernel<uint32_t, 0>);
CME_REGISTER_KERNEL(select_lookback_u32, 256, select_lookback_kernel<uint32_t, 0>);
CME_REGISTER_KERNEL(search_i32, 256, search_kernel<int, false>);
CME_REGISTER_KERNEL(search2_i32, 256, search2_kernel<int, false, 4096>);
CME_REGISTER_KERNEL(arg_partial_f32, 256, arg_partial_kernel<float, true>);
