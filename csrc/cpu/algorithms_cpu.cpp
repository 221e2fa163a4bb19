// OpenMP CPU backend of the data-parallel algorithms (the GPU versions are
// in csrc/hip/algorithms.hip): stable selection / compaction / partition,
// vectorised lower/upper bound, segmented reduction, arg-reduction and inner
// product. These are the Thrust calls of the reference (remove_copy_if,
// upper_bound, reduce_by_key, max_element, inner_product:
// hw/hw3/solution/solve_cipher_solution.cu:131-200) on the "runs without a
// GPU" path, built on the OpenMP idiom of hw/hw_final/programming/fp.cu:130-152.
//
// Selection is two-pass and stable: every thread counts the selected items of
// its contiguous share, the per-thread counts are exclusive-scanned, then each
// thread writes its share at its offset -- the CPU analogue of the GPU's
// reduce-then-scan compaction.
#include <omp.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

#include "cme213/cpu_common.h"

namespace {

inline void share(long long n, int t, int nt, long long* b, long long* e) {
    *b = n * t / nt;
    *e = n * (t + 1) / nt;
}

// raw element as an unsigned word of `esize` bytes (predicates compare bitwise)
inline uint64_t word(const uint8_t* x, long long i, int esize) {
    switch (esize) {
        case 1: return x[i];
        case 4: {
            uint32_t v;
            memcpy(&v, x + 4 * i, 4);
            return v;
        }
        default: {
            uint64_t v;
            memcpy(&v, x + 8 * i, 8);
            return v;
        }
    }
}

// pred: 0 flags[i] != 0; 1 x[i] != value; 2 head of a run (i == 0 or x[i] != x[i-1])
inline bool selected(const uint8_t* x, const uint8_t* flags, long long i, int esize, int pred, uint64_t value,
                     bool invert) {
    bool s;
    if (pred == 0)
        s = flags[i] != 0;
    else if (pred == 1)
        s = word(x, i, esize) != value;
    else
        s = i == 0 || word(x, i, esize) != word(x, i - 1, esize);
    return s != invert;
}

template <typename T>
long long bound(const T* s, long long n, T q, bool upper) {
    long long lo = 0, hi = n;
    while (lo < hi) {
        const long long mid = lo + (hi - lo) / 2;
        const bool go_right = upper ? !(q < s[mid]) : (s[mid] < q);
        if (go_right)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

template <typename T>
void search_t(const void* sorted, long long n, const void* q, long long nq, bool upper, int64_t* out) {
    const T* s = (const T*)sorted;
    const T* qq = (const T*)q;
#pragma omp parallel for schedule(static)
    for (long long i = 0; i < nq; ++i) out[i] = bound<T>(s, n, qq[i], upper);
}

template <typename T>
T identity(int op) {
    if (op == 0) return T(0);
    if (std::numeric_limits<T>::has_infinity)
        return op == 1 ? -std::numeric_limits<T>::infinity() : std::numeric_limits<T>::infinity();
    return op == 1 ? std::numeric_limits<T>::lowest() : std::numeric_limits<T>::max();
}

template <typename T>
void seg_reduce_t(const void* vals, const int64_t* off, long long nseg, int op, void* out) {
    const T* v = (const T*)vals;
    T* o = (T*)out;
#pragma omp parallel for schedule(dynamic, 256)
    for (long long s = 0; s < nseg; ++s) {
        T acc = identity<T>(op);
        for (int64_t i = off[s]; i < off[s + 1]; ++i) {
            const T x = v[i];
            if (op == 0)
                acc += x;
            else if (op == 1)
                acc = x > acc ? x : acc;
            else
                acc = x < acc ? x : acc;
        }
        o[s] = acc;
    }
}

// first index of the max (min); NaN never wins a comparison
template <typename T>
void arg_reduce_t(const void* x, long long n, bool is_max, void* val, int64_t* idx) {
    const T* v = (const T*)x;
    const int nt = omp_get_max_threads();
    std::vector<T> bv(nt);
    std::vector<long long> bi(nt, -1);
#pragma omp parallel num_threads(nt)
    {
        const int t = omp_get_thread_num(), tn = omp_get_num_threads();
        long long b, e;
        share(n, t, tn, &b, &e);
        if (b < e) {
            T best = v[b];
            long long bidx = b;
            for (long long i = b + 1; i < e; ++i)
                if (is_max ? v[i] > best : v[i] < best) best = v[i], bidx = i;
            bv[t] = best;
            bi[t] = bidx;
        }
    }
    T best{};
    long long bidx = -1;
    for (int t = 0; t < nt; ++t) {  // threads hold increasing index ranges: strict compare keeps the first
        if (bi[t] < 0) continue;
        if (bidx < 0 || (is_max ? bv[t] > best : bv[t] < best)) best = bv[t], bidx = bi[t];
    }
    memcpy(val, &best, sizeof(T));
    *idx = bidx;
}

}  // namespace

// mode 0: selected values, compacted; 1: their int64 indices; 2: stable
// partition (selected values, then the rest). *count = number selected.
CME_CPU_EXPORT int cme_cpu_select(const void* x, const uint8_t* flags, long long n, int esize, int pred,
                                  uint64_t value, int invert, int mode, void* out, long long* count) {
    if (esize != 1 && esize != 4 && esize != 8) return 1;
    if (n <= 0) {
        *count = 0;
        return 0;
    }
    if (pred == 0 && !flags) return 1;
    const uint8_t* xb = (const uint8_t*)x;
    uint8_t* ob = (uint8_t*)out;
    const int nt = omp_get_max_threads();
    std::vector<long long> off(nt + 1, 0);
    long long total = 0;
#pragma omp parallel num_threads(nt)
    {
        const int t = omp_get_thread_num(), tn = omp_get_num_threads();
        long long b, e;
        share(n, t, tn, &b, &e);
        long long c = 0;
        for (long long i = b; i < e; ++i) c += selected(xb, flags, i, esize, pred, value, invert != 0);
        off[t + 1] = c;
#pragma omp barrier
#pragma omp single
        {
            for (int k = 1; k <= tn; ++k) off[k] += off[k - 1];
            total = off[tn];
        }
        long long w = off[t];          // selected items go here
        long long r = total + (b - off[t]);  // mode 2: the rest, after every selected item
        for (long long i = b; i < e; ++i) {
            const bool s = selected(xb, flags, i, esize, pred, value, invert != 0);
            if (mode == 1) {
                if (s) ((int64_t*)out)[w++] = i;
            } else if (s) {
                memcpy(ob + (size_t)w++ * esize, xb + (size_t)i * esize, esize);
            } else if (mode == 2) {
                memcpy(ob + (size_t)r++ * esize, xb + (size_t)i * esize, esize);
            }
        }
    }
    *count = total;
    return 0;
}

// dtype: 0 f32, 1 i32, 2 u32, 3 i64, 4 f64
CME_CPU_EXPORT int cme_cpu_search(const void* sorted, long long n, const void* q, long long nq, int dtype, int upper,
                                  int64_t* out) {
    switch (dtype) {
        case 0: search_t<float>(sorted, n, q, nq, upper != 0, out); return 0;
        case 1: search_t<int32_t>(sorted, n, q, nq, upper != 0, out); return 0;
        case 2: search_t<uint32_t>(sorted, n, q, nq, upper != 0, out); return 0;
        case 3: search_t<int64_t>(sorted, n, q, nq, upper != 0, out); return 0;
        case 4: search_t<double>(sorted, n, q, nq, upper != 0, out); return 0;
        default: return 1;
    }
}

// op: 0 sum, 1 max, 2 min; dtype: 0 f32, 1 i32, 3 i64, 4 f64
CME_CPU_EXPORT int cme_cpu_seg_reduce(const void* vals, const int64_t* offsets, long long nseg, int dtype, int op,
                                      void* out) {
    switch (dtype) {
        case 0: seg_reduce_t<float>(vals, offsets, nseg, op, out); return 0;
        case 1: seg_reduce_t<int32_t>(vals, offsets, nseg, op, out); return 0;
        case 3: seg_reduce_t<int64_t>(vals, offsets, nseg, op, out); return 0;
        case 4: seg_reduce_t<double>(vals, offsets, nseg, op, out); return 0;
        default: return 1;
    }
}

// (value, first index) of the max / min; dtype as seg_reduce
CME_CPU_EXPORT int cme_cpu_arg_reduce(const void* x, long long n, int dtype, int is_max, void* val, int64_t* idx) {
    if (n <= 0) return 1;
    switch (dtype) {
        case 0: arg_reduce_t<float>(x, n, is_max != 0, val, idx); return 0;
        case 1: arg_reduce_t<int32_t>(x, n, is_max != 0, val, idx); return 0;
        case 3: arg_reduce_t<int64_t>(x, n, is_max != 0, val, idx); return 0;
        case 4: arg_reduce_t<double>(x, n, is_max != 0, val, idx); return 0;
        default: return 1;
    }
}

// op 0: sum(a*b) of fp32 with fp64 accumulation; op 1: count of equal 32-bit words
CME_CPU_EXPORT int cme_cpu_inner_product(const void* a, const void* b, long long n, int op, double* out) {
    double acc = 0.0;
    if (op == 0) {
        const float* x = (const float*)a;
        const float* y = (const float*)b;
#pragma omp parallel for reduction(+ : acc) schedule(static)
        for (long long i = 0; i < n; ++i) acc += (double)x[i] * (double)y[i];
    } else {
        const uint32_t* x = (const uint32_t*)a;
        const uint32_t* y = (const uint32_t*)b;
        long long c = 0;
#pragma omp parallel for reduction(+ : c) schedule(static)
        for (long long i = 0; i < n; ++i) c += (x[i] == y[i]);
        acc = (double)c;
    }
    *out = acc;
    return 0;
}
