// OpenMP CPU backends for scans / reductions / segmented scans (oracles and
// GPU-less path). Parallel scan = per-thread block sums, serial scan of the
// sums, per-thread add-back (the CPU analogue of scan-then-add).
#include <omp.h>

#include <cstdint>
#include <vector>

#include "cme213/cpu_common.h"

namespace {

template <typename T>
void scan_impl(const T* in, T* out, long long n, bool exclusive) {
    int nt = omp_get_max_threads();
    std::vector<T> sums(nt + 1, T(0));
#pragma omp parallel num_threads(nt)
    {
        int t = omp_get_thread_num();
        int tn = omp_get_num_threads();
        long long b = n * t / tn, e = n * (t + 1) / tn;
        T acc = T(0);
        for (long long i = b; i < e; ++i) acc += in[i];
        sums[t + 1] = acc;
#pragma omp barrier
#pragma omp single
        for (int k = 1; k <= tn; ++k) sums[k] += sums[k - 1];
        T run = sums[t];
        for (long long i = b; i < e; ++i) {
            T v = in[i];
            if (exclusive) {
                out[i] = run;
                run += v;
            } else {
                run += v;
                out[i] = run;
            }
        }
    }
}

template <typename T>
void reduce_impl(const T* in, long long n, int op, T* out) {
    T acc;
    if (op == 0) {
        double a = 0;  // fp64 accumulation for the oracle
#pragma omp parallel for reduction(+ : a)
        for (long long i = 0; i < n; ++i) a += (double)in[i];
        acc = (T)a;
    } else if (op == 1) {
        acc = in[0];
#pragma omp parallel for reduction(max : acc)
        for (long long i = 0; i < n; ++i) acc = in[i] > acc ? in[i] : acc;
    } else {
        acc = in[0];
#pragma omp parallel for reduction(min : acc)
        for (long long i = 0; i < n; ++i) acc = in[i] < acc ? in[i] : acc;
    }
    *out = acc;
}

}  // namespace

CME_CPU_EXPORT int cme_cpu_scan(const void* in, void* out, long long n, int dtype, int exclusive) {
    if (dtype == 0) scan_impl((const float*)in, (float*)out, n, exclusive);
    else if (dtype == 1) scan_impl((const int*)in, (int*)out, n, exclusive);
    else if (dtype == 2) scan_impl((const uint32_t*)in, (uint32_t*)out, n, exclusive);
    else return 1;
    return 0;
}

CME_CPU_EXPORT int cme_cpu_reduce(const void* in, long long n, int dtype, int op, void* out) {
    if (n <= 0) return 1;
    if (dtype == 0) reduce_impl((const float*)in, n, op, (float*)out);
    else if (dtype == 1) reduce_impl((const int*)in, n, op, (int*)out);
    else return 1;
    return 0;
}

// Sequential inclusive segmented scan (the reference checker's semantics,
// hw/hw_final/programming/aux/reference_spMVscan-released.cu:38-54), with an
// optional fused multiply. Parallelised over segments found from the flags.
CME_CPU_EXPORT int cme_cpu_segscan(const float* in, const float* xmul, float* out, const void* flags, int mode,
                                   long long n) {
    auto head = [&](long long i) -> bool {
        if (mode == 0) return ((const uint8_t*)flags)[i] != 0;
        return (((const uint32_t*)flags)[i >> 5] >> (i & 31)) & 1u;
    };
    std::vector<long long> starts;
    starts.push_back(0);
    for (long long i = 1; i < n; ++i)
        if (head(i)) starts.push_back(i);
    starts.push_back(n);
    long long ns = (long long)starts.size() - 1;
#pragma omp parallel for schedule(dynamic, 64)
    for (long long sgi = 0; sgi < ns; ++sgi) {
        float run = 0.f;
        for (long long i = starts[sgi]; i < starts[sgi + 1]; ++i) {
            float v = xmul ? in[i] * xmul[i] : in[i];
            run = (i == starts[sgi]) ? v : run + v;
            out[i] = run;
        }
    }
    return 0;
}
