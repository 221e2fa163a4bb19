// OpenMP CPU sorts (hw4 parity, and the oracle for the GPU sorts).
//
// Radix sort: LSD, `num_bits` per pass, each pass = per-block histograms
// (omp parallel for) -> global digit totals -> exclusive scan -> per-block
// push-down offsets -> per-block stable scatter (omp parallel for), ping-pong
// buffers (hw/hw4/programming/radixsort.cpp:22-121; solution blocks n/8).
// Merge sort: recursive omp tasks with a serial std::sort cut-off, ping-pong
// buffers and a parallel merge that splits the left run at its median and the
// right run at upper_bound (hw/hw4/programming/mergesort.cpp:31-144).
#include <omp.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "cme213/cpu_common.h"

namespace {

// vin / vout: optional 32-bit values carried with the keys (stable)
void radix_pass(const uint32_t* in, uint32_t* out, long long n, int shift, int bits, int nblocks,
                const uint32_t* vin = nullptr, uint32_t* vout = nullptr) {
    const uint32_t nb = 1u << bits, mask = nb - 1;
    std::vector<uint32_t> hist((size_t)nblocks * nb, 0);
    const long long bs = (n + nblocks - 1) / nblocks;
#pragma omp parallel for schedule(static)
    for (int b = 0; b < nblocks; ++b) {
        uint32_t* h = &hist[(size_t)b * nb];
        const long long e = std::min(n, (b + 1) * bs);
        for (long long i = b * bs; i < e; ++i) ++h[(in[i] >> shift) & mask];
    }
    // offsets[b][d] = sum over digits < d of all blocks + sum of digit d in blocks < b
    std::vector<uint64_t> base(nb, 0);
    uint64_t run = 0;
    for (uint32_t d = 0; d < nb; ++d) {
        base[d] = run;
        for (int b = 0; b < nblocks; ++b) run += hist[(size_t)b * nb + d];
    }
    std::vector<uint64_t> off((size_t)nblocks * nb);
    for (uint32_t d = 0; d < nb; ++d) {
        uint64_t r = base[d];
        for (int b = 0; b < nblocks; ++b) {
            off[(size_t)b * nb + d] = r;
            r += hist[(size_t)b * nb + d];
        }
    }
#pragma omp parallel for schedule(static)
    for (int b = 0; b < nblocks; ++b) {
        uint64_t* o = &off[(size_t)b * nb];
        const long long e = std::min(n, (b + 1) * bs);
        if (vin) {
            for (long long i = b * bs; i < e; ++i) {
                const uint64_t d = o[(in[i] >> shift) & mask]++;
                out[d] = in[i];
                vout[d] = vin[i];
            }
        } else {
            for (long long i = b * bs; i < e; ++i) out[o[(in[i] >> shift) & mask]++] = in[i];
        }
    }
}

void merge_serial(const int* a, long long na, const int* b, long long nb, int* out) {
    std::merge(a, a + na, b, b + nb, out);
}

void parallel_merge(const int* a, long long na, const int* b, long long nb, int* out, long long merge_thr) {
    if (na + nb <= merge_thr) {
        merge_serial(a, na, b, nb, out);
        return;
    }
    if (na < nb) {  // split the longer run at its median
        std::swap(a, b);
        std::swap(na, nb);
    }
    const long long ma = na / 2;
    const long long mb = std::upper_bound(b, b + nb, a[ma]) - b;
#pragma omp task
    parallel_merge(a, ma, b, mb, out, merge_thr);
#pragma omp task
    parallel_merge(a + ma, na - ma, b + mb, nb - mb, out + ma + mb, merge_thr);
#pragma omp taskwait
}

// Returns 1 if the sorted result is in `a`, -1 if it is in `tmp` (the
// reference's ping-pong status convention, mergesort.cpp:146-195).
int merge_sort(int* a, int* tmp, long long n, long long sort_thr, long long merge_thr) {
    if (n <= sort_thr) {
        std::sort(a, a + n);
        return 1;
    }
    const long long h = n / 2;
    int sl = 0, sr = 0;
#pragma omp task shared(sl)
    sl = merge_sort(a, tmp, h, sort_thr, merge_thr);
#pragma omp task shared(sr)
    sr = merge_sort(a + h, tmp + h, n - h, sort_thr, merge_thr);
#pragma omp taskwait
    // bring both halves into the same buffer (copy-fixup when they disagree)
    if (sl != sr) {
        if (sr == -1) std::memcpy(a + h, tmp + h, (n - h) * sizeof(int));  // both halves now in a (sl == 1)
        else std::memcpy(tmp + h, a + h, (n - h) * sizeof(int));            // both halves now in tmp (sl == -1)
    }
    const int* src = sl == 1 ? a : tmp;
    int* dst = sl == 1 ? tmp : a;
    parallel_merge(src, h, src + h, n - h, dst, merge_thr);
    return -sl;
}

}  // namespace

CME_CPU_EXPORT int cme_cpu_radix_sort_u32(uint32_t* keys, uint32_t* tmp, long long n, int num_bits, int nblocks) {
    if (num_bits < 1 || num_bits > 16) return 1;
    if (nblocks <= 0) nblocks = std::max(1, omp_get_max_threads() * 4);
    uint32_t *in = keys, *out = tmp;
    int passes = 0;
    for (int shift = 0; shift < 32; shift += num_bits, ++passes) {
        radix_pass(in, out, n, shift, std::min(num_bits, 32 - shift), nblocks);
        std::swap(in, out);
    }
    if (in != keys) std::memcpy(keys, in, n * sizeof(uint32_t));
    return 0;
}

// Key-value LSD radix sort over the low `key_bits` bits (32 = full keys;
// fewer = a counting sort for small key ranges, Lecture16). Stable.
CME_CPU_EXPORT int cme_cpu_radix_sort_kv_u32(uint32_t* keys, uint32_t* ktmp, uint32_t* vals, uint32_t* vtmp,
                                             long long n, int num_bits, int key_bits) {
    if (num_bits < 1 || num_bits > 16 || key_bits < 1 || key_bits > 32) return 1;
    const int nblocks = std::max(1, omp_get_max_threads() * 4);
    uint32_t *in = keys, *out = ktmp, *vi = vals, *vo = vtmp;
    for (int shift = 0; shift < key_bits; shift += num_bits) {
        radix_pass(in, out, n, shift, std::min(num_bits, key_bits - shift), nblocks, vi, vo);
        std::swap(in, out);
        std::swap(vi, vo);
    }
    if (in != keys) {
        std::memcpy(keys, in, n * sizeof(uint32_t));
        std::memcpy(vals, vi, n * sizeof(uint32_t));
    }
    return 0;
}

CME_CPU_EXPORT int cme_cpu_radix_sort_serial_u32(uint32_t* keys, uint32_t* tmp, long long n, int num_bits) {
    if (num_bits < 1 || num_bits > 16) return 1;
    uint32_t *in = keys, *out = tmp;
    for (int shift = 0; shift < 32; shift += num_bits) {
        const int bits = std::min(num_bits, 32 - shift);
        const uint32_t nb = 1u << bits, mask = nb - 1;
        std::vector<uint64_t> cnt(nb + 1, 0);
        for (long long i = 0; i < n; ++i) ++cnt[((in[i] >> shift) & mask) + 1];
        for (uint32_t d = 0; d < nb; ++d) cnt[d + 1] += cnt[d];
        for (long long i = 0; i < n; ++i) out[cnt[(in[i] >> shift) & mask]++] = in[i];
        std::swap(in, out);
    }
    if (in != keys) std::memcpy(keys, in, n * sizeof(uint32_t));
    return 0;
}

CME_CPU_EXPORT int cme_cpu_merge_sort_i32(int* a, int* tmp, long long n, long long sort_thr, long long merge_thr,
                                          int* status) {
    int st = 1;
#pragma omp parallel
#pragma omp single
    st = merge_sort(a, tmp, n, std::max(1LL, sort_thr), std::max(2LL, merge_thr));
    *status = st;
    return 0;
}
