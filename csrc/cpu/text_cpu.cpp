// OpenMP CPU backend of the hw3 text kernels (the GPU versions are in
// csrc/hip/text.hip): byte histogram, digraph table, per-residue letter
// histograms, shifted-match counts (index of coincidence), sanitize
// (lower-case + keep a-z: stream compaction) and the Vigenere shift.
//
// Reference: the Thrust pipelines of hw/hw3/programming/create_cipher.cu:
// 111-142 and hw/hw3/solution/solve_cipher_solution.cu:131-200, plus the
// OpenMP CPU pattern of hw/hw_final/programming/fp.cu:130-152. Histograms are
// privatised per thread and merged (no atomics); compaction is count ->
// exclusive scan of per-thread counts -> write, so the output order is the
// input order.
#include <omp.h>

#include <cstdint>
#include <cstring>
#include <vector>

#include "cme213/cpu_common.h"

namespace {

// [begin, end) of thread t's contiguous share of n items
inline void share(long long n, int t, int nt, long long* b, long long* e) {
    *b = n * t / nt;
    *e = n * (t + 1) / nt;
}

template <typename Fn>
void privatised_hist(long long n, int nbins, int32_t* out, Fn&& body) {
    const int nt = omp_get_max_threads();
    std::vector<int64_t> local((size_t)nt * nbins, 0);
#pragma omp parallel num_threads(nt)
    {
        const int t = omp_get_thread_num(), tn = omp_get_num_threads();
        long long b, e;
        share(n, t, tn, &b, &e);
        body(b, e, local.data() + (size_t)t * nbins);
    }
#pragma omp parallel for schedule(static)
    for (int k = 0; k < nbins; ++k) {
        int64_t s = 0;
        for (int t = 0; t < nt; ++t) s += local[(size_t)t * nbins + k];
        out[k] = (int32_t)s;
    }
}

}  // namespace

CME_CPU_EXPORT int cme_cpu_histogram_u8(const uint8_t* x, long long n, int lo, int nbins, int32_t* out) {
    if (nbins <= 0) return 1;
    privatised_hist(n, nbins, out, [&](long long b, long long e, int64_t* h) {
        for (long long i = b; i < e; ++i) {
            const int v = (int)x[i] - lo;
            if (v >= 0 && v < nbins) ++h[v];
        }
    });
    return 0;
}

// 26x26 counts of the non-overlapping pairs (t[2i], t[2i+1]) of letters
CME_CPU_EXPORT int cme_cpu_digraphs(const uint8_t* t, long long n, int32_t* out) {
    privatised_hist(n / 2, 676, out, [&](long long b, long long e, int64_t* h) {
        for (long long i = b; i < e; ++i) {
            const int a = (int)t[2 * i] - 'a', c = (int)t[2 * i + 1] - 'a';
            if (a >= 0 && a < 26 && c >= 0 && c < 26) ++h[a * 26 + c];
        }
    });
    return 0;
}

// [period][26] letter counts of t[r::period]
CME_CPU_EXPORT int cme_cpu_residue_hist(const uint8_t* t, long long n, int period, int32_t* out) {
    if (period <= 0) return 1;
    privatised_hist(n, period * 26, out, [&](long long b, long long e, int64_t* h) {
        long long r = b % period;
        for (long long i = b; i < e; ++i) {
            const int v = (int)t[i] - 'a';
            if (v >= 0 && v < 26) ++h[r * 26 + v];
            if (++r == period) r = 0;
        }
    });
    return 0;
}

// counts[k] = #{i : t[i] == t[i + s0 + k]}, k in [0, ns)
CME_CPU_EXPORT int cme_cpu_match_count(const uint8_t* t, long long n, int s0, int ns, int64_t* out) {
    for (int k = 0; k < ns; ++k) {
        const long long s = (long long)s0 + k;
        int64_t c = 0;
        if (s < n) {
#pragma omp parallel for reduction(+ : c) schedule(static)
            for (long long i = 0; i < n - s; ++i) c += (t[i] == t[i + s]);
        }
        out[k] = c;
    }
    return 0;
}

// lower-case, keep a-z; *count = kept bytes (out holds them in input order)
CME_CPU_EXPORT int cme_cpu_sanitize(const uint8_t* raw, long long n, uint8_t* out, long long* count) {
    const int nt = omp_get_max_threads();
    std::vector<long long> off(nt + 1, 0);
#pragma omp parallel num_threads(nt)
    {
        const int t = omp_get_thread_num(), tn = omp_get_num_threads();
        long long b, e;
        share(n, t, tn, &b, &e);
        long long c = 0;
        for (long long i = b; i < e; ++i) {
            const uint8_t r = raw[i];
            c += (r >= 'a' && r <= 'z') || (r >= 'A' && r <= 'Z');
        }
        off[t + 1] = c;
#pragma omp barrier
#pragma omp single
        for (int k = 1; k <= tn; ++k) off[k] += off[k - 1];
        long long w = off[t];
        for (long long i = b; i < e; ++i) {
            const uint8_t r = raw[i];
            if (r >= 'A' && r <= 'Z')
                out[w++] = r + 32;
            else if (r >= 'a' && r <= 'z')
                out[w++] = r;
        }
#pragma omp single
        *count = off[tn];
    }
    return 0;
}

// out[i] = 'a' + (t[i] - 'a' + sign * shifts[i % period]) mod 26
CME_CPU_EXPORT int cme_cpu_vigenere(const uint8_t* t, long long n, const int32_t* shifts, int period, int sign,
                                    uint8_t* out) {
    if (period <= 0) return 1;
#pragma omp parallel
    {
        const int th = omp_get_thread_num(), tn = omp_get_num_threads();
        long long b, e;
        share(n, th, tn, &b, &e);
        long long r = b % period;
        for (long long i = b; i < e; ++i) {
            int v = ((int)t[i] - 'a' + sign * (shifts[r] % 26)) % 26;
            if (v < 0) v += 26;
            out[i] = (uint8_t)('a' + v);
            if (++r == period) r = 0;
        }
    }
    return 0;
}
