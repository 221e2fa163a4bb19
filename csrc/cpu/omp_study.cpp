// OpenMP semantics study (slides/Lecture13-15): loop schedules on an
// imbalanced iteration space, and task-based (fork/join) vs parallel-for
// reductions. Times come from omp_get_wtime (the hw4 harness's timer).
#include <omp.h>

#include <cmath>

#include "cme213/cpu_common.h"

namespace {

// iteration i costs O(i * work / n) flops: triangular imbalance
inline double busy(long long i, long long n, int work) {
    const long long reps = 1 + (i * work) / n;
    double x = 1.0 + 1e-9 * (double)i;
    for (long long r = 0; r < reps; ++r) x = x * 1.0000001 + 1e-7;
    return x;
}

double task_sum(const double* x, long long n, long long cutoff) {
    if (n <= cutoff) {
        double s = 0.0;
        for (long long i = 0; i < n; ++i) s += x[i];
        return s;
    }
    double a = 0.0, b = 0.0;
    const long long h = n / 2;
#pragma omp task shared(a) firstprivate(x, h, cutoff)
    a = task_sum(x, h, cutoff);
#pragma omp task shared(b) firstprivate(x, n, h, cutoff)
    b = task_sum(x + h, n - h, cutoff);
#pragma omp taskwait
    return a + b;
}

}  // namespace

// schedule: 0 static, 1 static with chunk, 2 dynamic, 3 guided. Writes the
// elapsed seconds and a checksum (so the work is not optimised away).
CME_CPU_EXPORT int cme_cpu_omp_schedule(long long n, int work, int schedule, int chunk, int threads, double* seconds,
                                        double* checksum) {
    if (threads > 0) omp_set_num_threads(threads);
    double s = 0.0;
    const double t0 = omp_get_wtime();
    switch (schedule) {
        case 0:
#pragma omp parallel for schedule(static) reduction(+ : s)
            for (long long i = 0; i < n; ++i) s += busy(i, n, work);
            break;
        case 1:
#pragma omp parallel for schedule(static, chunk) reduction(+ : s)
            for (long long i = 0; i < n; ++i) s += busy(i, n, work);
            break;
        case 2:
#pragma omp parallel for schedule(dynamic, chunk) reduction(+ : s)
            for (long long i = 0; i < n; ++i) s += busy(i, n, work);
            break;
        case 3:
#pragma omp parallel for schedule(guided, chunk) reduction(+ : s)
            for (long long i = 0; i < n; ++i) s += busy(i, n, work);
            break;
        default: return 1;
    }
    *seconds = omp_get_wtime() - t0;
    *checksum = s;
    return 0;
}

// Sum of x[0..n): mode 0 parallel-for reduction, 1 recursive tasks
// (parallel + single + task/taskwait, the hw4 merge-sort pattern).
CME_CPU_EXPORT int cme_cpu_omp_sum(const double* x, long long n, int mode, long long cutoff, double* out,
                                   double* seconds) {
    const double t0 = omp_get_wtime();
    double s = 0.0;
    if (mode == 0) {
#pragma omp parallel for reduction(+ : s)
        for (long long i = 0; i < n; ++i) s += x[i];
    } else {
#pragma omp parallel
#pragma omp single
        s = task_sum(x, n, cutoff > 0 ? cutoff : 1 << 16);
    }
    *seconds = omp_get_wtime() - t0;
    *out = s;
    return 0;
}
