// Thread policy of the OpenMP CPU backend (the reference's OMP_NUM_THREADS
// sweeps, hw/hw4/programming/pa4.pbs:21-29): the team size every entry point
// uses, settable at run time, and what the runtime was started with.
#include <omp.h>
#include <stdlib.h>
#include <string.h>

#include "cme213/cpu_common.h"

// threads: the team size of the next parallel region; procs: processors the
// runtime sees; policy (16 bytes): OMP_WAIT_POLICY / GOMP_SPINCOUNT as the
// runtime read them at load ("passive", "active", "spin=<n>" or "default")
CME_CPU_EXPORT int cme_cpu_runtime_info(int* threads, int* procs, char* policy) {
    *threads = omp_get_max_threads();
    *procs = omp_get_num_procs();
    const char* w = getenv("OMP_WAIT_POLICY");
    const char* s = getenv("GOMP_SPINCOUNT");
    if (w && *w) {
        strncpy(policy, (w[0] == 'p' || w[0] == 'P') ? "passive" : "active", 15);
    } else if (s && *s) {
        strncpy(policy, "spin=", 15);
        strncat(policy, s, 9);
    } else {
        strncpy(policy, "default", 15);
    }
    policy[15] = 0;
    return 0;
}

// team size of every later parallel region (n >= 1)
CME_CPU_EXPORT int cme_cpu_set_threads(int n) {
    if (n < 1) return 1;
    omp_set_num_threads(n);
    return 0;
}
