// diag.cpp -- libga_amd_diag.so: measurement helpers for bench.py and tools/, over
// libga_amd.so's public ABI only (include/ga_amd_diag.h).  Kept out of the product
// library: nothing a GA build links depends on it.
#include "../../include/comex.h"
#include "../../include/ga_amd_diag.h"
#include <time.h>

extern "C" unsigned long long gaamd_time_blocking_accs(int op, void *scale, void *const *srcs, int *ss,
                                                       void *const *dsts, int *ds, int *count, int levels, int proc,
                                                       int nsets, int steps) {
    if (nsets <= 0 || steps <= 0) return 0;
    timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < steps; ++i)
        if (comex_accs(op, scale, srcs[i % nsets], ss, dsts[i % nsets], ds, count, levels, proc, COMEX_GROUP_WORLD) !=
            COMEX_SUCCESS)
            return 0;
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (unsigned long long)(t1.tv_sec - t0.tv_sec) * 1000000000ull + (unsigned long long)(t1.tv_nsec - t0.tv_nsec);
}
