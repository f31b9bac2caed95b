/*
 * ga_amd_diag.h -- libga_amd_diag.so: measurement helpers over libga_amd.so's
 * public ABI (bench.py, tools/).  Not part of the drop-in boundary: a GA build
 * neither links nor needs it.
 */
#ifndef GA_AMD_DIAG_H
#define GA_AMD_DIAG_H

#if defined(__cplusplus)
extern "C" {
#endif

/* `steps` blocking comex_accs calls issued from C, the k-th on pointer set
 * k % nsets (srcs[k], dsts[k]); the elapsed wall-clock ns, 0 if a call failed.
 * The rate a C or Fortran caller (GA's NGA_Acc -> ARMCI_AccS) sees, without the
 * Python interpreter's per-call cost. */
unsigned long long gaamd_time_blocking_accs(int op, void *scale, void *const *srcs, int *ss, void *const *dsts,
                                            int *ds, int *count, int levels, int proc, int nsets, int steps);

#if defined(__cplusplus)
}
#endif

#endif /* GA_AMD_DIAG_H */
