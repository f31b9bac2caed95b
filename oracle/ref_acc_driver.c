/*
 * ref_acc_driver.c -- thin C entry points around the REFERENCE's own typed
 * accumulate kernel, compiled from the reference source where it lies:
 *
 *     #include "acc.h"   ->  /root/reference/comex/src-common/acc.h:106-154
 *
 * TEST INFRASTRUCTURE ONLY (parity checker / CPU baseline).  Built by
 * oracle/Makefile into oracle/_ref/libref_acc.so (git-ignored); never linked by
 * the product library.
 *
 * acc.h is a header of static inline functions; it needs only <mpi.h> (pulled
 * in by comex.h; MPICH's header is present in the image at /opt/conda/include,
 * no MPI symbol is referenced) and the configure results passed as -D flags:
 * HAVE_BLAS=0 (the reference's CMake default, ENABLE_BLAS OFF), SIZEOF_INT=4,
 * SIZEOF_LONG=8, BLAS_SIZE=8.  The rest of the MPI-PR transport (comex.c) needs
 * the MPI library and its generated config, so it is not built here; the
 * odometer below is the restatement of comex.c:6936-6961 (nb_accs per-row
 * loop) that drives the reference _acc exactly as nb_acc does for self/SMP
 * targets (comex.c:6228-6260).
 */
#include <assert.h>
#include <string.h>
#include "acc.h"

int ref_acc(int op, int bytes, void *dst, const void *src, const void *scale)
{
    _acc(op, bytes, dst, src, scale);
    return 0;
}

int ref_accs(int op, const void *scale, const char *src, const int *src_stride,
             char *dst, const int *dst_stride, const int *count, int stride_levels)
{
    int i, j;
    long src_idx, dst_idx;
    int n1dim;
    int src_bvalue[7], src_bunit[7];
    int dst_bvalue[7], dst_bunit[7];

    if (0 == stride_levels) {
        _acc(op, count[0], dst, src, scale);
        return 0;
    }
    n1dim = 1;
    for (i = 1; i <= stride_levels; i++) n1dim *= count[i];
    src_bvalue[0] = 0; src_bvalue[1] = 0; src_bunit[0] = 1; src_bunit[1] = 1;
    dst_bvalue[0] = 0; dst_bvalue[1] = 0; dst_bunit[0] = 1; dst_bunit[1] = 1;
    for (i = 2; i <= stride_levels; i++) {
        src_bvalue[i] = 0;
        dst_bvalue[i] = 0;
        src_bunit[i] = src_bunit[i - 1] * count[i - 1];
        dst_bunit[i] = dst_bunit[i - 1] * count[i - 1];
    }
    for (i = 0; i < n1dim; i++) {
        src_idx = 0;
        dst_idx = 0;
        for (j = 1; j <= stride_levels; j++) {
            src_idx += (long)src_bvalue[j] * (long)src_stride[j - 1];
            if ((i + 1) % src_bunit[j] == 0) src_bvalue[j]++;
            if (src_bvalue[j] > (count[j] - 1)) src_bvalue[j] = 0;
        }
        for (j = 1; j <= stride_levels; j++) {
            dst_idx += (long)dst_bvalue[j] * (long)dst_stride[j - 1];
            if ((i + 1) % dst_bunit[j] == 0) dst_bvalue[j]++;
            if (dst_bvalue[j] > (count[j] - 1)) dst_bvalue[j] = 0;
        }
        _acc(op, count[0], dst + dst_idx, src + src_idx, scale);
    }
    return 0;
}

#include "mt_split.h"

static int ref_esize(int op)
{
    switch (op) {
    case COMEX_ACC_INT: return sizeof(int);
    case COMEX_ACC_DBL: return sizeof(double);
    case COMEX_ACC_FLT: return sizeof(float);
    case COMEX_ACC_CPL: return sizeof(SingleComplex);
    case COMEX_ACC_DCP: return sizeof(DoubleComplex);
    case COMEX_ACC_LNG: return sizeof(long);
    }
    return 1;
}

/* P workers on P slabs of the patch (bench.py CPU baseline) */
int ref_accs_mt(int op, const void *scale, const char *src, const int *src_stride,
                char *dst, const int *dst_stride, const int *count, int stride_levels,
                int nthreads)
{
    return mt_accs(ref_accs, ref_esize(op), op, scale, src, src_stride, dst, dst_stride, count,
                   stride_levels, nthreads);
}

/* io-vector accumulate to a self/SMP target: one _acc per (src[i], dst[i]) pair,
 * as nb_accv does for such targets (comex.c:7327-7400 -> nb_acc 6228-6260) */
int ref_accv(int op, const void *scale, void *const *src, void *const *dst, long n, int bytes)
{
    long i;
    for (i = 0; i < n; i++) _acc(op, bytes, dst[i], src[i], scale);
    return 0;
}
