/*
 * armci_acc.h -- the legacy ARMCI accumulate kernels (armci/src/include/acc.h)
 * exported by libga_amd.so, MI355X-native.
 *
 * The reference's legacy ARMCI (armci/src) applies a strided accumulate 2-D
 * slab by 2-D slab: armci_acc_2D (armci/src/xfer/strided.c:257-328) turns the
 * byte counts and byte strides into element counts and element leading
 * dimensions (integer division, so a stride that is not a multiple of the
 * element size is truncated) and calls the c_?_accumulate_2d_ loop of
 * caccumulate.c for the type, column by column:
 *     A(r,c) += alpha * B(r,c)         r < rows, c < cols, A(ald,*), B(bld,*)
 * with the complex forms (caccumulate.c:183-184, 212-213)
 *     A.real += alpha.real*B.real - alpha.imag*B.imag
 *     A.imag += alpha.imag*B.real + alpha.real*B.imag
 * (bit-identical to comex acc.h's ordering: the products commute).  The _u_
 * forms are the 4-way unrolled loops (caccumulate.c:385-700); their results are
 * the same element for element.
 *
 * Here every entry point runs the 2-D patch as one strided accumulate kernel
 * on the GPU (the comex_accs path on this rank): A and B may be HBM, comex
 * segments, pinned or pageable host memory.  The call returns when A holds the
 * result, as the reference's loop does.  Requires comex_init / ARMCI_Init.
 */
#ifndef GA_AMD_ARMCI_ACC_H
#define GA_AMD_ARMCI_ACC_H

#if defined(__cplusplus) || defined(c_plusplus)
extern "C" {
#endif

typedef struct {
    float real;
    float imag;
} complex_t;

typedef struct {
    double real;
    double imag;
} dcomplex_t;

/* acc.h:15-42: A[0..rows) += alpha * B[0..rows) */
void c_d_accumulate_1d_(const double *alpha, double *A, const double *B, const int *rows);
void c_f_accumulate_1d_(const float *alpha, float *A, const float *B, const int *rows);
void c_c_accumulate_1d_(const complex_t *alpha, complex_t *A, const complex_t *B, const int *rows);
void c_z_accumulate_1d_(const dcomplex_t *alpha, dcomplex_t *A, const dcomplex_t *B, const int *rows);
void c_i_accumulate_1d_(const int *alpha, int *A, const int *B, const int *rows);
void c_l_accumulate_1d_(const long *alpha, long *A, const long *B, const int *rows);
void c_ll_accumulate_1d_(const long long *alpha, long long *A, const long long *B, const int *rows);

/* acc.h:43-91: column-major A(ald, cols) += alpha * B(bld, cols) over rows x cols */
void c_d_accumulate_2d_(const double *alpha, const int *rows, const int *cols, double *A, const int *ald,
                        const double *B, const int *bld);
void c_f_accumulate_2d_(const float *alpha, const int *rows, const int *cols, float *A, const int *ald,
                        const float *B, const int *bld);
void c_c_accumulate_2d_(const complex_t *alpha, const int *rows, const int *cols, complex_t *A, const int *ald,
                        const complex_t *B, const int *bld);
void c_z_accumulate_2d_(const dcomplex_t *alpha, const int *rows, const int *cols, dcomplex_t *A, const int *ald,
                        const dcomplex_t *B, const int *bld);
void c_i_accumulate_2d_(const int *alpha, const int *rows, const int *cols, int *A, const int *ald, const int *B,
                        const int *bld);
void c_l_accumulate_2d_(const long *alpha, const int *rows, const int *cols, long *A, const int *ald, const long *B,
                        const int *bld);
void c_ll_accumulate_2d_(const long long *alpha, const int *rows, const int *cols, long long *A, const int *ald,
                         const long long *B, const int *bld);

/* acc.h:93-141: the unrolled forms */
void c_d_accumulate_2d_u_(const double *alpha, const int *rows, const int *cols, double *A, const int *ald,
                          const double *B, const int *bld);
void c_f_accumulate_2d_u_(const float *alpha, const int *rows, const int *cols, float *A, const int *ald,
                          const float *B, const int *bld);
void c_c_accumulate_2d_u_(const complex_t *alpha, const int *rows, const int *cols, complex_t *A, const int *ald,
                          const complex_t *B, const int *bld);
void c_z_accumulate_2d_u_(const dcomplex_t *alpha, const int *rows, const int *cols, dcomplex_t *A,
                          const int *ald, const dcomplex_t *B, const int *bld);
void c_i_accumulate_2d_u_(const int *alpha, const int *rows, const int *cols, int *A, const int *ald, const int *B,
                          const int *bld);
void c_l_accumulate_2d_u_(const long *alpha, const int *rows, const int *cols, long *A, const int *ald,
                          const long *B, const int *bld);
void c_ll_accumulate_2d_u_(const long long *alpha, const int *rows, const int *cols, long long *A, const int *ald,
                           const long long *B, const int *bld);

/* strided.c:257-328: one 2-D slab of a legacy strided accumulate on local
 * memory.  op is ARMCI_ACC_INT..ARMCI_ACC_LNG; bytes, src_stride and dst_stride
 * are in bytes and become element counts by integer division as in the
 * reference.  proc must be this rank (the reference reaches other ranks'
 * memory only through shared-memory mappings); lockit is accepted and unused:
 * one GPU stream already orders the accumulates of this process. */
void armci_acc_2D(int op, void *scale, int proc, void *src_ptr, void *dst_ptr, int bytes, int cols, int src_stride,
                  int dst_stride, int lockit);

#if defined(__cplusplus) || defined(c_plusplus)
}
#endif

#endif /* GA_AMD_ARMCI_ACC_H */
