/*
 * armci.h -- the ARMCI subset on the strided pack/unpack + accumulate path,
 * as exported by libga_amd.so.
 *
 * Drop-in for /root/reference/comex/src-armci/armci.h for the calls GA's
 * global/src makes on this path (onesided.c:375-1453).  Every ARMCI_X is a weak
 * alias of PARMCI_X (as comex/src-armci/capi.c:14-27 does), so PMPI-style
 * interposers (comex/tools/armci_prof.c, GA's WAPI layer) keep working.
 * Constants are value-identical (armci.h:178-191).
 */
#ifndef _ARMCI_H
#define _ARMCI_H

#include <stdlib.h>

#if defined(__cplusplus) || defined(c_plusplus)
extern "C" {
#endif

/* armci.h:17-23 */
typedef struct {
    void **src_ptr_array;
    void **dst_ptr_array;
    int ptr_array_len;
    int bytes;
} armci_giov_t;
typedef long armci_size_t;
typedef int armci_hdl_t;       /* armci.h:250 */

#define ARMCI_ACC_OFF 36       /* armci.h:183-191 */
#define ARMCI_ACC_INT (ARMCI_ACC_OFF + 1)
#define ARMCI_ACC_DBL (ARMCI_ACC_OFF + 2)
#define ARMCI_ACC_FLT (ARMCI_ACC_OFF + 3)
#define ARMCI_ACC_CPL (ARMCI_ACC_OFF + 4)
#define ARMCI_ACC_DCP (ARMCI_ACC_OFF + 5)
#define ARMCI_ACC_LNG (ARMCI_ACC_OFF + 6)
#define ARMCI_MAX_STRIDE_LEVEL 8

#define ARMCI_INIT_HANDLE(hdl)

/* armci.h:26-30, 155-158 */
extern int ARMCI_Init();
extern int ARMCI_Init_args(int *argc, char ***argv);
extern int ARMCI_Initialized();
extern void ARMCI_Finalize();
extern void ARMCI_Barrier();
extern void ARMCI_Error(const char *msg, int code);
extern void ARMCI_Fence(int proc);
extern void ARMCI_AllFence();

/* contiguous + strided one-sided: armci.h:32-101 */
extern int ARMCI_Put(void *src, void *dst, int bytes, int proc);
extern int ARMCI_PutS(void *src_ptr, int src_stride_arr[], void *dst_ptr, int dst_stride_arr[],
                      int count[], int stride_levels, int proc);
extern int ARMCI_Acc(int optype, void *scale, void *src, void *dst, int bytes, int proc);
extern int ARMCI_AccS(int optype, void *scale, void *src_ptr, int src_stride_arr[],
                      void *dst_ptr, int dst_stride_arr[], int count[], int stride_levels,
                      int proc);
extern int ARMCI_Get(void *src, void *dst, int bytes, int proc);
extern int ARMCI_GetS(void *src_ptr, int src_stride_arr[], void *dst_ptr, int dst_stride_arr[],
                      int count[], int stride_levels, int proc);

/* vector: armci.h:103-118 */
extern int ARMCI_PutV(armci_giov_t darr[], int len, int proc);
extern int ARMCI_GetV(armci_giov_t darr[], int len, int proc);
extern int ARMCI_AccV(int op, void *scale, armci_giov_t darr[], int len, int proc);

/* non-blocking: armci.h:273-366 */
extern int ARMCI_NbPut(void *src, void *dst, int bytes, int proc, armci_hdl_t *nb_handle);
extern int ARMCI_NbPutS(void *src_ptr, int src_stride_arr[], void *dst_ptr, int dst_stride_arr[],
                        int count[], int stride_levels, int proc, armci_hdl_t *nb_handle);
extern int ARMCI_NbAccS(int optype, void *scale, void *src_ptr, int src_stride_arr[],
                        void *dst_ptr, int dst_stride_arr[], int count[], int stride_levels,
                        int proc, armci_hdl_t *nb_handle);
extern int ARMCI_NbGet(void *src, void *dst, int bytes, int proc, armci_hdl_t *nb_handle);
extern int ARMCI_NbGetS(void *src_ptr, int src_stride_arr[], void *dst_ptr, int dst_stride_arr[],
                        int count[], int stride_levels, int proc, armci_hdl_t *nb_handle);
extern int ARMCI_Wait(armci_hdl_t *nb_handle);
extern int ARMCI_Test(armci_hdl_t *nb_handle);
extern int ARMCI_WaitAll();
extern int ARMCI_WaitProc(int proc);

/* memory: armci.h:146-153 */
extern int ARMCI_Malloc(void *ptr_arr[], armci_size_t bytes);
extern int ARMCI_Malloc_memdev(void *ptr_arr[], armci_size_t bytes, const char *device);
extern int ARMCI_Free(void *ptr);
extern int ARMCI_Free_memdev(void *ptr);
extern void *ARMCI_Malloc_local(armci_size_t bytes);
extern int ARMCI_Free_local(void *ptr);

/* contiguity collapse used by the strided wrappers (comex/src-armci/armci.c:114) */
extern int armci_check_contiguous(int *src_stride, int *dst_stride, int *count, int n_stride);

/* profiling layer (comex/src-armci/parmci.h): same signatures, P-prefixed */
extern int PARMCI_Init();
extern int PARMCI_Init_args(int *argc, char ***argv);
extern int PARMCI_Initialized();
extern void PARMCI_Finalize();
extern void PARMCI_Barrier();
extern void PARMCI_Fence(int proc);
extern void PARMCI_AllFence();
extern int PARMCI_Put(void *src, void *dst, int bytes, int proc);
extern int PARMCI_PutS(void *src_ptr, int src_stride_arr[], void *dst_ptr, int dst_stride_arr[],
                       int count[], int stride_levels, int proc);
extern int PARMCI_Acc(int optype, void *scale, void *src, void *dst, int bytes, int proc);
extern int PARMCI_AccS(int optype, void *scale, void *src_ptr, int src_stride_arr[],
                       void *dst_ptr, int dst_stride_arr[], int count[], int stride_levels,
                       int proc);
extern int PARMCI_Get(void *src, void *dst, int bytes, int proc);
extern int PARMCI_GetS(void *src_ptr, int src_stride_arr[], void *dst_ptr, int dst_stride_arr[],
                       int count[], int stride_levels, int proc);
extern int PARMCI_PutV(armci_giov_t darr[], int len, int proc);
extern int PARMCI_GetV(armci_giov_t darr[], int len, int proc);
extern int PARMCI_AccV(int op, void *scale, armci_giov_t darr[], int len, int proc);
extern int PARMCI_NbPut(void *src, void *dst, int bytes, int proc, armci_hdl_t *nb_handle);
extern int PARMCI_NbPutS(void *src_ptr, int src_stride_arr[], void *dst_ptr, int dst_stride_arr[],
                         int count[], int stride_levels, int proc, armci_hdl_t *nb_handle);
extern int PARMCI_NbAccS(int optype, void *scale, void *src_ptr, int src_stride_arr[],
                         void *dst_ptr, int dst_stride_arr[], int count[], int stride_levels,
                         int proc, armci_hdl_t *nb_handle);
extern int PARMCI_NbGet(void *src, void *dst, int bytes, int proc, armci_hdl_t *nb_handle);
extern int PARMCI_NbGetS(void *src_ptr, int src_stride_arr[], void *dst_ptr, int dst_stride_arr[],
                         int count[], int stride_levels, int proc, armci_hdl_t *nb_handle);
extern int PARMCI_Wait(armci_hdl_t *nb_handle);
extern int PARMCI_Test(armci_hdl_t *nb_handle);
extern int PARMCI_WaitAll();
extern int PARMCI_WaitProc(int proc);
extern int PARMCI_Malloc(void *ptr_arr[], armci_size_t bytes);
extern int PARMCI_Malloc_memdev(void *ptr_arr[], armci_size_t bytes, const char *device);
extern int PARMCI_Free(void *ptr);
extern int PARMCI_Free_memdev(void *ptr);
extern void *PARMCI_Malloc_local(armci_size_t bytes);
extern int PARMCI_Free_local(void *ptr);

#if defined(__cplusplus) || defined(c_plusplus)
}
#endif

#endif /* _ARMCI_H */
