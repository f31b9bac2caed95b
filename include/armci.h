/*
 * armci.h -- the ARMCI API exported by libga_amd.so.
 *
 * Drop-in for /root/reference/comex/src-armci/armci.h (+ parmci.h): the same
 * prototypes and constant values for every call GA's global/src links against
 * (tests/c/global_src_link.c references each one).  Every ARMCI_X that
 * comex/src-armci/capi.c wraps is a weak alias of PARMCI_X here too, so
 * PMPI-style interposers (comex/tools/armci_prof.c, GA's WAPI layer) keep
 * working.  Differences, all where the reference has no MPI-free meaning:
 *   - ARMCI_Init_mpi_comm / armci_group_comm take / return an MPI_Comm and are
 *     declared only when <mpi.h> was included first (no <mpi.h> dependency
 *     otherwise); the library itself has no MPI link dependency and uses the
 *     caller's MPI (MPICH ABI) only through these calls (ga_amd/csrc/mpi_bridge.cpp);
 *   - ARMCI_PutS_flag / _flag_dir / ARMCI_Put_flag are implemented (put, then
 *     the flag after remote completion) where the reference asserts;
 *   - ARMCI_Same_node returns 0 exactly as the reference (no direct load/store
 *     into another rank's segment from the host).
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

#define ARMCI_SWAP 10          /* armci.h:178-181 */
#define ARMCI_SWAP_LONG 11
#define ARMCI_FETCH_AND_ADD 12
#define ARMCI_FETCH_AND_ADD_LONG 13

#define ARMCI_ACC_OFF 36       /* armci.h:183-191 */
#define ARMCI_ACC_INT (ARMCI_ACC_OFF + 1)
#define ARMCI_ACC_DBL (ARMCI_ACC_OFF + 2)
#define ARMCI_ACC_FLT (ARMCI_ACC_OFF + 3)
#define ARMCI_ACC_CPL (ARMCI_ACC_OFF + 4)
#define ARMCI_ACC_DCP (ARMCI_ACC_OFF + 5)
#define ARMCI_ACC_LNG (ARMCI_ACC_OFF + 6)
#define ARMCI_MAX_STRIDE_LEVEL 8

#define ARMCI_INIT_HANDLE(hdl)

#define FAIL  -1               /* armci.h:166-173 */
#define FAIL2 -2
#define FAIL3 -3
#define FAIL4 -4
#define FAIL5 -5
#define FAIL6 -6
#define FAIL7 -7
#define FAIL8 -8

typedef int ARMCI_Group;       /* armci.h:254 */
typedef int armci_domain_t;    /* armci.h:232-233 */
#define ARMCI_DOMAIN_SMP 0

/* armci.h:384-397: non-collective memory */
typedef struct armci_meminfo_ds {
    char *armci_addr;
    char *addr;
    size_t size;
    int cpid;
    long idlist[128];
} armci_meminfo_t;

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

#ifdef MPI_VERSION
/* init over an external communicator (armci.h:28; armci.c:427-440): the
 * communicator's ranks are ARMCI's world; 1 on success */
extern int ARMCI_Init_mpi_comm(MPI_Comm comm);
/* the group's communicator (groups.c); world: a dup of the init communicator */
extern MPI_Comm armci_group_comm(ARMCI_Group *group);
#endif

/* flagged puts (armci.h:37-66) */
extern int ARMCI_Put_flag(void *src, void *dst, int bytes, int *f, int v, int proc);
extern int ARMCI_PutS_flag(void *src_ptr, int src_stride_arr[], void *dst_ptr, int dst_stride_arr[],
                           int count[], int stride_levels, int *flag, int val, int proc);
extern int ARMCI_PutS_flag_dir(void *src_ptr, int src_stride_arr[], void *dst_ptr, int dst_stride_arr[],
                               int count[], int stride_levels, int *flag, int val, int proc);

/* single values (armci.h:120-144) */
extern int ARMCI_PutValueInt(int src, void *dst, int proc);
extern int ARMCI_PutValueLong(long src, void *dst, int proc);
extern int ARMCI_PutValueFloat(float src, void *dst, int proc);
extern int ARMCI_PutValueDouble(double src, void *dst, int proc);
extern int ARMCI_GetValueInt(void *src, int proc);
extern long ARMCI_GetValueLong(void *src, int proc);
extern float ARMCI_GetValueFloat(void *src, int proc);
extern double ARMCI_GetValueDouble(void *src, int proc);
extern int ARMCI_NbPutValueInt(int src, void *dst, int proc, armci_hdl_t *nb_handle);
extern int ARMCI_NbPutValueLong(long src, void *dst, int proc, armci_hdl_t *nb_handle);
extern int ARMCI_NbPutValueFloat(float src, void *dst, int proc, armci_hdl_t *nb_handle);
extern int ARMCI_NbPutValueDouble(double src, void *dst, int proc, armci_hdl_t *nb_handle);

/* non-blocking vector (armci.h:312-331) */
extern int ARMCI_NbGetV(armci_giov_t darr[], int len, int proc, armci_hdl_t *nb_handle);
extern int ARMCI_NbPutV(armci_giov_t darr[], int len, int proc, armci_hdl_t *nb_handle);
extern int ARMCI_NbAccV(int op, void *scale, armci_giov_t darr[], int len, int proc, armci_hdl_t *nb_handle);
extern void ARMCI_SET_AGGREGATE_HANDLE(armci_hdl_t *nb_handle);
extern void ARMCI_UNSET_AGGREGATE_HANDLE(armci_hdl_t *nb_handle);

/* atomics, mutexes, locality (armci.h:155-164, 232-241) */
extern int ARMCI_Rmw(int op, void *ploc, void *prem, int extra, int proc);
extern int ARMCI_Create_mutexes(int num);
extern int ARMCI_Destroy_mutexes();
extern void ARMCI_Lock(int mutex, int proc);
extern void ARMCI_Unlock(int mutex, int proc);
extern int ARMCI_Same_node(int proc);
extern void ARMCI_Cleanup();
extern void ARMCI_Set_shm_limit(unsigned long shmemlimit);
extern int ARMCI_Uses_shm();
extern void ARMCI_Copy(void *src, void *dst, int n);
extern int armci_notify(int proc);
extern int armci_notify_wait(int proc, int *pval);
extern int armci_domain_nprocs(armci_domain_t domain, int id);
extern int armci_domain_id(armci_domain_t domain, int glob_proc_id);
extern int armci_domain_glob_proc_id(armci_domain_t domain, int id, int loc_proc_id);
extern int armci_domain_my_id(armci_domain_t domain);
extern int armci_domain_count(armci_domain_t domain);
extern int armci_domain_same_id(armci_domain_t domain, int proc);

/* processor groups (armci.h:255-270; comex/src-armci/groups.c) */
extern void ARMCI_GroupFence(ARMCI_Group *group);
extern void ARMCI_Group_create(int n, int *pid_list, ARMCI_Group *group_out);
extern void ARMCI_Group_create_child(int n, int *pid_list, ARMCI_Group *group_out, ARMCI_Group *group_parent);
extern void ARMCI_Group_free(ARMCI_Group *group);
extern int ARMCI_Group_rank(ARMCI_Group *group, int *rank);
extern void ARMCI_Group_size(ARMCI_Group *group, int *size);
extern void ARMCI_Group_set_default(ARMCI_Group *group);
extern void ARMCI_Group_get_default(ARMCI_Group *group_out);
extern void ARMCI_Group_get_world(ARMCI_Group *group_out);
extern int ARMCI_Absolute_id(ARMCI_Group *group, int group_rank);
extern int ARMCI_Uses_shm_grp(ARMCI_Group *group);
extern int ARMCI_Malloc_group(void *ptr_arr[], armci_size_t bytes, ARMCI_Group *group);
extern int ARMCI_Malloc_group_memdev(void *ptr_arr[], armci_size_t bytes, ARMCI_Group *group, const char *device);
extern int ARMCI_Free_group(void *ptr, ARMCI_Group *group);

/* non-collective memory (armci.h:398-401) */
extern void ARMCI_Memget(size_t bytes, armci_meminfo_t *meminfo, int memflg);
extern void *ARMCI_Memat(armci_meminfo_t *meminfo, long offset);
extern void ARMCI_Memdt(armci_meminfo_t *meminfo, long offset);
extern void ARMCI_Memctl(armci_meminfo_t *meminfo);

/* strided copies between a local patch and a contiguous buffer (comex/src-armci/iterator.c:158-193):
 * write = patch -> buf (pack), read = buf -> patch (unpack) */
extern void armci_write_strided(void *ptr, int stride_levels, int stride_arr[], int count[], char *buf);
extern void armci_read_strided(void *ptr, int stride_levels, int stride_arr[], int count[], char *buf);

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
#ifdef MPI_VERSION
extern int PARMCI_Init_mpi_comm(MPI_Comm comm);
#endif
extern void PARMCI_GroupFence(ARMCI_Group *group);
extern int PARMCI_Create_mutexes(int num);
extern int PARMCI_Destroy_mutexes();
extern void PARMCI_Lock(int mutex, int proc);
extern void PARMCI_Unlock(int mutex, int proc);
extern int PARMCI_Rmw(int op, void *ploc, void *prem, int extra, int proc);
extern int PARMCI_Put_flag(void *src, void *dst, int bytes, int *f, int v, int proc);
extern int PARMCI_PutS_flag(void *src_ptr, int src_stride_arr[], void *dst_ptr, int dst_stride_arr[],
                            int count[], int stride_levels, int *flag, int val, int proc);
extern int PARMCI_PutS_flag_dir(void *src_ptr, int src_stride_arr[], void *dst_ptr, int dst_stride_arr[],
                                int count[], int stride_levels, int *flag, int val, int proc);
extern int PARMCI_PutValueInt(int src, void *dst, int proc);
extern int PARMCI_PutValueLong(long src, void *dst, int proc);
extern int PARMCI_PutValueFloat(float src, void *dst, int proc);
extern int PARMCI_PutValueDouble(double src, void *dst, int proc);
extern int PARMCI_GetValueInt(void *src, int proc);
extern long PARMCI_GetValueLong(void *src, int proc);
extern float PARMCI_GetValueFloat(void *src, int proc);
extern double PARMCI_GetValueDouble(void *src, int proc);
extern int PARMCI_NbPutValueInt(int src, void *dst, int proc, armci_hdl_t *nb_handle);
extern int PARMCI_NbPutValueLong(long src, void *dst, int proc, armci_hdl_t *nb_handle);
extern int PARMCI_NbPutValueFloat(float src, void *dst, int proc, armci_hdl_t *nb_handle);
extern int PARMCI_NbPutValueDouble(double src, void *dst, int proc, armci_hdl_t *nb_handle);
extern int PARMCI_NbGetV(armci_giov_t darr[], int len, int proc, armci_hdl_t *nb_handle);
extern int PARMCI_NbPutV(armci_giov_t darr[], int len, int proc, armci_hdl_t *nb_handle);
extern int PARMCI_NbAccV(int op, void *scale, armci_giov_t darr[], int len, int proc, armci_hdl_t *nb_handle);
extern void PARMCI_Memget(size_t bytes, armci_meminfo_t *meminfo, int memflg);
extern void *PARMCI_Memat(armci_meminfo_t *meminfo, long offset);
extern void PARMCI_Memdt(armci_meminfo_t *meminfo, long offset);
extern void PARMCI_Memctl(armci_meminfo_t *meminfo);
extern void PARMCI_Copy(void *src, void *dst, int n);
extern int parmci_notify(int proc);
extern int parmci_notify_wait(int proc, int *pval);

#if defined(__cplusplus) || defined(c_plusplus)
}
#endif

#endif /* _ARMCI_H */
