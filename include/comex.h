/*
 * comex.h -- ComEx C API of the MI355X-native strided pack/unpack + typed
 * accumulate library (libga_amd.so).
 *
 * Drop-in for /root/reference/comex/src-common/comex.h: same prototypes, same
 * constant values, same argument conventions (count[0] in BYTES, count[1..L]
 * in elements, strides in bytes as int, stride_levels = ndim-1 <= 7).  Each
 * entry point cites the reference declaration it replaces.  Differences:
 *   - `extern "C"` (the reference writes `extern "c"`, comex.h:10, which does
 *     not compile as C++);
 *   - no <mpi.h> dependency: comex_init_comm / comex_group_comm are declared
 *     only when the includer has already included <mpi.h> (MPICH ABI; the
 *     library looks the caller's MPI functions up at the call);
 *   - segments from comex_malloc live in the owner GPU's HBM (hipMalloc),
 *     exported to the other ranks of the node by IPC handle.
 */
#ifndef _COMEX_H
#define _COMEX_H

#include <stdlib.h>

#if defined(__cplusplus) || defined(c_plusplus)
extern "C" {
#endif

/* comex.h:13-18 */
typedef struct {
    void **src;  /* array of source starting addresses */
    void **dst;  /* array of destination starting addresses */
    int count;   /* size of address arrays (src[count],dst[count]) */
    int bytes;   /* length in bytes for each src[i]/dst[i] pair */
} comex_giov_t;

typedef int comex_request_t;   /* comex.h:20 */
typedef int comex_group_t;     /* comex.h:22 */

#define COMEX_GROUP_WORLD 0    /* comex.h:24-25 */
#define COMEX_GROUP_NULL -1

#define COMEX_SUCCESS 0        /* comex.h:27-28 */
#define COMEX_FAILURE 1

#define COMEX_SWAP 10          /* comex.h:30-33 */
#define COMEX_SWAP_LONG 11
#define COMEX_FETCH_AND_ADD 12
#define COMEX_FETCH_AND_ADD_LONG 13

#define COMEX_ACC_OFF 36       /* comex.h:35-41 */
#define COMEX_ACC_INT (COMEX_ACC_OFF + 1)
#define COMEX_ACC_DBL (COMEX_ACC_OFF + 2)
#define COMEX_ACC_FLT (COMEX_ACC_OFF + 3)
#define COMEX_ACC_CPL (COMEX_ACC_OFF + 4)
#define COMEX_ACC_DCP (COMEX_ACC_OFF + 5)
#define COMEX_ACC_LNG (COMEX_ACC_OFF + 6)

#define COMEX_MAX_STRIDE_LEVEL 8   /* comex.h:43 */

/* init / teardown: comex.h:50-88 */
extern int comex_init();
extern int comex_init_args(int *argc, char ***argv);
#ifdef MPI_VERSION
/* comex.h:58 (comex.c:726-730): the communicator's ranks are ComEx's world */
extern int comex_init_comm(MPI_Comm comm);
#endif
extern int comex_initialized();
extern int comex_finalize();
extern void comex_error(const char *msg, int code);

/* groups: comex.h:107-186 */
extern int comex_group_create(int n, int *pid_list, comex_group_t group, comex_group_t *new_group);
extern int comex_group_free(comex_group_t group);
extern int comex_group_rank(comex_group_t group, int *rank);
extern int comex_group_size(comex_group_t group, int *size);
extern int comex_group_translate_world(comex_group_t group, int group_rank, int *world_rank);
/* comex.h:159: ranks of group_from in group_to (MPI_UNDEFINED = -32766 if absent) */
extern int comex_group_translate_ranks(int n, comex_group_t group_from, int *ranks_from,
                                       comex_group_t group_to, int *ranks_to);
#ifdef MPI_VERSION
/* comex.h:147: the group's communicator; only after comex_init_comm (a runtime
 * bootstrapped without MPI has none, and the call aborts) */
extern int comex_group_comm(comex_group_t group, MPI_Comm *comm);
#endif
extern int comex_barrier(comex_group_t group);

/* put: comex.h:199-302 */
extern int comex_put(void *src, void *dst, int bytes, int proc, comex_group_t group);
extern int comex_puts(void *src, int *src_stride, void *dst, int *dst_stride,
                      int *count, int stride_levels, int proc, comex_group_t group);
extern int comex_putv(comex_giov_t *darr, int len, int proc, comex_group_t group);
extern int comex_nbput(void *src, void *dst, int bytes, int proc, comex_group_t group,
                       comex_request_t *nb_handle);
extern int comex_nbputs(void *src, int *src_stride, void *dst, int *dst_stride,
                        int *count, int stride_levels, int proc, comex_group_t group,
                        comex_request_t *nb_handle);
extern int comex_nbputv(comex_giov_t *darr, int len, int proc, comex_group_t group,
                        comex_request_t *nb_handle);

/* accumulate: comex.h:305-413 -- the hot path */
extern int comex_acc(int op, void *scale, void *src, void *dst, int bytes,
                     int proc, comex_group_t group);
extern int comex_accs(int op, void *scale, void *src, int *src_stride,
                      void *dst, int *dst_stride, int *count, int stride_levels,
                      int proc, comex_group_t group);
extern int comex_accv(int op, void *scale, comex_giov_t *darr, int len,
                      int proc, comex_group_t group);
extern int comex_nbacc(int op, void *scale, void *src, void *dst, int bytes,
                       int proc, comex_group_t group, comex_request_t *nb_handle);
extern int comex_nbaccs(int op, void *scale, void *src, int *src_stride,
                        void *dst, int *dst_stride, int *count, int stride_levels,
                        int proc, comex_group_t group, comex_request_t *nb_handle);
extern int comex_nbaccv(int op, void *scale, comex_giov_t *darr, int len,
                        int proc, comex_group_t group, comex_request_t *nb_handle);

/* get: comex.h:426-521 */
extern int comex_get(void *src, void *dst, int bytes, int proc, comex_group_t group);
extern int comex_gets(void *src, int *src_stride, void *dst, int *dst_stride,
                      int *count, int stride_levels, int proc, comex_group_t group);
extern int comex_getv(comex_giov_t *darr, int len, int proc, comex_group_t group);
extern int comex_nbget(void *src, void *dst, int bytes, int proc, comex_group_t group,
                       comex_request_t *nb_handle);
extern int comex_nbgets(void *src, int *src_stride, void *dst, int *dst_stride,
                        int *count, int stride_levels, int proc, comex_group_t group,
                        comex_request_t *nb_handle);
extern int comex_nbgetv(comex_giov_t *darr, int len, int proc, comex_group_t group,
                        comex_request_t *nb_handle);

/* memory: comex.h:528-580.  comex_malloc is collective over `group`; ptr_arr[r]
 * receives rank r's segment address (in r's address space, as in the
 * reference); the segment is HBM on r's GPU.  comex_malloc_local returns
 * pinned, device-mapped host memory. */
extern int comex_malloc(void **ptr_arr, size_t bytes, comex_group_t group);
extern int comex_malloc_mem_dev(void **ptr_arr, size_t bytes, comex_group_t group,
                                const char *device);
extern int comex_free(void *ptr, comex_group_t group);
extern int comex_free_dev(void *ptr, comex_group_t group);
extern void *comex_malloc_local(size_t bytes);
extern int comex_free_local(void *ptr);

/* atomics and mutexes: comex.h:607-670.  comex_rmw is applied by the owner of
 * prem (its GPU, behind every earlier operation on those bytes); mutexes are
 * words in the owner node's shared memory (at most 4096 per rank). */
extern int comex_create_mutexes(int num);
extern int comex_destroy_mutexes();
extern int comex_lock(int mutex, int proc);
extern int comex_unlock(int mutex, int proc);
extern int comex_rmw(int op, void *ploc, void *prem, int extra, int proc, comex_group_t group);

/* completion: comex.h:588-709 */
extern int comex_fence_proc(int proc, comex_group_t group);
extern int comex_fence_all(comex_group_t group);
extern int comex_wait(comex_request_t *nb_handle);
extern int comex_test(comex_request_t *nb_handle, int *status);
extern int comex_wait_all(comex_group_t group);
extern int comex_wait_proc(int proc, comex_group_t group);

#if defined(__cplusplus) || defined(c_plusplus)
}
#endif

#endif /* _COMEX_H */
