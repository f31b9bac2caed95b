// armci.cpp -- ARMCI over the MI355X ComEx runtime (include/armci.h).
//
// Reference: comex/src-armci/armci.c (PARMCI_* over comex_*) and capi.c
// (ARMCI_* as weak wrappers of PARMCI_* for PMPI-style profiling).
//   PARMCI_AccS/GetS/PutS  armci.c:225-239, 335-349, 682-697: a patch that
//     armci_check_contiguous() (armci.c:114-170) proves contiguous goes to the
//     1-D comex_acc/get/put of prod(count) bytes, everything else to comex_*s.
//   PARMCI_NbAccS/NbGetS/NbPutS armci.c:553-640: same, non-blocking.
#include "../../include/armci.h"
#include "../../include/comex.h"
#include "runtime.hpp"
#include <string.h>

extern "C" {

// groups.c:10: ARMCI's default processor group (the world group until GA sets one)
int ARMCI_Default_Proc_Group = 0;

// armci.c:114-170 ("#if 1" CMX-merge variant): physical leading dims are
// src_ld[i] = stride[i]/stride[i-1]; contiguous iff every dimension below the
// first partial one is full and everything above it has count 1.
int armci_check_contiguous(int *src_stride, int *dst_stride, int *count, int n_stride) {
    int ret = 1, stridelen = 1, gap = 0;
    int src_ld[8] = {0}, dst_ld[8] = {0};
    if (n_stride > 0) {
        src_ld[0] = src_stride[0];
        dst_ld[0] = dst_stride[0];
    }
    for (int i = 1; i < n_stride; ++i) {
        src_ld[i] = src_stride[i] / src_stride[i - 1];
        dst_ld[i] = dst_stride[i] / dst_stride[i - 1];
    }
    for (int i = 0; i < n_stride; ++i) {
        const long prod = (long)stridelen * count[i];
        if (stridelen != 0 && (prod > 2147483647L || prod < -2147483647L - 1)) { ret = 0; break; }   // int overflow guard
        stridelen = (int)prod;
        const bool partial = count[i] < src_ld[i] || count[i] < dst_ld[i];
        if (partial && gap == 1) { ret = 0; break; }
        if (partial) gap = 1;
        else if (count[i] != 1 && gap == 1) { ret = 0; break; }
    }
    if (gap == 1 && ret == 1 && n_stride > 0 && count[n_stride] != 1) ret = 0;
    return ret;
}

static int contiguous_bytes(int *count, int stride_levels) {
    long lcount = 1;
    for (int i = 0; i <= stride_levels; ++i) lcount *= count[i];
    return (int)lcount;   // the reference's int product (armci.c:231-233)
}

// The reference collapses a contiguous patch to one comex_acc/put/get of
// (int)prod(count) bytes (armci.c:231-233); above 2 GiB that product wraps and
// the call moves the wrong number of bytes.  Patches
// that large -- a whole 8 GiB GA block of a 32768^2 f64 array on one GPU -- keep
// the strided path instead, which computes what the collapse means.
static bool collapse(int *ss, int *ds, int *count, int levels) {
    if (!armci_check_contiguous(ss, ds, count, levels)) return false;
    long lcount = 1;
    for (int i = 0; i <= levels; ++i) lcount *= count[i];
    return lcount <= 2147483647L;
}

int PARMCI_Init() {
    ARMCI_Default_Proc_Group = 0;
    return comex_init();
}
int PARMCI_Init_args(int *argc, char ***argv) {
    ARMCI_Default_Proc_Group = 0;
    return comex_init_args(argc, argv);
}
// PARMCI_Init_mpi_comm / armci_group_comm: mpi_bridge.cpp (MPI_Comm in the signature)
int PARMCI_Initialized() { return comex_initialized(); }
void PARMCI_Finalize() { comex_finalize(); }
void PARMCI_Barrier() { comex_barrier(ARMCI_Default_Proc_Group); }
void PARMCI_GroupFence(ARMCI_Group *group) { comex_fence_all(*group > 0 ? *group : COMEX_GROUP_WORLD); }
void PARMCI_Fence(int proc) { comex_fence_proc(proc, COMEX_GROUP_WORLD); }
void PARMCI_AllFence() { comex_fence_all(COMEX_GROUP_WORLD); }
void ARMCI_Error(const char *msg, int code) { comex_error(msg, code); }

int PARMCI_Put(void *src, void *dst, int bytes, int proc) {
    return comex_put(src, dst, bytes, proc, COMEX_GROUP_WORLD);
}
int PARMCI_PutS(void *src, int *ss, void *dst, int *ds, int *count, int levels, int proc) {
    if (collapse(ss, ds, count, levels))
        return comex_put(src, dst, contiguous_bytes(count, levels), proc, COMEX_GROUP_WORLD);
    return comex_puts(src, ss, dst, ds, count, levels, proc, COMEX_GROUP_WORLD);
}
int PARMCI_Acc(int op, void *scale, void *src, void *dst, int bytes, int proc) {
    return comex_acc(op, scale, src, dst, bytes, proc, COMEX_GROUP_WORLD);
}
int PARMCI_AccS(int op, void *scale, void *src, int *ss, void *dst, int *ds, int *count, int levels, int proc) {
    if (collapse(ss, ds, count, levels))
        return comex_acc(op, scale, src, dst, contiguous_bytes(count, levels), proc, COMEX_GROUP_WORLD);
    return comex_accs(op, scale, src, ss, dst, ds, count, levels, proc, COMEX_GROUP_WORLD);
}
int PARMCI_Get(void *src, void *dst, int bytes, int proc) {
    return comex_get(src, dst, bytes, proc, COMEX_GROUP_WORLD);
}
int PARMCI_GetS(void *src, int *ss, void *dst, int *ds, int *count, int levels, int proc) {
    if (collapse(ss, ds, count, levels))
        return comex_get(src, dst, contiguous_bytes(count, levels), proc, COMEX_GROUP_WORLD);
    return comex_gets(src, ss, dst, ds, count, levels, proc, COMEX_GROUP_WORLD);
}

// armci_giov_t and comex_giov_t have the same layout (armci.c:175-184 converts
// field by field); copy so the types stay independent.
static std::vector<comex_giov_t> to_comex(armci_giov_t *a, int len) {
    std::vector<comex_giov_t> v((size_t)len);
    for (int i = 0; i < len; ++i) {
        v[i].src = a[i].src_ptr_array;
        v[i].dst = a[i].dst_ptr_array;
        v[i].count = a[i].ptr_array_len;
        v[i].bytes = a[i].bytes;
    }
    return v;
}
int PARMCI_PutV(armci_giov_t *darr, int len, int proc) {
    auto v = to_comex(darr, len);
    return comex_putv(v.data(), len, proc, COMEX_GROUP_WORLD);
}
int PARMCI_GetV(armci_giov_t *darr, int len, int proc) {
    auto v = to_comex(darr, len);
    return comex_getv(v.data(), len, proc, COMEX_GROUP_WORLD);
}
int PARMCI_AccV(int op, void *scale, armci_giov_t *darr, int len, int proc) {
    auto v = to_comex(darr, len);
    return comex_accv(op, scale, v.data(), len, proc, COMEX_GROUP_WORLD);
}

int PARMCI_NbPut(void *src, void *dst, int bytes, int proc, armci_hdl_t *h) {
    return comex_nbput(src, dst, bytes, proc, COMEX_GROUP_WORLD, h);
}
int PARMCI_NbPutS(void *src, int *ss, void *dst, int *ds, int *count, int levels, int proc, armci_hdl_t *h) {
    if (collapse(ss, ds, count, levels))
        return comex_nbput(src, dst, contiguous_bytes(count, levels), proc, COMEX_GROUP_WORLD, h);
    return comex_nbputs(src, ss, dst, ds, count, levels, proc, COMEX_GROUP_WORLD, h);
}
int PARMCI_NbAccS(int op, void *scale, void *src, int *ss, void *dst, int *ds, int *count, int levels, int proc,
                  armci_hdl_t *h) {
    if (collapse(ss, ds, count, levels))
        return comex_nbacc(op, scale, src, dst, contiguous_bytes(count, levels), proc, COMEX_GROUP_WORLD, h);
    return comex_nbaccs(op, scale, src, ss, dst, ds, count, levels, proc, COMEX_GROUP_WORLD, h);
}
int PARMCI_NbGet(void *src, void *dst, int bytes, int proc, armci_hdl_t *h) {
    return comex_nbget(src, dst, bytes, proc, COMEX_GROUP_WORLD, h);
}
int PARMCI_NbGetS(void *src, int *ss, void *dst, int *ds, int *count, int levels, int proc, armci_hdl_t *h) {
    if (collapse(ss, ds, count, levels))
        return comex_nbget(src, dst, contiguous_bytes(count, levels), proc, COMEX_GROUP_WORLD, h);
    return comex_nbgets(src, ss, dst, ds, count, levels, proc, COMEX_GROUP_WORLD, h);
}
int PARMCI_NbPutV(armci_giov_t *darr, int len, int proc, armci_hdl_t *h) {
    auto v = to_comex(darr, len);
    return comex_nbputv(v.data(), len, proc, COMEX_GROUP_WORLD, h);
}
int PARMCI_NbGetV(armci_giov_t *darr, int len, int proc, armci_hdl_t *h) {
    auto v = to_comex(darr, len);
    return comex_nbgetv(v.data(), len, proc, COMEX_GROUP_WORLD, h);
}
int PARMCI_NbAccV(int op, void *scale, armci_giov_t *darr, int len, int proc, armci_hdl_t *h) {
    auto v = to_comex(darr, len);
    return comex_nbaccv(op, scale, v.data(), len, proc, COMEX_GROUP_WORLD, h);
}
void ARMCI_SET_AGGREGATE_HANDLE(armci_hdl_t *) {}     // armci.c:904-912: no aggregation needed
void ARMCI_UNSET_AGGREGATE_HANDLE(armci_hdl_t *) {}

// ---- single values (armci.c:316-332, 615-662, 717-743) ----
int PARMCI_PutValueInt(int src, void *dst, int proc) { return comex_put(&src, dst, sizeof(int), proc, 0); }
int PARMCI_PutValueLong(long src, void *dst, int proc) { return comex_put(&src, dst, sizeof(long), proc, 0); }
int PARMCI_PutValueFloat(float src, void *dst, int proc) { return comex_put(&src, dst, sizeof(float), proc, 0); }
int PARMCI_PutValueDouble(double src, void *dst, int proc) {
    return comex_put(&src, dst, sizeof(double), proc, 0);
}
// a non-blocking put of a value that lives on the caller's stack: the reference
// sends it from the stack too (comex_nbput), so the value is copied before return
int PARMCI_NbPutValueInt(int src, void *dst, int proc, armci_hdl_t *h) {
    const int rc = comex_put(&src, dst, sizeof(int), proc, 0);
    if (h) *h = -1;
    return rc;
}
int PARMCI_NbPutValueLong(long src, void *dst, int proc, armci_hdl_t *h) {
    const int rc = comex_put(&src, dst, sizeof(long), proc, 0);
    if (h) *h = -1;
    return rc;
}
int PARMCI_NbPutValueFloat(float src, void *dst, int proc, armci_hdl_t *h) {
    const int rc = comex_put(&src, dst, sizeof(float), proc, 0);
    if (h) *h = -1;
    return rc;
}
int PARMCI_NbPutValueDouble(double src, void *dst, int proc, armci_hdl_t *h) {
    const int rc = comex_put(&src, dst, sizeof(double), proc, 0);
    if (h) *h = -1;
    return rc;
}
int PARMCI_GetValueInt(void *src, int proc) {
    int v = 0;
    comex_get(src, &v, sizeof(int), proc, 0);
    return v;
}
long PARMCI_GetValueLong(void *src, int proc) {
    long v = 0;
    comex_get(src, &v, sizeof(long), proc, 0);
    return v;
}
float PARMCI_GetValueFloat(void *src, int proc) {
    float v = 0;
    comex_get(src, &v, sizeof(float), proc, 0);
    return v;
}
double PARMCI_GetValueDouble(void *src, int proc) {
    double v = 0;
    comex_get(src, &v, sizeof(double), proc, 0);
    return v;
}

// ---- flagged puts (armci.c:699-712; the reference asserts): the data, its
// remote completion (fence), then the flag -- so a reader that sees the flag
// sees the data ----
int PARMCI_PutS_flag(void *src, int *ss, void *dst, int *ds, int *count, int levels, int *flag, int val, int proc) {
    PARMCI_PutS(src, ss, dst, ds, count, levels, proc);
    comex_fence_proc(proc, COMEX_GROUP_WORLD);
    return comex_put(&val, flag, sizeof(int), proc, COMEX_GROUP_WORLD);
}
int PARMCI_PutS_flag_dir(void *src, int *ss, void *dst, int *ds, int *count, int levels, int *flag, int val,
                         int proc) {
    return PARMCI_PutS_flag(src, ss, dst, ds, count, levels, flag, val, proc);
}
int PARMCI_Put_flag(void *src, void *dst, int bytes, int *f, int v, int proc) {
    comex_put(src, dst, bytes, proc, COMEX_GROUP_WORLD);
    comex_fence_proc(proc, COMEX_GROUP_WORLD);
    return comex_put(&v, f, sizeof(int), proc, COMEX_GROUP_WORLD);
}

// ---- atomics and mutexes (armci.c:282-292, 449, 755, 771) ----
int PARMCI_Rmw(int op, void *ploc, void *prem, int extra, int proc) {
    return comex_rmw(op, ploc, prem, extra, proc, COMEX_GROUP_WORLD);
}
int PARMCI_Create_mutexes(int num) { return comex_create_mutexes(num); }
int PARMCI_Destroy_mutexes() { return comex_destroy_mutexes(); }
void PARMCI_Lock(int mutex, int proc) { comex_lock(mutex, proc); }
void PARMCI_Unlock(int mutex, int proc) { comex_unlock(mutex, proc); }

// ---- shared-memory queries (armci.c:875-935) ----
int ARMCI_Same_node(int proc) {   // the reference's answer: no host load/store into another rank's segment
    (void)proc;
    return 0;
}
int ARMCI_Uses_shm() { return 0; }
int ARMCI_Uses_shm_group() { return 0; }
int ARMCI_Uses_shm_grp(ARMCI_Group *group) {
    (void)group;
    return 0;
}
void ARMCI_Set_shm_limit(unsigned long shmemlimit) { (void)shmemlimit; }
void ARMCI_Cleanup() { comex_finalize(); }
void PARMCI_Copy(void *src, void *dst, int n) {   // armci.c:891-895 asserts: not a supported call
    (void)src;
    (void)dst;
    comex_error("ARMCI_Copy is not supported (the reference asserts)", n);
}
int parmci_notify(int proc) {
    comex_error("armci_notify is not supported (the reference asserts)", proc);
    return 0;
}
int parmci_notify_wait(int proc, int *pval) {
    (void)pval;
    comex_error("armci_notify_wait is not supported (the reference asserts)", proc);
    return 0;
}

// ---- locality domains (armci.c:24-95, 806-867): ranks binned by node; when the
// nodes do not hold equally many ranks, every rank is its own domain ----
static int ppn_and_node(int *my_node) {
    gaamd::Runtime &r = gaamd::rt();
    int nodes = r.nnodes > 0 ? r.nnodes : 1;
    int ppn = r.size / nodes;
    bool uniform = ppn * nodes == r.size;
    for (int q = 0; q < r.size && uniform; ++q)   // block placement, equal sizes
        if (q / ppn != (r.node_of.empty() ? 0 : r.node_of[q])) uniform = false;
    if (!uniform) ppn = 1;
    if (my_node) *my_node = r.rank / ppn;
    return ppn;
}
int armci_domain_nprocs(armci_domain_t, int) { return ppn_and_node(nullptr); }
int armci_domain_id(armci_domain_t, int glob_proc_id) { return glob_proc_id / ppn_and_node(nullptr); }
int armci_domain_glob_proc_id(armci_domain_t, int id, int loc_proc_id) {
    return id * ppn_and_node(nullptr) + loc_proc_id;
}
int armci_domain_my_id(armci_domain_t) {
    int node = 0;
    ppn_and_node(&node);
    return node;
}
int armci_domain_count(armci_domain_t) { return gaamd::rt().size / ppn_and_node(nullptr); }
int armci_domain_same_id(armci_domain_t, int proc) {
    const int ppn = ppn_and_node(nullptr);
    return proc / ppn == gaamd::rt().rank / ppn;
}

// ---- processor groups (comex/src-armci/groups.c) ----
int ARMCI_Group_rank(ARMCI_Group *id, int *rank) { return comex_group_rank(*id, rank); }
void ARMCI_Group_size(ARMCI_Group *id, int *size) { comex_group_size(*id, size); }
int ARMCI_Absolute_id(ARMCI_Group *id, int group_rank) {
    int w = -1;
    comex_group_translate_world(*id, group_rank, &w);
    return w;
}
void ARMCI_Group_set_default(ARMCI_Group *id) { ARMCI_Default_Proc_Group = *id; }
void ARMCI_Group_get_default(ARMCI_Group *group_out) { *group_out = ARMCI_Default_Proc_Group; }
void ARMCI_Group_get_world(ARMCI_Group *group_out) { *group_out = COMEX_GROUP_WORLD; }
void ARMCI_Group_free(ARMCI_Group *id) { comex_group_free(*id); }
void ARMCI_Group_create_child(int n, int *pid_list, ARMCI_Group *id_child, ARMCI_Group *id_parent) {
    comex_group_create(n, pid_list, *id_parent, id_child);
}
void ARMCI_Group_create(int n, int *pid_list, ARMCI_Group *group_out) {
    comex_group_create(n, pid_list, ARMCI_Default_Proc_Group, group_out);
}

// ---- iterator.c:158-193: a local patch to / from a contiguous buffer, through
// the same strided copy kernels as comex_puts/gets on this rank ----
static void packed_strides_of(const int *count, int levels, int *ps) {
    long acc = count[0];
    for (int j = 0; j < levels; ++j) {
        ps[j] = (int)acc;
        acc *= count[j + 1];
    }
}
void armci_write_strided(void *ptr, int stride_levels, int stride_arr[], int count[], char *buf) {
    if (count[0] <= 0) comex_error("armci_write_strided: count[0] must be > 0", count[0]);
    int ps[8];
    packed_strides_of(count, stride_levels, ps);
    int me = 0;
    comex_group_rank(COMEX_GROUP_WORLD, &me);
    comex_puts(ptr, stride_arr, buf, ps, count, stride_levels, me, COMEX_GROUP_WORLD);
}
void armci_read_strided(void *ptr, int stride_levels, int stride_arr[], int count[], char *buf) {
    if (count[0] <= 0) comex_error("armci_read_strided: count[0] must be > 0", count[0]);
    int ps[8];
    packed_strides_of(count, stride_levels, ps);
    int me = 0;
    comex_group_rank(COMEX_GROUP_WORLD, &me);
    comex_puts(buf, ps, ptr, stride_arr, count, stride_levels, me, COMEX_GROUP_WORLD);
}

int PARMCI_Wait(armci_hdl_t *h) { return comex_wait(h); }
int PARMCI_Test(armci_hdl_t *h) {
    int status = 0;
    comex_test(h, &status);
    return status;
}
int PARMCI_WaitAll() { return comex_wait_all(COMEX_GROUP_WORLD); }
int PARMCI_WaitProc(int proc) { return comex_wait_proc(proc, COMEX_GROUP_WORLD); }

int PARMCI_Malloc(void *ptr_arr[], armci_size_t bytes) {
    return comex_malloc(ptr_arr, (size_t)bytes, ARMCI_Default_Proc_Group);
}
int PARMCI_Malloc_memdev(void *ptr_arr[], armci_size_t bytes, const char *device) {
    return comex_malloc_mem_dev(ptr_arr, (size_t)bytes, ARMCI_Default_Proc_Group, device);
}
int PARMCI_Free(void *ptr) { return comex_free(ptr, ARMCI_Default_Proc_Group); }
int PARMCI_Free_memdev(void *ptr) { return comex_free_dev(ptr, ARMCI_Default_Proc_Group); }
int ARMCI_Malloc_group(void *ptr_arr[], armci_size_t bytes, ARMCI_Group *group) {
    return comex_malloc(ptr_arr, (size_t)bytes, *group);
}
int ARMCI_Malloc_group_memdev(void *ptr_arr[], armci_size_t bytes, ARMCI_Group *group, const char *device) {
    return comex_malloc_mem_dev(ptr_arr, (size_t)bytes, *group, device);
}
int ARMCI_Free_group(void *ptr, ARMCI_Group *group) { return comex_free(ptr, *group); }

// ---- non-collective memory (armci.c:460-538) ----
void PARMCI_Memget(size_t bytes, armci_meminfo_t *meminfo, int memflg) {
    int rank = 0;
    comex_group_rank(COMEX_GROUP_WORLD, &rank);
    if (bytes == 0) comex_error("PARMCI_Memget: size must be > 0", 0);
    if (!meminfo) comex_error("PARMCI_Memget: Invalid arg #2 (NULL ptr)", 0);
    if (memflg != 0) comex_error("PARMCI_Memget: Invalid memflg", memflg);
    void *p = comex_malloc_local(bytes);
    if (!p) comex_error("PARMCI_Memget failed", (int)bytes);
    meminfo->armci_addr = (char *)p;
    meminfo->addr = (char *)p;
    meminfo->size = bytes;
    meminfo->cpid = rank;
}
void *PARMCI_Memat(armci_meminfo_t *meminfo, long offset) {
    (void)offset;
    if (!meminfo) comex_error("PARMCI_Memat: Invalid arg #1 (NULL ptr)", 0);
    return meminfo->addr;
}
void PARMCI_Memdt(armci_meminfo_t *meminfo, long offset) {
    (void)meminfo;
    (void)offset;
}
void PARMCI_Memctl(armci_meminfo_t *meminfo) {
    int rank = 0;
    comex_group_rank(COMEX_GROUP_WORLD, &rank);
    if (!meminfo) comex_error("PARMCI_Memget: Invalid arg #2 (NULL ptr)", 0);
    if (meminfo->cpid == rank) comex_free_local(meminfo->addr);   // only the creator deletes it
    meminfo->addr = nullptr;
    meminfo->armci_addr = nullptr;
}
void *PARMCI_Malloc_local(armci_size_t bytes) { return comex_malloc_local((size_t)bytes); }
int PARMCI_Free_local(void *ptr) { return comex_free_local(ptr); }

// ---- ARMCI_* = weak aliases of PARMCI_* (comex/src-armci/capi.c) ----------
#define GA_WEAK(name, target) __attribute__((weak, alias(#target)))
int ARMCI_Init() GA_WEAK(ARMCI_Init, PARMCI_Init);
int ARMCI_Init_args(int *, char ***) GA_WEAK(ARMCI_Init_args, PARMCI_Init_args);
int ARMCI_Initialized() GA_WEAK(ARMCI_Initialized, PARMCI_Initialized);
void ARMCI_Finalize() GA_WEAK(ARMCI_Finalize, PARMCI_Finalize);
void ARMCI_Barrier() GA_WEAK(ARMCI_Barrier, PARMCI_Barrier);
void ARMCI_Fence(int) GA_WEAK(ARMCI_Fence, PARMCI_Fence);
void ARMCI_AllFence() GA_WEAK(ARMCI_AllFence, PARMCI_AllFence);
int ARMCI_Put(void *, void *, int, int) GA_WEAK(ARMCI_Put, PARMCI_Put);
int ARMCI_PutS(void *, int *, void *, int *, int *, int, int) GA_WEAK(ARMCI_PutS, PARMCI_PutS);
int ARMCI_Acc(int, void *, void *, void *, int, int) GA_WEAK(ARMCI_Acc, PARMCI_Acc);
int ARMCI_AccS(int, void *, void *, int *, void *, int *, int *, int, int) GA_WEAK(ARMCI_AccS, PARMCI_AccS);
int ARMCI_Get(void *, void *, int, int) GA_WEAK(ARMCI_Get, PARMCI_Get);
int ARMCI_GetS(void *, int *, void *, int *, int *, int, int) GA_WEAK(ARMCI_GetS, PARMCI_GetS);
int ARMCI_PutV(armci_giov_t *, int, int) GA_WEAK(ARMCI_PutV, PARMCI_PutV);
int ARMCI_GetV(armci_giov_t *, int, int) GA_WEAK(ARMCI_GetV, PARMCI_GetV);
int ARMCI_AccV(int, void *, armci_giov_t *, int, int) GA_WEAK(ARMCI_AccV, PARMCI_AccV);
int ARMCI_NbPut(void *, void *, int, int, armci_hdl_t *) GA_WEAK(ARMCI_NbPut, PARMCI_NbPut);
int ARMCI_NbPutS(void *, int *, void *, int *, int *, int, int, armci_hdl_t *) GA_WEAK(ARMCI_NbPutS, PARMCI_NbPutS);
int ARMCI_NbAccS(int, void *, void *, int *, void *, int *, int *, int, int, armci_hdl_t *)
    GA_WEAK(ARMCI_NbAccS, PARMCI_NbAccS);
int ARMCI_NbGet(void *, void *, int, int, armci_hdl_t *) GA_WEAK(ARMCI_NbGet, PARMCI_NbGet);
int ARMCI_NbGetS(void *, int *, void *, int *, int *, int, int, armci_hdl_t *) GA_WEAK(ARMCI_NbGetS, PARMCI_NbGetS);
int ARMCI_Wait(armci_hdl_t *) GA_WEAK(ARMCI_Wait, PARMCI_Wait);
int ARMCI_Test(armci_hdl_t *) GA_WEAK(ARMCI_Test, PARMCI_Test);
int ARMCI_WaitAll() GA_WEAK(ARMCI_WaitAll, PARMCI_WaitAll);
int ARMCI_WaitProc(int) GA_WEAK(ARMCI_WaitProc, PARMCI_WaitProc);
int ARMCI_Malloc(void **, armci_size_t) GA_WEAK(ARMCI_Malloc, PARMCI_Malloc);
int ARMCI_Malloc_memdev(void **, armci_size_t, const char *) GA_WEAK(ARMCI_Malloc_memdev, PARMCI_Malloc_memdev);
int ARMCI_Free(void *) GA_WEAK(ARMCI_Free, PARMCI_Free);
int ARMCI_Free_memdev(void *) GA_WEAK(ARMCI_Free_memdev, PARMCI_Free_memdev);
void *ARMCI_Malloc_local(armci_size_t) GA_WEAK(ARMCI_Malloc_local, PARMCI_Malloc_local);
int ARMCI_Free_local(void *) GA_WEAK(ARMCI_Free_local, PARMCI_Free_local);
void ARMCI_GroupFence(ARMCI_Group *) GA_WEAK(ARMCI_GroupFence, PARMCI_GroupFence);
int ARMCI_Create_mutexes(int) GA_WEAK(ARMCI_Create_mutexes, PARMCI_Create_mutexes);
int ARMCI_Destroy_mutexes() GA_WEAK(ARMCI_Destroy_mutexes, PARMCI_Destroy_mutexes);
void ARMCI_Lock(int, int) GA_WEAK(ARMCI_Lock, PARMCI_Lock);
void ARMCI_Unlock(int, int) GA_WEAK(ARMCI_Unlock, PARMCI_Unlock);
int ARMCI_Rmw(int, void *, void *, int, int) GA_WEAK(ARMCI_Rmw, PARMCI_Rmw);
int ARMCI_Put_flag(void *, void *, int, int *, int, int) GA_WEAK(ARMCI_Put_flag, PARMCI_Put_flag);
int ARMCI_PutS_flag(void *, int *, void *, int *, int *, int, int *, int, int) GA_WEAK(ARMCI_PutS_flag, PARMCI_PutS_flag);
int ARMCI_PutS_flag_dir(void *, int *, void *, int *, int *, int, int *, int, int)
    GA_WEAK(ARMCI_PutS_flag_dir, PARMCI_PutS_flag_dir);
int ARMCI_PutValueInt(int, void *, int) GA_WEAK(ARMCI_PutValueInt, PARMCI_PutValueInt);
int ARMCI_PutValueLong(long, void *, int) GA_WEAK(ARMCI_PutValueLong, PARMCI_PutValueLong);
int ARMCI_PutValueFloat(float, void *, int) GA_WEAK(ARMCI_PutValueFloat, PARMCI_PutValueFloat);
int ARMCI_PutValueDouble(double, void *, int) GA_WEAK(ARMCI_PutValueDouble, PARMCI_PutValueDouble);
int ARMCI_GetValueInt(void *, int) GA_WEAK(ARMCI_GetValueInt, PARMCI_GetValueInt);
long ARMCI_GetValueLong(void *, int) GA_WEAK(ARMCI_GetValueLong, PARMCI_GetValueLong);
float ARMCI_GetValueFloat(void *, int) GA_WEAK(ARMCI_GetValueFloat, PARMCI_GetValueFloat);
double ARMCI_GetValueDouble(void *, int) GA_WEAK(ARMCI_GetValueDouble, PARMCI_GetValueDouble);
int ARMCI_NbPutValueInt(int, void *, int, armci_hdl_t *) GA_WEAK(ARMCI_NbPutValueInt, PARMCI_NbPutValueInt);
int ARMCI_NbPutValueLong(long, void *, int, armci_hdl_t *) GA_WEAK(ARMCI_NbPutValueLong, PARMCI_NbPutValueLong);
int ARMCI_NbPutValueFloat(float, void *, int, armci_hdl_t *) GA_WEAK(ARMCI_NbPutValueFloat, PARMCI_NbPutValueFloat);
int ARMCI_NbPutValueDouble(double, void *, int, armci_hdl_t *)
    GA_WEAK(ARMCI_NbPutValueDouble, PARMCI_NbPutValueDouble);
int ARMCI_NbGetV(armci_giov_t *, int, int, armci_hdl_t *) GA_WEAK(ARMCI_NbGetV, PARMCI_NbGetV);
int ARMCI_NbPutV(armci_giov_t *, int, int, armci_hdl_t *) GA_WEAK(ARMCI_NbPutV, PARMCI_NbPutV);
int ARMCI_NbAccV(int, void *, armci_giov_t *, int, int, armci_hdl_t *) GA_WEAK(ARMCI_NbAccV, PARMCI_NbAccV);
void ARMCI_Memget(size_t, armci_meminfo_t *, int) GA_WEAK(ARMCI_Memget, PARMCI_Memget);
void *ARMCI_Memat(armci_meminfo_t *, long) GA_WEAK(ARMCI_Memat, PARMCI_Memat);
void ARMCI_Memdt(armci_meminfo_t *, long) GA_WEAK(ARMCI_Memdt, PARMCI_Memdt);
void ARMCI_Memctl(armci_meminfo_t *) GA_WEAK(ARMCI_Memctl, PARMCI_Memctl);
void ARMCI_Copy(void *, void *, int) GA_WEAK(ARMCI_Copy, PARMCI_Copy);
int armci_notify(int) GA_WEAK(armci_notify, parmci_notify);
int armci_notify_wait(int, int *) GA_WEAK(armci_notify_wait, parmci_notify_wait);

}  // extern "C"
