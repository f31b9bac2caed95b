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

extern "C" {

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

int PARMCI_Init() { return comex_init(); }
int PARMCI_Init_args(int *argc, char ***argv) { return comex_init_args(argc, argv); }
int PARMCI_Initialized() { return comex_initialized(); }
void PARMCI_Finalize() { comex_finalize(); }
void PARMCI_Barrier() { comex_barrier(COMEX_GROUP_WORLD); }
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
int PARMCI_Wait(armci_hdl_t *h) { return comex_wait(h); }
int PARMCI_Test(armci_hdl_t *h) {
    int status = 0;
    comex_test(h, &status);
    return status;
}
int PARMCI_WaitAll() { return comex_wait_all(COMEX_GROUP_WORLD); }
int PARMCI_WaitProc(int proc) { return comex_wait_proc(proc, COMEX_GROUP_WORLD); }

int PARMCI_Malloc(void *ptr_arr[], armci_size_t bytes) {
    return comex_malloc(ptr_arr, (size_t)bytes, COMEX_GROUP_WORLD);
}
int PARMCI_Malloc_memdev(void *ptr_arr[], armci_size_t bytes, const char *device) {
    return comex_malloc_mem_dev(ptr_arr, (size_t)bytes, COMEX_GROUP_WORLD, device);
}
int PARMCI_Free(void *ptr) { return comex_free(ptr, COMEX_GROUP_WORLD); }
int PARMCI_Free_memdev(void *ptr) { return comex_free_dev(ptr, COMEX_GROUP_WORLD); }
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

}  // extern "C"
