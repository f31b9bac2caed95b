// views.cpp -- device views of the pointers a ComEx call is given.
//
// The reference's transfers touch user buffers with the CPU (memcpy / _acc on
// mapped shared memory, comex.c:6218-6339); here every byte is moved by a GPU
// kernel, so each user pointer needs a device-accessible address: our segments
// and HBM as they are, pinned host memory through its device mapping, pageable
// host memory pinned for the call (hipHostRegister) or, where its pages are
// already registered elsewhere, staged through a device copy.
#include "comex_impl.hpp"
#include <string.h>
#include <algorithm>

namespace gaamd {

// device-visible without help: our segments, HBM, managed, pinned/registered host
// (No cache of device ranges across calls: hipFree returns the range's virtual
// addresses, and a later pageable host allocation can land there -- a cached
// "device" answer then hands the GPU an unmapped host address: a memory-access
// fault, round 3, test_pageable_sources_sharing_pages_back_to_back.)
bool direct_view(void *p, char **dev, bool *hbm) {
    if (hbm) *hbm = false;
    if (const int k = segment_kind(p)) {   // our HBM segment, or a host segment (same address)
        *dev = (char *)p;
        if (hbm) *hbm = k == 1;
        return true;
    }
    hipPointerAttribute_t at;
    memset(&at, 0, sizeof(at));
    hipError_t e = hipPointerGetAttributes(&at, p);
    if (e == hipSuccess && (at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged)) {
        *dev = (char *)p;
        if (hbm) *hbm = at.type == hipMemoryTypeDevice;
        return true;
    }
    if (e == hipSuccess && at.type == hipMemoryTypeHost && at.devicePointer) {
        *dev = (char *)at.devicePointer;
        return true;
    }
    (void)hipGetLastError();
    return false;
}

static void page_range(const void *p, int64_t lo, int64_t hi, uintptr_t &a0, uintptr_t &a1) {
    a0 = ((uintptr_t)p + lo) & ~(uintptr_t)(kPage - 1);
    a1 = (((uintptr_t)p + hi) + kPage - 1) & ~(uintptr_t)(kPage - 1);
}

// pin + map pageable host pages for this call; on failure (pages already
// registered by someone else) stage the span through a device copy instead
static bool register_range(uintptr_t a0, uintptr_t a1, char **dbase) {
    hipError_t e = hipHostRegister((void *)a0, a1 - a0, hipHostRegisterMapped);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    void *d = nullptr;
    GA_HIP(hipHostGetDevicePointer(&d, (void *)a0, 0));
    *dbase = (char *)d;
    return true;
}

static void stage_view(View &v, void *p, int64_t lo, int64_t hi, bool is_dst) {
    Runtime &r = rt();
    v.host = (char *)p;
    v.lo = lo;
    v.hi = hi;
    GA_HIP(hipMalloc((void **)&v.staged, (size_t)(hi - lo)));
    GA_HIP(hipMemcpyAsync(v.staged, (char *)p + lo, (size_t)(hi - lo), hipMemcpyHostToDevice, r.stream));
    v.dev = v.staged - lo;
    v.copy_back = is_dst;
}

// resolve src and dst of one local transfer; a pageable pair whose page
// ranges overlap is registered once as a union
void local_views(void *src, int64_t slo, int64_t shi, void *dst, int64_t dlo, int64_t dhi,
                        View &sv, View &dv) {
    char *d = nullptr;
    const bool sd = direct_view(src, &d, &sv.hbm);
    if (sd) sv.dev = d;
    const bool dd = direct_view(dst, &d, &dv.hbm);
    if (dd) dv.dev = d;
    uintptr_t s0 = 0, s1 = 0, d0 = 0, d1 = 0;
    if (!sd) page_range(src, slo, shi, s0, s1);
    if (!dd) page_range(dst, dlo, dhi, d0, d1);
    if (!sd && !dd && s0 < d1 && d0 < s1) {
        const uintptr_t u0 = std::min(s0, d0), u1 = std::max(s1, d1);
        char *base = nullptr;
        if (register_range(u0, u1, &base)) {
            sv.registered = (void *)u0;
            sv.dev = base + ((uintptr_t)src - u0);
            dv.dev = base + ((uintptr_t)dst - u0);
            return;
        }
        stage_view(sv, src, slo, shi, false);
        stage_view(dv, dst, dlo, dhi, true);
        return;
    }
    char *base = nullptr;
    if (!sd) {
        if (register_range(s0, s1, &base)) { sv.registered = (void *)s0; sv.dev = base + ((uintptr_t)src - s0); }
        else stage_view(sv, src, slo, shi, false);
    }
    if (!dd) {
        if (register_range(d0, d1, &base)) { dv.registered = (void *)d0; dv.dev = base + ((uintptr_t)dst - d0); }
        else stage_view(dv, dst, dlo, dhi, true);
    }
}

View local_view(void *p, int64_t lo, int64_t hi, bool is_dst) {
    View v;
    char *d = nullptr;
    if (direct_view(p, &d, &v.hbm)) { v.dev = d; return v; }
    uintptr_t a0, a1;
    page_range(p, lo, hi, a0, a1);
    char *base = nullptr;
    if (register_range(a0, a1, &base)) { v.registered = (void *)a0; v.dev = base + ((uintptr_t)p - a0); }
    else stage_view(v, p, lo, hi, is_dst);
    return v;
}

// after the kernel: copy a staged dst back, then unpin / free (stream synced by caller)
void release_view(View &v) {
    Runtime &r = rt();
    if (v.staged) {
        if (v.copy_back)
            GA_HIP(hipMemcpy(v.host + v.lo, v.staged, (size_t)(v.hi - v.lo), hipMemcpyDeviceToHost));
        GA_HIP(hipStreamSynchronize(r.stream));
        GA_HIP(hipFree(v.staged));
        v.staged = nullptr;
    }
    if (v.registered) GA_HIP(hipHostUnregister(v.registered));
    v.registered = nullptr;
}


}  // namespace gaamd
