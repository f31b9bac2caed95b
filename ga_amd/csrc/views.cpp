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
#include <sys/syscall.h>
#include <unistd.h>
#include <algorithm>
#include <deque>
#include <mutex>
#include <vector>

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

// Small pageable spans go through a per-thread pinned bounce buffer -- copied in, and out
// again for a destination -- instead of being registered for the call: registering and
// unregistering the pages costs ~20 us, most of a small call (a blocking 64-byte
// accumulate from pageable memory 37.6 us against 17.3 from pinned memory; NGA_Acc of a
// 4x4 patch from a local buffer 35.5 us; profiles/r05/lat/).  Only for callers that
// complete the transfer before their next one (the buffer is reused by the thread's next
// call); the asynchronous remote jobs keep registering.
constexpr int64_t kBounceMax = 128 << 10;
// The non-blocking ring (ring_view, below): 4 MiB per thread, spans up to 64 KiB.
constexpr int64_t kRingBytes = 4 << 20, kRingMax = 64 << 10, kRingAlign = 256;
namespace {
struct BounceBuf {
    char *host = nullptr, *dev = nullptr;
    size_t bytes = 0;
};
struct RingUse {
    int64_t off, end;   // [off, end) of the ring
    int stream;
    uint64_t seq, epoch;
};
struct NbRing {
    char *host = nullptr, *dev = nullptr;
    int64_t head = 0;          // next free byte
    int64_t pend_off = -1, pend_end = 0;   // taken by ring_view, not yet committed
    std::deque<RingUse> q;     // oldest first
};

void ring_retire(NbRing &g) {
    const RingUse u = g.q.front();
    g.q.pop_front();
    if (u.epoch == sched_epoch()) (void)sched_complete(u.stream, u.seq, true);   // else drained at finalize
}

// A thread's pinned buffers: both bounce buffers and its ring (a thread-pool
// caller -- OpenMP workers issuing nb calls -- must not leak pinned memory per thread).
// Every thread that allocated one is listed; a thread that ends frees its own, after the
// operations still reading its ring have completed; comex_finalize frees those of every
// thread still alive, when nothing is in flight any more (views_finalize).
struct ThreadPins;
std::mutex g_pins_mu;
std::vector<ThreadPins *> g_pins;
struct ThreadPins {
    BounceBuf bounce[2];
    NbRing ring;
    bool listed = false;
    void list() {
        if (listed) return;
        std::lock_guard<std::mutex> lk(g_pins_mu);
        g_pins.push_back(this);
        listed = true;
    }
    // no operation reads these buffers any more
    void free_all() {
        for (BounceBuf &b : bounce) {
            if (b.host) (void)hipHostFree(b.host);
            b = BounceBuf();
        }
        if (ring.host) (void)hipHostFree(ring.host);
        ring = NbRing();
    }
    ~ThreadPins() {
        if (!listed) return;
        {
            std::lock_guard<std::mutex> lk(g_pins_mu);
            g_pins.erase(std::remove(g_pins.begin(), g_pins.end(), this), g_pins.end());
        }
        // the main thread ends with the process, which returns everything (and the HIP
        // runtime may be going away by then)
        if ((pid_t)syscall(SYS_gettid) == getpid()) return;
        while (!ring.q.empty()) ring_retire(ring);
        free_all();
    }
};
thread_local ThreadPins t_pins;
}  // namespace
static ThreadPins &pins() { return t_pins; }

size_t views_pinned_threads() {
    std::lock_guard<std::mutex> lk(g_pins_mu);
    return g_pins.size();
}

void views_finalize() {
    std::lock_guard<std::mutex> lk(g_pins_mu);
    for (ThreadPins *t : g_pins) {
        t->free_all();
        t->listed = false;
    }
    g_pins.clear();
}

static char *bounce_buffer(int which, size_t bytes, char **dev) {
    ThreadPins &t = pins();   // [0] a source, [1] a destination (or both sides' union)
    BounceBuf &b = t.bounce[which];
    if (b.bytes < bytes) {
        if (b.host) GA_HIP(hipHostFree(b.host));   // this thread's previous transfer has completed
        b.bytes = std::max<size_t>(bytes, (size_t)64 << 10);
        GA_HIP(hipHostMalloc((void **)&b.host, b.bytes, hipHostMallocMapped));
        GA_HIP(hipHostGetDevicePointer((void **)&b.dev, b.host, 0));
        t.list();
    }
    *dev = b.dev;
    return b.host;
}

// [p + lo, p + hi) through bounce buffer `which`: the bytes copied in (a destination's
// too: an accumulate reads them, and the copy back covers the whole span)
static void bounce_view(View &v, void *p, int64_t lo, int64_t hi, bool is_dst, int which) {
    char *dev = nullptr;
    char *h = bounce_buffer(which, (size_t)(hi - lo), &dev);
    memcpy(h, (char *)p + lo, (size_t)(hi - lo));
    v.host = (char *)p;
    v.lo = lo;
    v.hi = hi;
    v.bounce = h;
    v.dev = dev - lo;
    v.copy_back = is_dst;
    v.wb_host = (char *)p;
    v.wb_bounce = h - lo;
}

void view_rows(View &v, const int *stride, const int *count, int levels, int64_t row_bytes) {
    v.wb_stride = stride;
    v.wb_count = count;
    v.wb_levels = levels;
    v.wb_row = row_bytes;
}

// the rows of a bounced destination back into the user's memory, in the odometer order
// of the descriptor (comex.c:6936-6961): no byte the kernel did not write is touched
static void write_back_rows(const View &v) {
    int idx[8] = {0};
    const int L = v.wb_levels;
    uint64_t rows = 1;
    for (int j = 1; j <= L; ++j) rows *= (uint64_t)v.wb_count[j];
    for (uint64_t r = 0; r < rows; ++r) {
        int64_t off = 0;
        for (int j = 0; j < L; ++j) off += (int64_t)idx[j] * v.wb_stride[j];
        memcpy(v.wb_host + off, v.wb_bounce + off, (size_t)v.wb_row);
        for (int j = 0; j < L; ++j) {
            if (++idx[j] < v.wb_count[j + 1]) break;
            idx[j] = 0;
        }
    }
}

// Non-blocking calls from small pageable sources: the bytes are copied into a per-thread
// pinned ring and the call returns with its kernel queued, as for a device source (ComEx
// lets the caller reuse the source only after the wait; here it may at once).  Before a
// ring range is written again, the operations that read it have completed.  Through the
// one-call bounce buffer above, such a call waited for its kernel: 11 us per
// comex_nbaccs of 64 B-4 KiB against 4 from HBM (profiles/r05/small/).
namespace {
// does [a, b) meet the ring bytes still in use ([front.off, head), circularly)?
bool ring_busy(const NbRing &g, int64_t a, int64_t b) {
    if (g.q.empty()) return false;
    const int64_t t = g.q.front().off, h = g.head;
    if (t < h) return a < h && t < b;
    return a < h || t < b;   // wrapped (or full): [t, end of ring) and [0, h)
}
}  // namespace

bool ring_view(View &v, void *p, int64_t lo, int64_t hi) {
    const int64_t n = hi - lo;
    if (n <= 0 || n > kRingMax) return false;
    ThreadPins &t = pins();
    NbRing &g = t.ring;
    if (!g.host) {
        GA_HIP(hipHostMalloc((void **)&g.host, kRingBytes, hipHostMallocMapped));
        GA_HIP(hipHostGetDevicePointer((void **)&g.dev, g.host, 0));
        t.list();
    }
    if (g.q.empty()) g.head = 0;
    // the copy keeps the source's offset within kRingAlign (the kernel's vector width
    // follows the src/dst alignment)
    const int64_t mis = (int64_t)(((uintptr_t)p + lo) % kRingAlign);
    const int64_t need = (mis + n + kRingAlign - 1) / kRingAlign * kRingAlign;
    int64_t off = g.head;
    if (off + need > kRingBytes) off = 0;
    while (ring_busy(g, off, off + need)) ring_retire(g);
    if (g.q.empty()) g.head = off;   // everything retired: the live region restarts here
    g.pend_off = off;
    g.pend_end = off + need;
    g.head = off + need;
    memcpy(g.host + off + mis, (char *)p + lo, (size_t)n);
    v.host = (char *)p;
    v.lo = lo;
    v.hi = hi;
    v.ring = true;
    v.dev = g.dev + off + mis - lo;
    return true;
}

void ring_commit(int stream, uint64_t seq) {
    NbRing &g = pins().ring;
    if (g.pend_off < 0) return;
    g.q.push_back({g.pend_off, g.pend_end, stream, seq, sched_epoch()});
    g.pend_off = -1;
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
                        View &sv, View &dv, bool ring_src) {
    char *d = nullptr;
    const bool sd = direct_view(src, &d, &sv.hbm);
    if (sd) sv.dev = d;
    const bool dd = direct_view(dst, &d, &dv.hbm);
    if (dd) dv.dev = d;
    uintptr_t s0 = 0, s1 = 0, d0 = 0, d1 = 0;
    if (!sd) page_range(src, slo, shi, s0, s1);
    if (!dd) page_range(dst, dlo, dhi, d0, d1);
    if (!sd && !dd && s0 < d1 && d0 < s1) {
        // both sides pageable on shared pages: one bounce of the union of the two spans
        const uintptr_t b0 = std::min((uintptr_t)src + slo, (uintptr_t)dst + dlo);
        const uintptr_t b1 = std::max((uintptr_t)src + shi, (uintptr_t)dst + dhi);
        if ((int64_t)(b1 - b0) <= kBounceMax) {
            // the union may hold bytes of neither buffer (other allocations between them):
            // copied in, but never back -- only dst's rows are (view_rows), or else dst's span
            bounce_view(dv, (void *)b0, 0, (int64_t)(b1 - b0), true, 1);
            char *base = dv.dev;
            sv.dev = base + ((uintptr_t)src - b0);
            dv.dev = base + ((uintptr_t)dst - b0);
            dv.host = (char *)dst;
            dv.lo = dlo;
            dv.hi = dhi;
            dv.wb_host = (char *)dst;
            dv.wb_bounce = dv.bounce + ((uintptr_t)dst - b0);
            return;
        }
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
        if (ring_src && dd && ring_view(sv, src, slo, shi)) {}   // the destination needs no sync either
        else if (shi - slo <= kBounceMax) bounce_view(sv, src, slo, shi, false, 0);
        else if (register_range(s0, s1, &base)) { sv.registered = (void *)s0; sv.dev = base + ((uintptr_t)src - s0); }
        else stage_view(sv, src, slo, shi, false);
    }
    if (!dd) {
        if (dhi - dlo <= kBounceMax) bounce_view(dv, dst, dlo, dhi, true, 1);
        else if (register_range(d0, d1, &base)) { dv.registered = (void *)d0; dv.dev = base + ((uintptr_t)dst - d0); }
        else stage_view(dv, dst, dlo, dhi, true);
    }
}

View local_view(void *p, int64_t lo, int64_t hi, bool is_dst, bool bounce_ok, bool ring_ok) {
    View v;
    char *d = nullptr;
    if (direct_view(p, &d, &v.hbm)) { v.dev = d; return v; }
    if (ring_ok && !is_dst && ring_view(v, p, lo, hi)) return v;
    if (bounce_ok && hi - lo <= kBounceMax) {
        bounce_view(v, p, lo, hi, is_dst, is_dst ? 1 : 0);
        return v;
    }
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
    if (v.bounce) {
        if (v.copy_back) {
            if (v.wb_levels >= 0) write_back_rows(v);
            else memcpy(v.wb_host + v.lo, v.wb_bounce + v.lo, (size_t)(v.hi - v.lo));
        }
        v.bounce = nullptr;
    }
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
