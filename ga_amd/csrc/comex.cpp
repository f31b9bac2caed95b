// comex.cpp -- the ComEx C API (include/comex.h) on MI355X.
//
// Reference: comex/src-mpi-pr/comex.c (MPI progress-rank transport).  The map:
//
//   comex_accs/nbaccs  (985-1007, 1998-2027) -> xfer(X_ACC)
//     nb_accs (6890-6962): L = 0 -> one _acc; self/SMP -> per-row _acc;
//     else pack -> progress rank -> unpack-acc.
//     Here: target = self -> ONE fused strided-acc kernel on this GPU's stream
//           (no pack, 24 B/element); target = other rank -> pack kernel into
//           this rank's exported staging HBM, request into the owner's inbox,
//           the owner's progress thread runs the unpack-acc kernel (reading the
//           packed bytes over xGMI) on the owner's stream, so accumulates into
//           one target are serialised by that target's stream as the
//           reference serialises them with sem_wait(semaphores[target]).
//   comex_puts/gets (6342-6427, 6617-6696)   -> xfer(X_PUT/X_GET): one strided
//           copy kernel; a remote side is addressed through its IPC mapping.
//   comex_malloc (2359-2605)                 -> hipMalloc in HBM + IPC handle
//           allgather (the reg_entry_t MPI_Allgather at 2461) + IPC open.
//   comex_fence_* (1074-1191), comex_barrier (1217-1234), comex_wait* (1776-1802).
//
// Host (non-HBM) buffers are accepted everywhere: pinned memory is used in
// place (device-mapped), pageable memory is registered for the call.  All
// arithmetic runs on the GPU; there is no CPU compute path.
#include <chrono>
#include "runtime.hpp"
#include "../../include/ga_amd.h"
#include "gaamd_kernels.h"
#include "../../include/comex.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <sched.h>
#include <deque>
#include <memory>
#include <algorithm>

namespace gaamd {

static const long kPage = 4096;

static void ensure_init() {
    if (!rt().initialized) fatal("comex used before comex_init");
}

// ---- groups ---------------------------------------------------------------
static std::vector<std::vector<int>> g_groups;   // group id - 1 -> world ranks

// world ranks of a comex group, in group-rank order
std::vector<int> group_members(int group) {
    Runtime &r = rt();
    std::vector<int> m;
    if (group == COMEX_GROUP_WORLD) {
        for (int q = 0; q < r.size; ++q) m.push_back(q);
        return m;
    }
    if (group < 1 || group > (int)g_groups.size() || g_groups[group - 1].empty())
        fatal("invalid comex group %d", group);
    return g_groups[group - 1];
}

int translate_world(int group, int proc) {
    Runtime &r = rt();
    if (group == COMEX_GROUP_WORLD) {
        if (proc < 0 || proc >= r.size) fatal("proc %d out of range [0,%d)", proc, r.size);
        return proc;
    }
    if (group < 1 || group > (int)g_groups.size() || g_groups[group - 1].empty())
        fatal("invalid comex group %d", group);
    const std::vector<int> &g = g_groups[group - 1];
    if (proc < 0 || proc >= (int)g.size()) fatal("proc %d out of range of group %d", proc, group);
    return g[proc];
}

// ---- pointer resolution ---------------------------------------------------
struct View {
    char *dev = nullptr;          // device-accessible address of the user pointer
    void *registered = nullptr;   // page base we registered for this call
    char *staged = nullptr;       // fallback: device copy of [host+lo, host+hi)
    char *host = nullptr;
    int64_t lo = 0, hi = 0;
    bool copy_back = false;
};

static bool find_segment_local(const void *p, int64_t lo, int64_t hi) {
    Runtime &r = rt();
    const uintptr_t a = (uintptr_t)p;
    for (const Segment &s : r.segs) {
        if (!s.live || s.peer.empty()) continue;
        const PeerMap &m = s.peer[r.rank];
        if (m.bytes && a + lo >= m.base && a + hi <= m.base + m.bytes) return true;
    }
    return false;
}

bool segment_local(const void *p, int64_t lo, int64_t hi) {
    std::lock_guard<std::mutex> g(rt().seg_mu);
    return find_segment_local(p, lo, hi);
}

// reg_cache_find for a rank on another node: inside one of its segments
bool segment_of_rank(int owner, uint64_t p, int64_t lo, int64_t hi) {
    Runtime &r = rt();
    std::lock_guard<std::mutex> g(r.seg_mu);
    for (const Segment &s : r.segs) {
        if (!s.live) continue;
        const PeerMap &m = s.peer[owner];
        if (m.bytes && p + lo >= m.base && p + hi <= m.base + m.bytes) return true;
    }
    return false;
}

static void check_remote(int owner, const void *p, int64_t lo, int64_t hi) {
    if (!segment_of_rank(owner, (uint64_t)(uintptr_t)p, lo, hi))
        fatal("address %p [%ld,%ld) of rank %d is not inside a comex_malloc segment", p, (long)lo, (long)hi, owner);
}

// ---- IPC address history ---------------------------------
// Every export, IPC mapping, unmapping and free of device memory this process
// does (or is told of: gaamd_dev_free) is recorded with its address range, so a
// refused hipIpcGetMemHandle can print which earlier event touched that range.
struct AddrEvent { char kind; uintptr_t lo, hi; int peer; };
static std::mutex g_addr_mu;
static std::deque<AddrEvent> g_addr_log;   // newest last, at most 4096
void addr_event(char kind, const void *p, size_t bytes, int peer) {
    std::lock_guard<std::mutex> g(g_addr_mu);
    g_addr_log.push_back({kind, (uintptr_t)p, (uintptr_t)p + bytes, peer});
    if (g_addr_log.size() > 4096) g_addr_log.pop_front();
}
// the tag a rank writes into a new exported block (do_malloc, the staging buffer)
static uint64_t seg_tag(int rank, uint64_t gen, int end) {
    return 0x67614d4453454700ull ^ ((uint64_t)rank << 40) ^ (gen << 1) ^ (uint64_t)end;
}

static std::vector<void *> g_quarantine;   // blocks whose IPC export was refused (freed at finalize)

static void addr_history(const void *p, size_t bytes) {
    std::lock_guard<std::mutex> g(g_addr_mu);
    const uintptr_t lo = (uintptr_t)p, hi = lo + bytes;
    int n = 0;
    for (const AddrEvent &e : g_addr_log) {
        if (e.lo < hi && lo < e.hi) {
            fprintf(stderr, "[ga_amd %d]   earlier %s [%p, %p) %s%d\n", rt().rank,
                    e.kind == 'x' ? "export" : e.kind == 'o' ? "IPC map" : e.kind == 'c' ? "IPC unmap" :
                    e.kind == 'f' ? "free" : e.kind == 'a' ? "alloc" : e.kind == 'r' ? "reuse (cached block)" : "?",
                    (void *)e.lo, (void *)e.hi, e.peer >= 0 ? "of rank " : "", e.peer);
            ++n;
        }
    }
    fprintf(stderr, "[ga_amd %d]   %d earlier events touched this range (of %zu logged)\n", rt().rank, n,
            g_addr_log.size());
}

static size_t mapped_size(const void *p) {
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return size;
}

static void ipc_close(void *mapped, int peer) {
    if (!mapped) return;
    addr_event('c', mapped, mapped_size(mapped), peer);
    GA_HIP(hipIpcCloseMemHandle(mapped));
}

// Map a same-node peer's HBM (IPC handle).  A failure is not fatal here: a job
// that never touches that peer's memory (owner-aligned accumulates, the weak-
// scaling bench) runs on; the first operation that needs the mapping aborts with
// this diagnosis (remote_view / the progress thread).
static void *ipc_open(hipIpcMemHandle_t h, int q, const char *what) {
    void *p = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        fprintf(stderr, "ga_amd rank %d: cannot map rank %d's %s over IPC (%s); operations that need it will "
                "abort (HSA_ENABLE_IPC_MODE_LEGACY=0 is required for dmabuf IPC)\n", rt().rank, q, what,
                hipGetErrorString(e));
        return nullptr;
    }
    addr_event('o', p, mapped_size(p), q);
    return p;
}

static const char *peer_staging_or_die(int src) {
    const char *p = rt().peer_staging[src];
    if (!p) fatal("rank %d's staging buffer is not mapped here (IPC open failed at comex_init)", src);
    return p;
}

// address of rank `owner`'s byte `p` (owner's address space) in this process
static char *remote_view(int owner, const void *p, int64_t lo, int64_t hi) {
    Runtime &r = rt();
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> g(r.seg_mu);
    for (const Segment &s : r.segs) {
        if (!s.live) continue;
        const PeerMap &m = s.peer[owner];
        if (m.bytes && a + lo >= m.base && a + hi <= m.base + m.bytes) {
            if (!m.mapped)
                fatal("rank %d's segment is not mapped here (another node, or its IPC open failed)", owner);
            return m.mapped + (a - m.base);
        }
    }
    fatal("address %p [%ld,%ld) of rank %d is not inside a comex_malloc segment", p, (long)lo, (long)hi, owner);
}

// device-visible without help: our segments, HBM, managed, pinned/registered host
// (No cache of device ranges across calls: hipFree returns the range's virtual
// addresses, and a later pageable host allocation can land there -- a cached
// "device" answer then hands the GPU an unmapped host address: a memory-access
// fault, round 3, test_pageable_sources_sharing_pages_back_to_back.)
static bool direct_view(void *p, char **dev) {
    if (find_segment_local(p, 0, 1)) { *dev = (char *)p; return true; }
    hipPointerAttribute_t at;
    memset(&at, 0, sizeof(at));
    hipError_t e = hipPointerGetAttributes(&at, p);
    if (e == hipSuccess && (at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged)) {
        *dev = (char *)p;
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
static void local_views(void *src, int64_t slo, int64_t shi, void *dst, int64_t dlo, int64_t dhi,
                        View &sv, View &dv) {
    char *d = nullptr;
    const bool sd = direct_view(src, &d);
    if (sd) sv.dev = d;
    const bool dd = direct_view(dst, &d);
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

static View local_view(void *p, int64_t lo, int64_t hi, bool is_dst = false) {
    View v;
    char *d = nullptr;
    if (direct_view(p, &d)) { v.dev = d; return v; }
    uintptr_t a0, a1;
    page_range(p, lo, hi, a0, a1);
    char *base = nullptr;
    if (register_range(a0, a1, &base)) { v.registered = (void *)a0; v.dev = base + ((uintptr_t)p - a0); }
    else stage_view(v, p, lo, hi, is_dst);
    return v;
}

static bool needs_sync(const View &v) { return v.registered || v.staged; }

// after the kernel: copy a staged dst back, then unpin / free (stream synced by caller)
static void release_view(View &v) {
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

// ---- non-blocking handles ------------------------------------------------
static int g_nb_job[kMaxNb];   // nb handle -> its remote accumulate job (0: none; see progress_jobs)
// nb handle -> a direct-source request (target, its posted sequence; 0: none):
// complete once the owner has applied it (the source is read in place)
static int g_nb_rt[kMaxNb];
static uint64_t g_nb_rseq[kMaxNb];
static std::vector<uint64_t> g_direct_last;   // per target: last direct-source request posted
static void run_job(int id);
static void wait_done(int t, uint64_t seq);

static int nb_alloc() {
    Runtime &r = rt();
    for (int k = 0; k < kMaxNb; ++k) {
        const int i = (r.nb_next + k) % kMaxNb;
        if (!r.nb_used[i]) {
            r.nb_used[i] = true;
            r.nb_next = (i + 1) % kMaxNb;
            return i;
        }
    }
    // table full: complete the oldest like nb_wait_for_handle (comex.c:5653)
    const int i = r.nb_next;
    if (g_nb_job[i]) run_job(g_nb_job[i]);
    g_nb_job[i] = 0;
    if (g_nb_rseq[i]) wait_done(g_nb_rt[i], g_nb_rseq[i]);
    g_nb_rseq[i] = 0;
    (void)sched_complete(r.nb_stream[i], r.nb_seq[i], true);
    r.nb_next = (i + 1) % kMaxNb;
    return i;
}

// handle of an op just enqueued on library stream `stream_idx` (`on_stream`),
// or of one with nothing left on a stream (completed in the call, or a remote
// accumulate job whose completion the handle's job id tracks)
static void nb_complete_now(comex_request_t *h, int stream_idx = 0, bool on_stream = false) {
    Runtime &r = rt();
    const int i = nb_alloc();
    g_nb_job[i] = 0;
    g_nb_rseq[i] = 0;
    r.nb_stream[i] = stream_idx;
    r.nb_seq[i] = on_stream ? sched_track(stream_idx) : 0;
    *h = i;
}

static Span span_of(const void *base, int64_t lo, int64_t hi) {
    Span s;
    s.lo = (int64_t)(uintptr_t)base + lo;
    s.hi = (int64_t)(uintptr_t)base + hi;
    return s;
}

// ---- remote accumulate: staging ring + owner inbox ------------------------
struct Pending { uint64_t seq, off, len; };
static std::vector<std::deque<Pending>> g_pend;   // per target

static size_t sub_ring_bytes() {
    Runtime &r = rt();
    return (r.staging_bytes / (size_t)r.size) & ~(size_t)255;
}

// ring space of a request: every reservation is a multiple of 256 bytes, so
// every request starts 256-byte aligned in the ring
static uint64_t ring_len(uint64_t len) { return (len + 255) & ~255ull; }

static void reap(int t) {
    Runtime &r = rt();
    const uint64_t done = r.shm->done[r.li(r.rank)][r.li(t)].load(std::memory_order_acquire);
    while (!g_pend[t].empty() && g_pend[t].front().seq <= done) g_pend[t].pop_front();
}

static void wait_done(int t, uint64_t seq) {
    Runtime &r = rt();
    for (unsigned spins = 0; r.shm->done[r.li(r.rank)][r.li(t)].load(std::memory_order_acquire) < seq; ++spins)
        if (spins > 256) sched_yield();
    reap(t);
}

// reserve `len` bytes in the staging sub-ring for target t (FIFO release)
static uint64_t stage_alloc(int t, uint64_t len) {
    Runtime &r = rt();
    const uint64_t sub = sub_ring_bytes();
    if (len > sub) fatal("staging request %lu exceeds ring %lu", (unsigned long)len, (unsigned long)sub);
    for (;;) {
        reap(t);
        std::deque<Pending> &q = g_pend[t];
        uint64_t &head = r.stage_head[t];
        if (q.empty()) {
            head = 0;
            return 0;
        }
        const uint64_t tail = q.front().off;   // oldest bytes still being read by the owner
        if (head > tail) {
            if (head + len <= sub) return head;
            if (len <= tail) return 0;             // wrap to the start of the ring
        } else if (head < tail) {
            if (head + len <= tail) return head;
        }                                          // head == tail with pending data: ring full
        wait_done(t, q.front().seq);
    }
}

static std::atomic<unsigned long long> g_route[4];   // gaamd_route_counts
static std::atomic<unsigned long long> g_owned[4];   // gaamd_owner_counts: requests applied, by kind

static void post_request(int t, int op, const void *scale, uint64_t dst_addr, const int *dst_stride,
                         const int *count, int levels, uint64_t off, uint64_t len, uint64_t rb, uint64_t re) {
    Runtime &r = rt();
    Inbox *ib = inbox_of(r.shm, r.li(t));
    const uint64_t ticket = ib->tail.fetch_add(1, std::memory_order_acq_rel);
    Request &q = ib->slot[ticket % kInboxSlots];
    // the slot belongs to our lap once the previous lap's ticket is consumed
    for (unsigned spins = 0; ib->head.load(std::memory_order_acquire) + kInboxSlots <= ticket; ++spins)
        if (spins > 256) sched_yield();
    for (unsigned spins = 0;; ++spins) {
        uint32_t expect = 0;
        if (q.state.compare_exchange_weak(expect, 1, std::memory_order_acq_rel)) break;
        if (spins > 256) sched_yield();
    }
    q.src_rank = r.rank;
    q.op = op;
    q.levels = levels;
    memset(q.count, 0, sizeof(q.count));
    memset(q.dst_stride, 0, sizeof(q.dst_stride));
    for (int j = 0; j <= levels; ++j) q.count[j] = count[j];
    for (int j = 0; j < levels; ++j) q.dst_stride[j] = dst_stride[j];
    q.dst_addr = dst_addr;
    q.staging_off = off;
    q.bytes = len;
    q.seq = (rb << 32) | (re & 0xffffffffull);   // row range travels in seq
    memset(q.scale, 0, sizeof(q.scale));
    if (scale) memcpy(q.scale, scale, (size_t)elem_size(op));
    q.kind = 0;
    g_route[0].fetch_add(1, std::memory_order_relaxed);
    q.iov_serial = 0;
    q.iov_align = 0;
    q.dst_hi = 0;
    q.state.store(2, std::memory_order_release);
}

// io-vector request: staging holds n packed source runs, then the n owner
// addresses (8-byte aligned)
// mode: 0 parallel, 1 in order on one lane (destinations overlap), 2 GPU-sorted runs
static void post_request_iov(int t, int op, const void *scale, int bytes, int n, uint64_t off, uint64_t len,
                             uint64_t dlo, uint64_t dhi, uint64_t align_or, int mode) {
    Runtime &r = rt();
    Inbox *ib = inbox_of(r.shm, r.li(t));
    const uint64_t ticket = ib->tail.fetch_add(1, std::memory_order_acq_rel);
    Request &q = ib->slot[ticket % kInboxSlots];
    for (unsigned spins = 0; ib->head.load(std::memory_order_acquire) + kInboxSlots <= ticket; ++spins)
        if (spins > 256) sched_yield();
    for (unsigned spins = 0;; ++spins) {
        uint32_t expect = 0;
        if (q.state.compare_exchange_weak(expect, 1, std::memory_order_acq_rel)) break;
        if (spins > 256) sched_yield();
    }
    q.src_rank = r.rank;
    q.op = op;
    q.levels = 0;
    memset(q.count, 0, sizeof(q.count));
    memset(q.dst_stride, 0, sizeof(q.dst_stride));
    q.count[0] = bytes;
    q.count[1] = n;
    q.dst_addr = dlo;
    q.dst_hi = dhi;
    q.staging_off = off;
    q.bytes = len;
    q.seq = 0;
    memset(q.scale, 0, sizeof(q.scale));
    if (scale) memcpy(q.scale, scale, (size_t)elem_size(op));
    q.kind = 1;
    g_route[2].fetch_add(1, std::memory_order_relaxed);
    q.iov_serial = mode;
    q.iov_align = align_or;
    q.state.store(2, std::memory_order_release);
}

// kind 3: the owner reads the source patch from this rank's segment directly
static void post_request_direct(int t, int op, const void *scale, uint64_t dst_addr, const int *dst_stride,
                                uint64_t src_addr, const int *src_stride, const int *count, int levels) {
    Runtime &r = rt();
    Inbox *ib = inbox_of(r.shm, r.li(t));
    const uint64_t ticket = ib->tail.fetch_add(1, std::memory_order_acq_rel);
    Request &q = ib->slot[ticket % kInboxSlots];
    for (unsigned spins = 0; ib->head.load(std::memory_order_acquire) + kInboxSlots <= ticket; ++spins)
        if (spins > 256) sched_yield();
    for (unsigned spins = 0;; ++spins) {
        uint32_t expect = 0;
        if (q.state.compare_exchange_weak(expect, 1, std::memory_order_acq_rel)) break;
        if (spins > 256) sched_yield();
    }
    q.src_rank = r.rank;
    q.op = op;
    q.levels = levels;
    memset(q.count, 0, sizeof(q.count));
    memset(q.dst_stride, 0, sizeof(q.dst_stride));
    memset(q.src_stride, 0, sizeof(q.src_stride));
    for (int j = 0; j <= levels; ++j) q.count[j] = count[j];
    for (int j = 0; j < levels; ++j) {
        q.dst_stride[j] = dst_stride[j];
        q.src_stride[j] = src_stride[j];
    }
    q.dst_addr = dst_addr;
    q.src_addr = src_addr;
    q.staging_off = 0;
    q.bytes = 0;
    q.seq = 0;
    memset(q.scale, 0, sizeof(q.scale));
    if (scale) memcpy(q.scale, scale, (size_t)elem_size(op));
    q.kind = 3;
    g_route[1].fetch_add(1, std::memory_order_relaxed);
    q.iov_serial = 0;
    q.iov_align = 0;
    q.dst_hi = 0;
    q.state.store(2, std::memory_order_release);
}

// kind 4: a get through the owner (COMEX_ENABLE_GET_SELF/SMP=0): the owner packs
// rows rb..re of its patch into our staging at `off` (nb_get's OP_GET message to the
// progress rank, comex.c:6188-6214)
static void post_request_get(int t, uint64_t src_addr, const int *src_stride, const int *count, int levels,
                             uint64_t off, uint64_t len, uint64_t rb, uint64_t re) {
    Runtime &r = rt();
    Inbox *ib = inbox_of(r.shm, r.li(t));
    const uint64_t ticket = ib->tail.fetch_add(1, std::memory_order_acq_rel);
    Request &q = ib->slot[ticket % kInboxSlots];
    for (unsigned spins = 0; ib->head.load(std::memory_order_acquire) + kInboxSlots <= ticket; ++spins)
        if (spins > 256) sched_yield();
    for (unsigned spins = 0;; ++spins) {
        uint32_t expect = 0;
        if (q.state.compare_exchange_weak(expect, 1, std::memory_order_acq_rel)) break;
        if (spins > 256) sched_yield();
    }
    q.src_rank = r.rank;
    q.op = kOpCopy;
    q.levels = levels;
    memset(q.count, 0, sizeof(q.count));
    memset(q.dst_stride, 0, sizeof(q.dst_stride));
    memset(q.src_stride, 0, sizeof(q.src_stride));
    for (int j = 0; j <= levels; ++j) q.count[j] = count[j];
    for (int j = 0; j < levels; ++j) q.src_stride[j] = src_stride[j];
    q.src_addr = src_addr;
    q.dst_addr = 0;
    q.staging_off = off;
    q.bytes = len;
    q.seq = (rb << 32) | (re & 0xffffffffull);
    memset(q.scale, 0, sizeof(q.scale));
    q.kind = 4;
    q.iov_serial = 0;
    q.iov_align = 0;
    q.dst_hi = 0;
    q.state.store(2, std::memory_order_release);
}

static uint64_t iov_list_off(int n, int bytes) { return (((uint64_t)n * (uint64_t)bytes) + 15) & ~15ull; }

static bool own_release_if_wanted();   // one-pass memory lock (below)
static bool one_pass_reap(bool wait);

// owner side: drain the inbox in ticket order
static void progress_loop() {
    Runtime &r = rt();
    GA_HIP(hipSetDevice(r.device));
    Inbox *ib = inbox_of(r.shm, r.li(r.rank));
    struct Inflight { hipEvent_t ev; int src; bool rmw; };
    // comex_rmw results: the kernel writes the old value here (pinned, device-mapped),
    // one slot per requester position on the node
    uint64_t *rmw_host = nullptr, *rmw_dev = nullptr;
    std::deque<Inflight> inflight;
    std::vector<hipEvent_t> pool;
    char *prog_work = nullptr;          // launch_iov_runs scratch of this thread
    size_t prog_work_bytes = 0;
    hipEvent_t prog_work_ev = nullptr;
    // idle policy: the reference's progress rank polls without sleeping
    // (comex.c:3379-3565); here the thread keeps polling (yielding the core)
    // while kernels it launched are in flight -- their completion releases the
    // requesters' staging and fences -- and for COMEX_AMD_PROGRESS_SPIN_US after
    // the last request (default 2000), then backs off to short sleeps
    static const double spin_s = [] {
        const char *e = getenv("COMEX_AMD_PROGRESS_SPIN_US");
        return (e ? atof(e) : 2000.0) * 1e-6;
    }();
    auto now_s = [] {
        timespec ts;
        clock_gettime(CLOCK_MONOTONIC, &ts);
        return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
    };
    double last_work = now_s();
    unsigned idle = 0;
    // Requests from a rank on ANOTHER GPU (r.peer_src): their bytes are read with
    // system-scope loads, on a pull stream of that source rank when nothing orders
    // them (one stream per source: different peers' chunks come over different
    // xGMI links and are applied side by side).  Where the rows' order matters the
    // bytes are first pulled into local scratch (per source rank, reused once the
    // kernel that read it has finished) and applied from there.
    std::vector<int> pull_slot(r.size, -1);
    {
        int k = 0;
        for (int q = 0; q < r.size; ++q)
            if (r.same_node(q) && r.peer_src(q)) pull_slot[q] = k++;
    }
    auto pull_stream = [&](int src) {
        const int np = (int)r.streams.size() - r.user_streams;
        return (np > 0 && pull_slot[src] >= 0) ? r.user_streams + pull_slot[src] % np : -1;
    };
    struct Scratch { char *p = nullptr; size_t bytes = 0; hipEvent_t ev = nullptr; };
    std::vector<Scratch> scratch(r.size);
    auto scratch_for = [&](int src, size_t need) -> char * {
        Scratch &x = scratch[src];
        if (x.ev) GA_HIP(hipEventSynchronize(x.ev));   // the previous reader has finished
        if (need > x.bytes) {
            if (x.p) GA_HIP(hipFree(x.p));
            x.bytes = std::max<size_t>(need, 1 << 20);
            GA_HIP(hipMalloc((void **)&x.p, x.bytes));
        }
        if (!x.ev) GA_HIP(hipEventCreateWithFlags(&x.ev, hipEventDisableTiming));
        return x.p;
    };
    // contiguous bytes of a peer GPU into local memory (system-scope loads)
    auto pull = [&](char *loc, const char *peer, uint64_t bytes, hipStream_t st) {
        for (uint64_t off = 0; off < bytes; off += (1ull << 30)) {
            int c1[1] = {(int)std::min<uint64_t>(bytes - off, 1ull << 30)};
            const int rc = launch_strided(kOpCopy, nullptr, peer + off, nullptr, loc + off, nullptr, c1, 0, st,
                                          nullptr, 0, ~0ull, false, true);
            if (rc) fatal("pull from rank's staging failed (%d)", rc);
        }
    };
    for (;;) {
        bool worked = false;
        const uint64_t h = ib->head.load(std::memory_order_relaxed);
        Request &q = ib->slot[h % kInboxSlots];
        // the slot's state is read ONCE per pass and the kind dispatched on that
        // reading: re-reading it per branch let a request that became ready between
        // the kind tests fall through to the last branch as a packed one (an
        // io-vector request applied as an 8-byte unpack-acc: a whole request lost)
        const bool ready = q.state.load(std::memory_order_acquire) == 2;
        if (ready && (q.kind < 0 || q.kind > 4))
            fatal("inbox request of unknown kind %d from rank %d", (int)q.kind, (int)q.src_rank);
        if (ready && q.kind == 1) {
            // io-vector accumulate (the _acc_iov_handler analogue, comex.c:4284-4397)
            const int src = q.src_rank;
            const bool peer = r.peer_src(src);
            const char *packed = peer_staging_or_die(src) + q.staging_off;
            hipEvent_t ev;
            if (pool.empty()) GA_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            else { ev = pool.back(); pool.pop_back(); }
            {
                std::lock_guard<std::mutex> g(r.launch_mu);
                Span dsp;
                dsp.lo = (int64_t)q.dst_addr;
                dsp.hi = (int64_t)q.dst_hi;
                const int si = sched_pick(span_of(packed, 0, (int64_t)q.bytes), dsp, 0, peer ? pull_stream(src) : -1);
                if (peer) {
                    // sources and owner addresses come from another GPU's staging: pull the
                    // request into local scratch first, then apply it from there
                    char *loc = scratch_for(src, q.bytes);
                    pull(loc, packed, q.bytes, r.streams[si]);
                    packed = loc;
                }
                IovDesc d;
                memset(&d, 0, sizeof(d));
                d.src_base = packed;
                d.dst_list = (const uint64_t *)(packed + iov_list_off(q.count[1], q.count[0]));
                d.bytes = q.count[0];
                d.n = (uint32_t)q.count[1];
                int rc;
                if (q.iov_serial == 2) {
                    // repeated destinations ordered on the GPU; the progress thread's own sort
                    // scratch, free once the previous runs kernel has finished
                    const size_t need = iov_runs_work_bytes(d.n);
                    if (prog_work_ev) GA_HIP(hipEventSynchronize(prog_work_ev));
                    if (need > prog_work_bytes) {
                        if (prog_work) GA_HIP(hipFree(prog_work));
                        prog_work_bytes = std::max<size_t>(need, 1 << 20);
                        GA_HIP(hipMalloc((void **)&prog_work, prog_work_bytes));
                    }
                    if (!prog_work_ev) GA_HIP(hipEventCreateWithFlags(&prog_work_ev, hipEventDisableTiming));
                    rc = launch_iov_runs(q.op, q.scale, d, q.iov_align, q.dst_addr,
                                         (q.dst_hi - q.dst_addr) / (uint64_t)d.bytes + 1, prog_work, prog_work_bytes,
                                         r.streams[si]);
                    GA_HIP(hipEventRecord(prog_work_ev, r.streams[si]));
                } else {
                    rc = launch_iov(q.op, q.scale, d, q.iov_align, q.iov_serial != 0, r.streams[si]);
                }
                if (rc) fatal("io-vector accumulate launch failed (%d)", rc);
                if (peer) GA_HIP(hipEventRecord(scratch[src].ev, r.streams[si]));
                GA_HIP(hipEventRecord(ev, r.streams[si]));
            }
            inflight.push_back({ev, src, false});
            g_owned[1].fetch_add(1, std::memory_order_relaxed);
            q.state.store(0, std::memory_order_release);
            ib->head.store(h + 1, std::memory_order_release);
            worked = true;
        } else if (ready && q.kind == 2) {
            // comex_rmw from a rank of this node (the progress rank's OP_FETCH_AND_ADD /
            // OP_SWAP): one lane on this GPU, after earlier operations on those bytes
            const int src = q.src_rank;
            if (!rmw_host) {
                GA_HIP(hipHostMalloc((void **)&rmw_host, sizeof(uint64_t) * kMaxRanks, hipHostMallocMapped));
                GA_HIP(hipHostGetDevicePointer((void **)&rmw_dev, rmw_host, 0));
            }
            uint64_t val = 0;
            memcpy(&val, q.scale, 8);
            hipEvent_t ev;
            if (pool.empty()) GA_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            else { ev = pool.back(); pool.pop_back(); }
            {
                std::lock_guard<std::mutex> g(r.launch_mu);
                const int si = sched_pick(Span(), span_of((void *)q.dst_addr, 0, (int64_t)q.bytes));
                const int rc = launch_rmw(q.op, (void *)q.dst_addr, (int)q.bytes, val, rmw_dev + r.li(src), r.streams[si]);
                if (rc) fatal("rmw launch failed (%d): misaligned word?", rc);
                GA_HIP(hipEventRecord(ev, r.streams[si]));
            }
            inflight.push_back({ev, src, true});
            g_owned[2].fetch_add(1, std::memory_order_relaxed);
            q.state.store(0, std::memory_order_release);
            ib->head.store(h + 1, std::memory_order_release);
            worked = true;
        } else if (ready && q.kind == 3) {
            // strided accumulate read straight from the requester's segment (one
            // pass: src read + dst read + dst write, as a local accumulate)
            const int src = q.src_rank;
            int64_t slo = 0, shi = 0, dlo = 0, dhi = 0;
            side_span_host(q.src_stride, q.count, q.levels, q.count[0], &slo, &shi);
            side_span_host(q.dst_stride, q.count, q.levels, q.count[0], &dlo, &dhi);
            const char *sp = remote_view(src, (const void *)q.src_addr, slo, shi);
            hipEvent_t ev;
            if (pool.empty()) GA_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            else { ev = pool.back(); pool.pop_back(); }
            {
                std::lock_guard<std::mutex> g(r.launch_mu);
                const bool peer = r.peer_src(src);
                const int si = sched_pick(span_of(sp, slo, shi), span_of((void *)q.dst_addr, dlo, dhi), 0,
                                          peer ? pull_stream(src) : -1);
                int rc = launch_strided(q.op, q.scale, sp, q.src_stride, (void *)q.dst_addr, q.dst_stride, q.count,
                                        q.levels, r.streams[si], nullptr, 0, ~0ull, false, peer);
                if (rc == kErrPeerOrdered) {
                    // rows whose order matters, source on another GPU: pack row ranges of
                    // <= 64 MiB into local scratch (system-scope loads), apply each from
                    // there; one stream keeps the ranges (and the reuse of the scratch) in order
                    uint64_t rows = 1;
                    for (int j = 1; j <= q.levels; ++j) rows *= (uint64_t)q.count[j];
                    const uint64_t per = std::max<uint64_t>(1, (64ull << 20) / (uint64_t)q.count[0]);
                    char *loc = scratch_for(src, std::min(rows, per) * (uint64_t)q.count[0]);
                    int ps[8];
                    int64_t acc = q.count[0];
                    for (int j = 0; j < q.levels; ++j) { ps[j] = (int)acc; acc *= q.count[j + 1]; }
                    rc = 0;
                    for (uint64_t rb = 0; rb < rows && !rc; rb += per) {
                        const uint64_t re = std::min(rows, rb + per);
                        char *base = loc - (int64_t)rb * q.count[0];   // row rb lands at the scratch start
                        rc = launch_strided(kOpCopy, nullptr, sp, q.src_stride, base, ps, q.count, q.levels,
                                            r.streams[si], nullptr, rb, re, false, true);
                        if (!rc)
                            rc = launch_strided(q.op, q.scale, base, ps, (void *)q.dst_addr, q.dst_stride, q.count,
                                                q.levels, r.streams[si], nullptr, rb, re);
                    }
                    GA_HIP(hipEventRecord(scratch[src].ev, r.streams[si]));
                }
                if (rc) fatal("direct accumulate launch failed (%d)", rc);
                GA_HIP(hipEventRecord(ev, r.streams[si]));
            }
            inflight.push_back({ev, src, false});
            g_owned[3].fetch_add(1, std::memory_order_relaxed);
            q.state.store(0, std::memory_order_release);
            ib->head.store(h + 1, std::memory_order_release);
            worked = true;
        } else if (ready && q.kind == 4) {
            // a get through us: rows rb..re of our patch packed into the requester's
            // staging (a rank on this GPU, or ourselves: the requester never routes a
            // get from another GPU here -- no rank writes another GPU's HBM)
            const int src = q.src_rank;
            const uint64_t rb = q.seq >> 32, re = q.seq & 0xffffffffull;
            int pstride[8];
            {
                int64_t acc = q.count[0];
                for (int j = 0; j < q.levels; ++j) { pstride[j] = (int)acc; acc *= q.count[j + 1]; }
            }
            char *stage = const_cast<char *>(peer_staging_or_die(src)) + q.staging_off;
            char *stage0 = stage - (int64_t)rb * q.count[0];
            int64_t slo = 0, shi = 0;
            side_span_host(q.src_stride, q.count, q.levels, q.count[0], &slo, &shi);
            hipEvent_t ev;
            if (pool.empty()) GA_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            else { ev = pool.back(); pool.pop_back(); }
            {
                std::lock_guard<std::mutex> g(r.launch_mu);
                const int si = sched_pick(span_of((void *)q.src_addr, slo, shi), span_of(stage, 0, (int64_t)q.bytes));
                const int rc = launch_strided(kOpCopy, nullptr, (const char *)q.src_addr, q.src_stride, stage0, pstride,
                                              q.count, q.levels, r.streams[si], nullptr, rb, re);
                if (rc) fatal("get pack launch failed (%d)", rc);
                GA_HIP(hipEventRecord(ev, r.streams[si]));
            }
            inflight.push_back({ev, src, false});
            g_owned[0].fetch_add(1, std::memory_order_relaxed);
            q.state.store(0, std::memory_order_release);
            ib->head.store(h + 1, std::memory_order_release);
            worked = true;
        } else if (ready && q.kind == 0) {
            const int src = q.src_rank;
            const char *packed = peer_staging_or_die(src) + q.staging_off;
            const uint64_t rb = q.seq >> 32, re = q.seq & 0xffffffffull;
            int pstride[8];
            {
                int64_t acc = q.count[0];
                for (int j = 0; j < q.levels; ++j) { pstride[j] = (int)acc; acc *= q.count[j + 1]; }
            }
            // packed rows rb..re start at staging_off; rebase the packed side
            const char *packed0 = packed - (int64_t)rb * q.count[0];
            hipEvent_t ev;
            if (pool.empty()) GA_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            else { ev = pool.back(); pool.pop_back(); }
            {
                std::lock_guard<std::mutex> g(r.launch_mu);
                const bool peer = r.peer_src(src);
                int64_t dlo = 0, dhi = 0;
                side_span_host(q.dst_stride, q.count, q.levels, q.count[0], &dlo, &dhi);
                const int si = sched_pick(span_of(packed, 0, (int64_t)q.bytes), span_of((void *)q.dst_addr, dlo, dhi),
                                          0, peer ? pull_stream(src) : -1);
                int rc = launch_strided(q.op, q.scale, packed0, pstride, (void *)q.dst_addr, q.dst_stride, q.count,
                                        q.levels, r.streams[si], nullptr, rb, re, false, peer);
                if (rc == kErrPeerOrdered) {
                    // the chunk's rows must apply in order: pull the packed chunk into local
                    // scratch first, then the ordinary unpack-acc from there
                    char *loc = scratch_for(src, q.bytes);
                    pull(loc, packed, q.bytes, r.streams[si]);
                    rc = launch_strided(q.op, q.scale, loc - (int64_t)rb * q.count[0], pstride, (void *)q.dst_addr,
                                        q.dst_stride, q.count, q.levels, r.streams[si], nullptr, rb, re);
                    GA_HIP(hipEventRecord(scratch[src].ev, r.streams[si]));
                }
                if (rc) fatal("unpack-acc launch failed (%d)", rc);
                GA_HIP(hipEventRecord(ev, r.streams[si]));
            }
            inflight.push_back({ev, src, false});
            g_owned[0].fetch_add(1, std::memory_order_relaxed);
            q.state.store(0, std::memory_order_release);
            ib->head.store(h + 1, std::memory_order_release);
            worked = true;
        }
        if (own_release_if_wanted()) worked = true;
        if (one_pass_reap(false)) worked = true;   // our one-pass kernels into peers' segments
        while (!inflight.empty()) {
            hipError_t e = hipEventQuery(inflight.front().ev);
            if (e == hipErrorNotReady) break;
            if (e != hipSuccess) fatal("unpack-acc failed: %s", hipGetErrorString(e));
            if (inflight.front().rmw) {
                RmwReply &rp = r.shm->rmw[r.li(inflight.front().src)];
                rp.value = rmw_host[r.li(inflight.front().src)];
                rp.seq.fetch_add(1, std::memory_order_release);
            }
            r.shm->done[r.li(inflight.front().src)][r.li(r.rank)].fetch_add(1, std::memory_order_release);
            pool.push_back(inflight.front().ev);
            inflight.pop_front();
            worked = true;
        }
        if (worked) {
            idle = 0;
            last_work = -1.0;   // refreshed on the next idle pass
            continue;
        }
        if (r.stop.load(std::memory_order_acquire) && inflight.empty() &&
            ib->head.load() == ib->tail.load())
            break;
        ++idle;
        if (!inflight.empty() || idle <= 64) {
            sched_yield();
            continue;
        }
        const double t = now_s();
        if (last_work < 0) last_work = t;
        if (t - last_work < spin_s) sched_yield();
        else usleep(idle > 4096 ? 200 : 20);
    }
    for (hipEvent_t e : pool) (void)hipEventDestroy(e);
    for (Scratch &x : scratch) {
        if (x.ev) {
            (void)hipEventSynchronize(x.ev);
            (void)hipEventDestroy(x.ev);
        }
        if (x.p) (void)hipFree(x.p);
    }
    if (prog_work_ev) {
        (void)hipEventSynchronize(prog_work_ev);
        (void)hipEventDestroy(prog_work_ev);
    }
    if (prog_work) (void)hipFree(prog_work);
    if (rmw_host) (void)hipHostFree(rmw_host);
}

// ---- asynchronous remote accumulate ---------------------------------------
// Reference: nb_accs -> nb_accs_packed (comex.c:6890-7109) packs the patch and
// sends it to the owner's progress rank, chunked.  Here a remote accumulate is
// a job: row-range chunks are packed into the exported staging sub-ring for
// the target as space allows, and each chunk is posted to the owner's inbox
// once its pack kernel has finished.  Jobs advance whenever the caller is in
// the library (any transfer, wait, test, fence), so the remote owners of one
// GA patch -- one ARMCI_NbAccS each (onesided.c:1421-1438) -- progress side by
// side instead of one owner after another.  Per target, chunks are posted in
// the order their staging was allocated: ring release stays FIFO and the
// owner's done counter matches the posted sequence.
struct Chunk { int job; uint64_t off, len, rb, re; hipEvent_t ev; };
struct RJob {
    int id = 0, t = 0, op = 0, levels = 0;
    unsigned char scale[16] = {};
    View sv;
    bool staged_src = false;
    int ss[8] = {}, ds[8] = {}, count[8] = {}, pstride[8] = {};
    char *dst = nullptr;
    int64_t slo = 0, shi = 0;
    uint64_t rows = 0, per_req = 0;
    uint64_t nchunks = 0, next_i = 0, first = 0;   // chunk c = (first + i) % nchunks, i = 0, 1, ...
    int outstanding = 0;
};
static std::deque<RJob> g_jobs;                 // unfinished jobs, creation order
static std::vector<std::deque<Chunk>> g_out;    // per target: packed or packing, not yet posted
static std::vector<hipEvent_t> g_chunk_ev;      // event pool
static int g_job_next = 1;

// stage_alloc without waiting: false when the ring has no room now
static bool try_stage_alloc(int t, uint64_t len, uint64_t &off) {
    Runtime &r = rt();
    const uint64_t sub = sub_ring_bytes();
    if (len > sub) fatal("staging request %lu exceeds ring %lu", (unsigned long)len, (unsigned long)sub);
    reap(t);
    std::deque<Pending> &q = g_pend[t];
    uint64_t &head = r.stage_head[t];
    if (q.empty()) { head = 0; off = 0; return true; }
    const uint64_t tail = q.front().off;
    if (head > tail) {
        if (head + len <= sub) { off = head; return true; }
        if (len <= tail) { off = 0; return true; }
    } else if (head < tail) {
        if (head + len <= tail) { off = head; return true; }
    }
    return false;
}

static RJob *find_job(int id) {
    for (RJob &j : g_jobs) if (j.id == id) return &j;
    return nullptr;
}

// one non-blocking pass over every job; true if anything moved
static bool progress_jobs() {
    Runtime &r = rt();
    if (g_jobs.empty()) return false;
    const uint64_t sub = sub_ring_bytes();
    bool any = false;
    // post chunks whose pack finished, per target in allocation order
    for (int t = 0; t < (int)g_out.size(); ++t) {
        std::deque<Chunk> &o = g_out[t];
        while (!o.empty()) {
            Chunk &c = o.front();
            const hipError_t e = hipEventQuery(c.ev);
            if (e == hipErrorNotReady) break;
            if (e != hipSuccess) fatal("pack kernel failed: %s", hipGetErrorString(e));
            RJob *j = find_job(c.job);
            post_request(t, j->op, j->scale, (uint64_t)(uintptr_t)j->dst, j->ds, j->count, j->levels,
                         (uint64_t)t * sub + c.off, c.len, c.rb, c.re);
            --j->outstanding;
            g_chunk_ev.push_back(c.ev);
            o.pop_front();
            any = true;
        }
    }
    // pack new chunks where the target's ring has room
    for (RJob &j : g_jobs) {
        while (j.next_i < j.nchunks) {
            const uint64_t c = (j.first + j.next_i) % j.nchunks;
            const uint64_t rb = c * j.per_req, re = std::min(j.rows, rb + j.per_req);
            const uint64_t len = (re - rb) * (uint64_t)j.count[0];
            uint64_t off = 0;
            if (!try_stage_alloc(j.t, ring_len(len), off)) break;
            const uint64_t seq = ++r.posted[j.t];
            g_pend[j.t].push_back({seq, off, ring_len(len)});
            r.stage_head[j.t] = off + ring_len(len);
            char *stage = r.staging + (size_t)j.t * sub + off;
            hipEvent_t ev;
            if (g_chunk_ev.empty()) GA_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            else { ev = g_chunk_ev.back(); g_chunk_ev.pop_back(); }
            {
                std::lock_guard<std::mutex> g(r.launch_mu);
                // a staged host src copy sits on stream 0 (ordered there at job start)
                const int si = j.staged_src ? 0 : sched_pick(span_of(j.sv.dev, j.slo, j.shi),
                                                             span_of(stage, 0, (int64_t)len), len);
                // rows [rb, re) of src into the slice, rebased so row rb lands at `stage`
                const int rc = launch_strided(kOpCopy, nullptr, j.sv.dev, j.ss, stage - (int64_t)rb * j.count[0],
                                              j.pstride, j.count, j.levels, r.streams[si], nullptr, rb, re);
                if (rc) fatal("pack launch failed (%d)", rc);
                GA_HIP(hipEventRecord(ev, r.streams[si]));
            }
            g_out[j.t].push_back({j.id, off, len, rb, re, ev});
            ++j.outstanding;
            ++j.next_i;
            any = true;
        }
    }
    // retire jobs whose every chunk is posted (the source is reusable)
    for (auto it = g_jobs.begin(); it != g_jobs.end();) {
        if (it->next_i >= it->nchunks && it->outstanding == 0) {
            release_view(it->sv);
            it = g_jobs.erase(it);
            any = true;
        } else {
            ++it;
        }
    }
    return any;
}

static void backoff(unsigned &spins) {
    if (++spins > 256) sched_yield();
}

static void run_job(int id) {
    for (unsigned spins = 0; find_job(id); backoff(spins))
        if (progress_jobs()) spins = 0;
}

static bool target_busy(int t) {
    for (const RJob &j : g_jobs) if (j.t == t) return true;
    return false;
}

static void drain_target(int t) {
    for (unsigned spins = 0; target_busy(t); backoff(spins))
        if (progress_jobs()) spins = 0;
}

static void drain_all_jobs() {
    for (unsigned spins = 0; !g_jobs.empty(); backoff(spins))
        if (progress_jobs()) spins = 0;
}

// start a remote accumulate; returns its job id (0: nothing to do)
// Are the rows of one side pairwise byte-disjoint?  Sufficient test: with the
// levels sorted by |stride|, each stride covers the whole extent below it.
static bool dst_rows_disjoint(const int *str, const int *count, int levels, int64_t row_bytes) {
    int64_t s[8];
    int64_t c[8];
    int n = 0;
    for (int j = 0; j < levels; ++j)
        if (count[j + 1] > 1) { s[n] = str[j] < 0 ? -(int64_t)str[j] : (int64_t)str[j]; c[n] = count[j + 1]; ++n; }
    for (int i = 1; i < n; ++i)
        for (int k = i; k > 0 && s[k] < s[k - 1]; --k) { std::swap(s[k], s[k - 1]); std::swap(c[k], c[k - 1]); }
    int64_t extent = row_bytes;
    for (int i = 0; i < n; ++i) {
        if (s[i] < extent) return false;
        extent = s[i] * (c[i] - 1) + extent;
    }
    return true;
}

static int remote_acc_start(int t, int op, const void *scale, void *src, const int *ss, void *dst, const int *ds,
                            const int *count, int levels) {
    Runtime &r = rt();
    const int esz = elem_size(op);
    const int64_t row_bytes = (int64_t)(count[0] / esz) * esz;
    uint64_t rows = 1;
    for (int j = 1; j <= levels; ++j) rows *= (uint64_t)count[j];
    if (rows == 0 || row_bytes == 0) return 0;
    if (!r.direct_pending.empty() && r.direct_pending[t]) {
        // an earlier put/get kernel writing or reading t's HBM through the IPC
        // mapping may still run on one of our streams, while the owner applies
        // this accumulate on its own stream: the pack below (and so the post,
        // which waits for the pack) is ordered after it, as the reference's
        // synchronous same-node put/acc are (comex.c:6084-6101, 6241-6260)
        std::lock_guard<std::mutex> g(r.launch_mu);
        sched_join();
        r.direct_pending[t] = 0;
    }
    RJob j;
    j.id = g_job_next++;
    if (g_job_next > (1 << 30)) g_job_next = 1;
    j.t = t;
    j.op = op;
    j.levels = levels;
    if (scale) memcpy(j.scale, scale, (size_t)esz);
    for (int k = 0; k <= levels; ++k) j.count[k] = count[k];
    // only whole elements travel (_acc applies bytes/sizeof(T) of them, acc.h:122):
    // packed rows of row_bytes keep every row element-aligned in staging
    j.count[0] = (int)row_bytes;
    for (int k = 0; k < levels; ++k) { j.ss[k] = ss[k]; j.ds[k] = ds[k]; }
    j.dst = (char *)dst;
    side_span_host(ss, count, levels, count[0], &j.slo, &j.shi);
    // destination must be a registered segment of the owner (reg_cache_find)
    int64_t dlo = 0, dhi = 0;
    side_span_host(ds, count, levels, count[0], &dlo, &dhi);
    (void)remote_view(t, dst, dlo, dhi);
    j.sv = local_view(src, j.slo, j.shi);
    j.staged_src = j.sv.staged != nullptr;
    if (j.staged_src) {
        std::lock_guard<std::mutex> g(r.launch_mu);
        sched_join();
    }
    const uint64_t sub = sub_ring_bytes();
    if ((uint64_t)row_bytes > sub) fatal("row of %ld bytes exceeds staging ring", (long)row_bytes);
    // An owner on another GPU pulls a chunk over one xGMI link (~64 GB/s per direction,
    // half a millisecond for a 32 MiB sub-ring) while the next chunk could already be
    // packed: COMEX_AMD_PEER_CHUNKS cuts the ring into that many slices for such targets,
    // so packing and posting chunk k+1 overlap the pull of chunk k.  Default 1, the only
    // setting measured: the one-GPU proxy (every peer treated as another GPU, 2-rank
    // exchange of C3, profiles/r03/s38) reads 2950-3140 GiB/s with 1, 2922-2941 with 2,
    // 2607-2637 with 4 -- there is no link to hide there, only per-chunk overhead.
    static const uint64_t peer_chunks = [] {
        const char *e = getenv("COMEX_AMD_PEER_CHUNKS");
        const long v = e ? atol(e) : 1;
        return (uint64_t)(v < 1 ? 1 : v);
    }();
    const uint64_t slices = (t != r.rank && r.peer_src(t)) ? peer_chunks : 1;
    j.per_req = std::max<uint64_t>(1, sub / slices / (uint64_t)row_bytes);
    j.rows = rows;
    int64_t acc = row_bytes;
    for (int k = 0; k < levels; ++k) { j.pstride[k] = (int)acc; acc *= count[k + 1]; }
    j.nchunks = (rows + j.per_req - 1) / j.per_req;
    // Chunks of one accumulate go out in row order, except that a requester starts at
    // chunk rank * nchunks / size when the patch's destination rows are pairwise
    // disjoint (then their order is free): when every rank accumulates the same rows of
    // an owner (a GA reduction, C5 M2), their chunks in flight then cover different
    // rows, which the owner can apply side by side instead of one after another.
    if (j.nchunks > 1 && t != r.rank && dst_rows_disjoint(ds, count, levels, row_bytes))
        j.first = (uint64_t)r.rank * j.nchunks / (uint64_t)r.size;
    if (g_out.size() != (size_t)r.size) g_out.resize(r.size);
    static const bool async_ok = [] {
        const char *e = getenv("COMEX_AMD_ASYNC_ACC");   // 0: every remote accumulate completes in its call
        return !e || atoi(e) != 0;
    }();
    const bool host_src = j.sv.registered || j.sv.staged || !async_ok;
    g_jobs.push_back(j);
    const int id = j.id;
    progress_jobs();
    if (host_src) {
        // pageable host source: its pages are pinned (or copied) for this call
        // only -- a view that outlived the call could be shadowed by another
        // call's registration of the same pages and unmapped under it -- so
        // the job completes before the call returns
        run_job(id);
        return 0;
    }
    return id;
}

static void fence_target(int t) {
    Runtime &r = rt();
    if (r.posted.empty()) return;   // no packed route in this job
    if (t != r.rank && !r.same_node(t)) { wire_fence(t); return; }
    drain_target(t);
    wait_done(t, r.posted[t]);
}

// With COMEX_ENABLE_{ACC,PUT}_{SELF,SMP} = 0 operations on this rank's own memory
// take the packed route: a blocking call returns once its chunks are posted,
// before the progress thread has applied them.  A later direct operation on this
// rank's memory (put, get, accumulate, io-vector, rmw) is ordered after them
// first, as the reference flushes before a self/SMP operation when fence_array
// is set (_fence_master, comex.c:6073-6080, 6228-6235).
static void fence_self_if_pending() {
    Runtime &r = rt();
    if (r.posted.empty()) return;
    if (target_busy(r.rank) ||
        r.shm->done[r.li(r.rank)][r.li(r.rank)].load(std::memory_order_acquire) < r.posted[r.rank])
        fence_target(r.rank);
}

// ---- the one transfer routine ---------------------------------------------
enum Xfer { X_ACC, X_PUT, X_GET };

// smallest payload sent by the direct-source route: below it the packed route's
// asynchronous pack beats the host drain of our streams the direct route needs
constexpr uint64_t kDirectSrcMin = 1ull << 20;

// [p+lo, p+hi) inside one of our HBM segments that rank t mapped at comex_malloc
static bool src_segment_shared(const void *p, int64_t lo, int64_t hi, int t) {
    Runtime &r = rt();
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> g(r.seg_mu);
    for (const Segment &s : r.segs) {
        if (!s.live || !s.device || s.peer.empty()) continue;
        const PeerMap &m = s.peer[r.rank];
        if (m.bytes && a + lo >= m.base && a + hi <= m.base + m.bytes) return s.peer[t].member;
    }
    return false;
}

static uint64_t payload_bytes(int64_t row_bytes, const int *count, int levels) {
    uint64_t n = (uint64_t)row_bytes;
    for (int j = 1; j <= levels; ++j) n *= (uint64_t)count[j];
    return n;
}

static int64_t row_bytes_of(int op, int count0) {
    const int esz = elem_size(op);
    return (op == kOpCopy) ? count0 : (int64_t)(count0 / esz) * esz;
}

// ---- one-pass accumulate between ranks sharing a GPU -----------------------
// VERDICT r2 item 4; the reference's SMP route: the worker maps the target's
// shared memory and runs _acc straight into it under the target's semaphore
// (comex.c:6241-6260).  Here, when the owner is on THIS GPU (its segment is local
// HBM seen through the IPC mapping), a same-node accumulate from a device-resident
// source that is not in one of our segments is one fused kernel of ours: src read
// + dst read + dst write, 3 x payload, instead of pack + owner unpack-acc (5 x).
// Exclusion per target (the semaphore) is the owner's node-shm memory lock:
//   * the owner takes its own lock before any launch that writes its segments
//     (own_write_guard, from sched_pick) and keeps it while such writes may be in
//     flight; its progress thread gives it up when a requester waits (mem_want):
//     every stream of the owner drained first (sched_sync_all);
//   * a requester takes the owner's lock, launches, and releases it once its
//     kernels' events completed (its progress thread, or a blocking call / wait /
//     fence) -- so the owner's next write (ordered after the host-observed
//     completion, one device: kernel-boundary coherence) sees the update.
// Lock holders never wait for another memory lock while holding launch_mu, and a
// requester's lock is released by event completion alone, so no wait cycle forms.
// A requester never writes its own segments while it holds another rank's lock
// (the one-pass launch writes only the remote view), so no cycle of locks forms.
// Across GPUs there is no one-pass route: the owner applies.
// smaller patches keep the asynchronous packed route (COMEX_AMD_ONE_PASS_MIN bytes; tests
// lower it so that random programs of small patches exercise the lock hand-offs).
// 64 KiB: one-pass beats the packed route from there up, alone (2 ranks of one GPU,
// tools/remote_sweep.py: latency 16.5 vs 43 us, pipelined 7.7 vs 18-20 us per call)
// and with every other rank accumulating into the same owner (39 vs 68 us per call
// at 64-256 KiB on 3 ranks, 79-83 vs 147-152 on 5; profiles/r03/s24, s25); below it
// the contended case was not better on the one-pass route.
static uint64_t one_pass_min() {
    static const uint64_t v = [] {
        const char *e = getenv("COMEX_AMD_ONE_PASS_MIN");
        return e ? (uint64_t)strtoull(e, nullptr, 10) : (64ull << 10);
    }();
    return v;
}

static bool in_own_segment(const Span &d) {
    Runtime &r = rt();
    std::lock_guard<std::mutex> g(r.seg_mu);
    for (const Segment &s : r.segs) {
        if (!s.live || !s.device || s.peer.empty()) continue;
        const PeerMap &m = s.peer[r.rank];
        if (m.bytes && d.lo < (int64_t)(m.base + m.bytes) && (int64_t)m.base < d.hi) return true;
    }
    return false;
}

// Caller holds launch_mu (sched_pick).  While a requester holds the lock this
// waits WITHOUT launch_mu: a thread holding launch_mu never waits for a memory
// lock, so lock holders (which need their own launch_mu to launch) always get it
// -- a requester holds one lock and waits only for its launch_mu and its kernel,
// the owner's release needs only its launch_mu: no cycle (with launch_mu held
// across the wait, eight ranks accumulating into each other could close one:
// rank A's progress thread holding A's launch_mu waiting for A's lock held by C,
// C waiting for its launch_mu held by its progress thread waiting for C's lock...).
static bool one_pass_reap_try();

void own_write_guard(const Span &dst) {
    Runtime &r = rt();
    if (!r.one_pass || r.own_holds || dst.lo >= dst.hi || !in_own_segment(dst)) return;
    std::atomic<uint32_t> &w = r.shm->mem_lock[r.li(r.rank)];
    std::atomic<uint32_t> &want = r.shm->mem_want[r.li(r.rank)];
    const uint32_t me = 1 + (uint32_t)r.li(r.rank);
    bool waiting = false;   // counted in mem_want: a requester holding our lock then hands it back
    for (unsigned spins = 0;; ++spins) {
        uint32_t e = 0;
        if (w.compare_exchange_weak(e, me, std::memory_order_acq_rel)) break;
        if (!waiting) {
            want.fetch_add(1, std::memory_order_acq_rel);
            waiting = true;
        }
        r.launch_mu.unlock();
        // while we wait for our own memory, hand back the locks of others we hold and
        // someone wants: the holder of ours may be waiting, in this same loop, for one
        // of them (locks are released on demand, so a waiter must never stop reaping)
        one_pass_reap_try();
        if (spins > 64) sched_yield();
        r.launch_mu.lock();
        if (r.own_holds) {   // another thread of this process took it meanwhile
            want.fetch_sub(1, std::memory_order_acq_rel);
            return;
        }
    }
    if (waiting) want.fetch_sub(1, std::memory_order_acq_rel);
    r.own_holds = true;
}

// progress thread: hand the memory lock to a waiting same-GPU requester
static bool own_release_if_wanted() {
    Runtime &r = rt();
    if (!r.one_pass || !r.shm->mem_want[r.li(r.rank)].load(std::memory_order_acquire)) return false;
    std::lock_guard<std::mutex> g(r.launch_mu);
    if (!r.own_holds) return false;
    sched_sync_all();   // every write of ours into our segments has finished
    r.own_holds = false;
    r.shm->mem_lock[r.li(r.rank)].store(0, std::memory_order_release);
    return true;
}

static std::atomic<unsigned long long> g_one_pass{0};   // gaamd_route_counts: one-pass accumulates issued

// The requester's side of the lock: per target, whether we hold its memory lock,
// the library streams our one-pass kernels into its segment were launched on since
// the last completion mark (`pending`), and the marks (events) recorded after them.
// A non-blocking one-pass returns after the launch and records nothing: an event
// per launch puts a marker packet between every two kernels of the stream (the
// cost the sparse completion marks of sched.cpp avoid).  The lock stays with us
// while nobody else wants it; when someone does (mem_want: the owner writing its
// own segment, or another requester), our progress thread marks the pending
// streams, and releases the lock once those marks completed.  A blocking call, a
// wait or a fence marks and waits at once.  Further one-pass accumulates into the
// same target while we hold its lock go straight on (stream order and sched_pick's
// range dependencies order them among themselves), unless someone else waits for
// the lock: then ours finish and it goes first.
struct OnePassHold {
    bool held = false;
    uint32_t pending = 0;
    double since = 0;   // steady-clock seconds at which we took the lock
    std::vector<hipEvent_t> evs;
};
// A holder with launches in flight keeps a wanted lock for up to this long after it
// took it (COMEX_AMD_ONE_PASS_LEASE_US): requesters streaming accumulates into one
// owner then hand the lock over once per lease instead of once per call, each
// hand-over costing a completion wait and a dispatch (tens of us against a few us
// of enqueue per call); the wait a requester sees stays bounded by the lease.
// Every rank but one accumulating into that one (tools/remote_sweep.py --all-to-one,
// profiles/r03/s26): 3 ranks 37 us per call per requester without a lease, 17.5-19.7
// with 100 us, 16.2-17.6 with 400 us; 5 ranks 77-82 / 36-58 / 36-40.
static double one_pass_lease_s() {
    static const double v = [] {
        const char *e = getenv("COMEX_AMD_ONE_PASS_LEASE_US");
        return (e ? atof(e) : 400.0) * 1e-6;
    }();
    return v;
}
static double steady_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static std::mutex g_op_mu;   // g_op_hold, g_op_pool; never held while waiting for a memory lock
static std::vector<OnePassHold> g_op_hold;
static std::vector<hipEvent_t> g_op_pool;

// record a completion mark on every stream with unmarked one-pass launches into
// this target (caller holds g_op_mu; takes launch_mu: the lock order is g_op_mu,
// then launch_mu, everywhere)
static void one_pass_mark(OnePassHold &h) {
    if (!h.pending) return;
    Runtime &r = rt();
    std::lock_guard<std::mutex> g(r.launch_mu);
    for (int si = 0; si < 32 && si < (int)r.streams.size(); ++si) {
        if (!(h.pending >> si & 1u)) continue;
        hipEvent_t ev;
        if (g_op_pool.empty()) GA_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        else { ev = g_op_pool.back(); g_op_pool.pop_back(); }
        GA_HIP(hipEventRecord(ev, r.streams[si]));
        h.evs.push_back(ev);
    }
    h.pending = 0;
}

static void one_pass_release(int t, OnePassHold &h) {   // caller holds g_op_mu; every event completed
    Runtime &r = rt();
    for (hipEvent_t e : h.evs) g_op_pool.push_back(e);
    h.evs.clear();
    h.held = false;
    r.shm->mem_lock[r.li(t)].store(0, std::memory_order_release);
}

// release the locks whose kernels have all completed (wait: mark and wait for them
// first; otherwise a lock nobody waits for stays with us until it is wanted);
// true if one was released.  Caller holds g_op_mu.
static bool one_pass_reap_locked(bool wait) {
    bool any = false;
    Runtime &r = rt();
    for (size_t t = 0; t < g_op_hold.size(); ++t) {
        OnePassHold &h = g_op_hold[t];
        if (!h.held) continue;
        if (h.pending) {
            if (!wait && (!r.shm->mem_want[r.li((int)t)].load(std::memory_order_acquire) ||
                          steady_s() - h.since < one_pass_lease_s()))
                continue;
            one_pass_mark(h);
        }
        bool done = true;
        for (hipEvent_t e : h.evs) {
            const hipError_t x = wait ? hipEventSynchronize(e) : hipEventQuery(e);
            if (x == hipErrorNotReady) { done = false; break; }
            if (x != hipSuccess) fatal("one-pass accumulate failed: %s", hipGetErrorString(x));
        }
        if (done) {
            one_pass_release((int)t, h);
            any = true;
        }
    }
    return any;
}

static bool one_pass_reap(bool wait) {
    std::lock_guard<std::mutex> g(g_op_mu);
    return one_pass_reap_locked(wait);
}

// from a memory-lock wait loop: reap what others want unless another thread of this
// process is in the bookkeeping (it reaps then, or it is the one-pass launch that
// holds g_op_mu only across a launch and an event wait)
static bool one_pass_reap_try() {
    std::unique_lock<std::mutex> g(g_op_mu, std::try_to_lock);
    if (!g.owns_lock()) return false;
    return one_pass_reap_locked(false);
}

// true: launched (blocking: complete on return; else `hdl` tracks it);
// false: not eligible (the caller takes another route)
static bool one_pass_acc(int t, int op, void *scale, void *src, const int *ss, void *dst, const int *ds,
                         const int *count, int levels, int64_t rbd, comex_request_t *hdl) {
    Runtime &r = rt();
    if (!r.one_pass || t == r.rank || !r.same_node(t) || !r.acc_smp_direct || r.peer_src(t)) return false;
    if (rbd <= 0 || payload_bytes(rbd, count, levels) < one_pass_min()) return false;
    int64_t slo = 0, shi = 0, dlo = 0, dhi = 0;
    side_span_host(ss, count, levels, rbd, &slo, &shi);
    side_span_host(ds, count, levels, rbd, &dlo, &dhi);
    char *sdev = nullptr;
    if (!direct_view(src, &sdev)) return false;   // host memory: the packed route pins / stages it
    hipPointerAttribute_t at;
    memset(&at, 0, sizeof(at));
    if (hipPointerGetAttributes(&at, src) == hipSuccess && at.type == hipMemoryTypeHost) return false;
    (void)hipGetLastError();
    char *dview = remote_view(t, dst, dlo, dhi);
    fence_target(t);   // our earlier packed chunks / direct-source requests to t are applied first
    std::atomic<uint32_t> &lk = r.shm->mem_lock[r.li(t)];
    std::atomic<uint32_t> &want = r.shm->mem_want[r.li(t)];
    const uint32_t me = 1 + (uint32_t)r.li(r.rank);
    std::unique_lock<std::mutex> og(g_op_mu);
    if (g_op_hold.size() != (size_t)r.size) g_op_hold.resize(r.size);
    if (g_op_hold[t].held && want.load(std::memory_order_acquire) > 0 &&
        steady_s() - g_op_hold[t].since >= one_pass_lease_s()) {
        // someone waits for t's memory: let ours finish and hand it over first
        one_pass_mark(g_op_hold[t]);
        for (hipEvent_t e : g_op_hold[t].evs) GA_HIP(hipEventSynchronize(e));
        one_pass_release(t, g_op_hold[t]);
    }
    if (!g_op_hold[t].held) {
        og.unlock();   // our progress thread may need it to release another target's lock meanwhile
        want.fetch_add(1, std::memory_order_acq_rel);
        for (unsigned spins = 0;; ++spins) {
            uint32_t e = 0;
            if (lk.compare_exchange_weak(e, me, std::memory_order_acq_rel)) break;
            if ((spins & 63) == 63) one_pass_reap_try();   // never stop handing back what others want
            if (spins > 64) sched_yield();
        }
        want.fetch_sub(1, std::memory_order_acq_rel);
        og.lock();
        g_op_hold[t].held = true;
        g_op_hold[t].since = steady_s();
    }
    int si;
    {
        std::lock_guard<std::mutex> g(r.launch_mu);
        si = sched_pick(span_of(sdev, slo, shi), span_of(dview, dlo, dhi), payload_bytes(rbd, count, levels));
        const int rc = launch_strided(op, scale, sdev, ss, dview, ds, count, levels, r.streams[si], last_launch_info());
        if (rc) fatal("one-pass accumulate launch failed (%d)", rc);
    }
    g_op_hold[t].pending |= 1u << si;
    g_one_pass.fetch_add(1, std::memory_order_relaxed);
    if (hdl) {
        og.unlock();
        nb_complete_now(hdl, si, true);
    } else {
        // blocking: the source is reusable on return -- mark, wait, and hand the lock back
        one_pass_mark(g_op_hold[t]);
        for (hipEvent_t e : g_op_hold[t].evs) GA_HIP(hipEventSynchronize(e));
        one_pass_release(t, g_op_hold[t]);
        og.unlock();
    }
    return true;
}

// A get from another GPU whose destination rows must be written in order (they
// overlap): the rows are packed into local scratch with system-scope loads, then
// copied to the destination by the ordered local kernel, in row ranges of
// <= 64 MiB on one stream.  Caller holds launch_mu; the scratch is reused only
// after the previous such get has finished.
static char *g_get_scratch = nullptr;
static size_t g_get_scratch_bytes = 0;
static hipEvent_t g_get_scratch_ev = nullptr;

static int get_via_scratch(const char *src, const int *ss, char *dst, const int *ds, const int *count, int levels,
                           hipStream_t st) {
    uint64_t rows = 1;
    for (int j = 1; j <= levels; ++j) rows *= (uint64_t)count[j];
    const uint64_t per = std::max<uint64_t>(1, (64ull << 20) / (uint64_t)count[0]);
    const size_t need = (size_t)(std::min(rows, per) * (uint64_t)count[0]);
    if (g_get_scratch_ev) GA_HIP(hipEventSynchronize(g_get_scratch_ev));
    else GA_HIP(hipEventCreateWithFlags(&g_get_scratch_ev, hipEventDisableTiming));
    if (need > g_get_scratch_bytes) {
        if (g_get_scratch) GA_HIP(hipFree(g_get_scratch));
        g_get_scratch_bytes = std::max<size_t>(need, 1 << 20);
        GA_HIP(hipMalloc((void **)&g_get_scratch, g_get_scratch_bytes));
    }
    int ps[8];
    int64_t acc = count[0];
    for (int j = 0; j < levels; ++j) { ps[j] = (int)acc; acc *= count[j + 1]; }
    int rc = 0;
    for (uint64_t rb = 0; rb < rows && !rc; rb += per) {
        const uint64_t re = std::min(rows, rb + per);
        char *base = g_get_scratch - (int64_t)rb * count[0];
        rc = launch_strided(kOpCopy, nullptr, src, ss, base, ps, count, levels, st, nullptr, rb, re, false, true);
        if (!rc) rc = launch_strided(kOpCopy, nullptr, base, ps, dst, ds, count, levels, st, nullptr, rb, re);
    }
    GA_HIP(hipEventRecord(g_get_scratch_ev, st));
    return rc;
}

// ---- host-side stamps (diagnostic) -----------------------------------------
// CLOCK_BOOTTIME ns (the clock rocprofv3 stamps kernels with) at fixed points of the
// last strided call and the last comex_wait_all, for placing the bench's value
// region edges on a kernel trace.  Off unless gaamd_stamps(1).
static std::atomic<bool> g_stamp_on{false};
static uint64_t g_stamp[8];
static inline void stamp(int i) {
    if (!g_stamp_on.load(std::memory_order_relaxed)) return;
    timespec ts;
    clock_gettime(CLOCK_BOOTTIME, &ts);
    g_stamp[i] = (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

// ---- the reference's route toggles beyond SELF/SMP --------------------------
static std::atomic<unsigned long long> g_toggle[3];   // gaamd_toggle_counts: rows, pairs, owner gets

// the reference's self/SMP test (comex.c:6365-6377, 6634-6647, 6910-6913,
// 7120-7122, 7224-7226, 7336-7338): true when the self or SMP route applies to an
// operation on `world`; only otherwise are the PACKED / IOV toggles consulted
static bool self_smp_route(Xfer kind, int world) {
    Runtime &r = rt();
    const bool self = kind == X_ACC ? r.acc_self_direct : (kind == X_PUT ? r.put_self_direct : r.get_self_direct);
    const bool smp = kind == X_ACC ? r.acc_smp_direct : (kind == X_PUT ? r.put_smp_direct : r.get_smp_direct);
    return world == r.rank ? self : (smp && r.same_node(world));
}

static int xfer_contig(Xfer kind, int op, void *scale, void *src, void *dst, int bytes, int proc, int group,
                       comex_request_t *hdl);

// contiguous operations issued non-blocking, at most 32 outstanding (the handle
// table holds kMaxNb), all complete when the window is flushed
struct ContigWindow {
    std::deque<comex_request_t> h;
    void issue(Xfer kind, int op, void *scale, void *src, void *dst, int bytes, int proc, int group) {
        comex_request_t x = -1;
        xfer_contig(kind, op, scale, src, dst, bytes, proc, group, &x);
        h.push_back(x);
        if (h.size() >= 32) {
            comex_wait(&h.front());
            h.pop_front();
        }
    }
    void flush() {
        for (comex_request_t &x : h) comex_wait(&x);
        h.clear();
    }
};

// COMEX_ENABLE_{ACC,PUT,GET}_PACKED=0: the patch row by row, each row a contiguous
// operation, in the odometer order of nb_accs / nb_puts / nb_gets (comex.c:6918-6961)
static int xfer_rows(Xfer kind, int op, void *scale, char *src, const int *ss, char *dst, const int *ds,
                     const int *count, int levels, int proc, int group, comex_request_t *hdl) {
    uint64_t rows = 1;
    for (int j = 1; j <= levels; ++j) rows *= (uint64_t)count[j];
    int idx[8] = {0};
    ContigWindow w;
    for (uint64_t i = 0; i < rows; ++i) {
        int64_t so = 0, dof = 0;
        for (int j = 1; j <= levels; ++j) {
            so += (int64_t)idx[j] * ss[j - 1];
            dof += (int64_t)idx[j] * ds[j - 1];
        }
        w.issue(kind, op, scale, src + so, dst + dof, count[0], proc, group);
        for (int j = 1; j <= levels; ++j) {
            if (++idx[j] < count[j]) break;
            idx[j] = 0;
        }
    }
    w.flush();
    g_toggle[0].fetch_add(1, std::memory_order_relaxed);
    if (hdl) nb_complete_now(hdl);
    return COMEX_SUCCESS;
}

// COMEX_ENABLE_GET_SELF/SMP=0: a get from a rank on this GPU (or from ourselves)
// through the owner.  Row ranges of at most half the staging sub-ring for t: we
// reserve the slice, post a kind-4 request, the owner's progress thread packs the
// rows into it and counts the request done, we unpack the slice into dst.  One
// range at a time (this is the reference's test route, not a fast path).
static void get_via_owner(int t, char *src, const int *ss, char *dst, const int *ds, const int *count, int levels) {
    Runtime &r = rt();
    const uint64_t sub = sub_ring_bytes();
    const uint64_t row = (uint64_t)count[0];
    if (row > sub / 2) {
        // pieces of a long row become one more level (they lie back to back on both
        // sides), the rows' tails a second patch
        if (levels + 1 >= kMaxLevels) fatal("get of %lu-byte rows at %d levels exceeds the staging ring", (unsigned long)row, levels);
        const uint64_t piece = std::max<uint64_t>(16, (sub / 2) / 16 * 16);
        const uint64_t k = row / piece, tail = row - k * piece;
        int cb[8], ssb[8], dsb[8];
        cb[0] = (int)piece;
        cb[1] = (int)k;
        ssb[0] = dsb[0] = (int)piece;
        for (int j = 0; j < levels; ++j) {
            cb[j + 2] = count[j + 1];
            ssb[j + 1] = ss[j];
            dsb[j + 1] = ds[j];
        }
        get_via_owner(t, src, ssb, dst, dsb, cb, levels + 1);
        if (tail) {
            int ct[8];
            for (int j = 0; j <= levels; ++j) ct[j] = count[j];
            ct[0] = (int)tail;
            get_via_owner(t, src + k * piece, ss, dst + k * piece, ds, ct, levels);
        }
        return;
    }
    uint64_t rows = 1;
    for (int j = 1; j <= levels; ++j) rows *= (uint64_t)count[j];
    int64_t slo = 0, shi = 0, dlo = 0, dhi = 0;
    side_span_host(ss, count, levels, (int64_t)row, &slo, &shi);
    side_span_host(ds, count, levels, (int64_t)row, &dlo, &dhi);
    check_remote(t, src, slo, shi);
    drain_target(t);   // our earlier chunks to t are posted first: its done counter stays in order
    View dv = local_view(dst, dlo, dhi, true);
    const bool host_side = needs_sync(dv);
    int pstride[8];
    {
        int64_t acc = (int64_t)row;
        for (int j = 0; j < levels; ++j) { pstride[j] = (int)acc; acc *= count[j + 1]; }
    }
    const uint64_t per = std::max<uint64_t>(1, (sub / 2) / row);
    for (uint64_t rb = 0; rb < rows; rb += per) {
        const uint64_t re = std::min(rows, rb + per), len = (re - rb) * row;
        const uint64_t off = stage_alloc(t, ring_len(len));
        const uint64_t seq = ++r.posted[t];
        g_pend[t].push_back({seq, off, ring_len(len)});
        r.stage_head[t] = off + ring_len(len);
        post_request_get(t, (uint64_t)(uintptr_t)src, ss, count, levels, (uint64_t)t * sub + off, len, rb, re);
        wait_done(t, seq);   // the owner's pack kernel has completed
        const char *stage0 = r.staging + (size_t)t * sub + off - (int64_t)(rb * row);
        std::lock_guard<std::mutex> g(r.launch_mu);
        int si = 0;
        if (host_side) sched_join();
        else si = sched_pick(span_of(stage0, (int64_t)(rb * row), (int64_t)(re * row)), span_of(dv.dev, dlo, dhi),
                             len);
        const int rc = launch_strided(kOpCopy, nullptr, stage0, pstride, dv.dev, ds, count, levels, r.streams[si],
                                      nullptr, rb, re);
        if (rc) fatal("get unpack launch failed (%d)", rc);
        GA_HIP(hipStreamSynchronize(r.streams[si]));   // the slice is free for the next request
    }
    release_view(dv);
    g_toggle[2].fetch_add(1, std::memory_order_relaxed);
}

static int xfer(Xfer kind, int op, void *scale, void *src, int *ss, void *dst, int *ds, int *count,
                int levels, int proc, int group, comex_request_t *hdl) {
    stamp(0);
    ensure_init();
    Runtime &r = rt();
    progress_jobs();   // pending remote accumulates advance on every call
    if (levels < 0 || levels >= COMEX_MAX_STRIDE_LEVEL) fatal("stride_levels %d out of range", levels);
    if (!count) fatal("count is NULL");
    uint64_t rows = 1;
    for (int j = 1; j <= levels; ++j) {
        if (count[j] < 0) fatal("count[%d] = %d < 0", j, count[j]);
        rows *= (uint64_t)count[j];
    }
    if (rows > 0 && count[0] <= 0) fatal("count[0] = %d bytes must be > 0", count[0]);   // nb_acc COMEX_ASSERT(bytes > 0)
    if (!src || !dst) fatal("NULL src or dst");
    if (kind == X_ACC) {
        if (!elem_size(op) || op == kOpCopy) fatal("unknown accumulate op %d", op);
        if (!scale) fatal("NULL scale");
    }
    const int world = translate_world(group, proc);
    const int cop = (kind == X_ACC) ? op : kOpCopy;
    if (hdl) *hdl = -1;
    if (rows == 0) {
        if (hdl) nb_complete_now(hdl);
        return COMEX_SUCCESS;
    }
    if (levels > 0 && !(kind == X_ACC ? r.acc_packed : (kind == X_PUT ? r.put_packed : r.get_packed)) &&
        !self_smp_route(kind, world))
        return xfer_rows(kind, op, scale, (char *)src, ss, (char *)dst, ds, count, levels, proc, group, hdl);

    if (world != r.rank && !r.same_node(world)) {
        // another node: the message protocol (wire.cpp)
        const int64_t rb = row_bytes_of(cop, count[0]);
        int64_t slo = 0, shi = 0, dlo = 0, dhi = 0;
        if (kind == X_GET) {
            side_span_host(ss, count, levels, count[0], &slo, &shi);
            side_span_host(ds, count, levels, count[0], &dlo, &dhi);
            check_remote(world, src, slo, shi);
            View dv = local_view(dst, dlo, dhi, true);
            wire_get_strided((uint64_t)(uintptr_t)src, ss, dv.dev, ds, count, levels, world);
            release_view(dv);
        } else {
            side_span_host(ss, count, levels, count[0], &slo, &shi);
            side_span_host(ds, count, levels, rb, &dlo, &dhi);
            check_remote(world, dst, dlo, dhi);
            View sv = local_view(src, slo, shi);
            wire_send_strided(cop, scale, sv.dev, ss, (uint64_t)(uintptr_t)dst, ds, count, levels, world);
            release_view(sv);
        }
        if (hdl) nb_complete_now(hdl);
        return COMEX_SUCCESS;
    }

    // an owner on this GPU: the one-pass route (our kernel writes its segment under its
    // memory lock), whether or not the source lies in one of our segments -- no host
    // drain of our streams and no hand-off to the owner's progress thread, which the
    // direct-source route below needs
    if (kind == X_ACC && world != r.rank &&
        one_pass_acc(world, op, scale, src, ss, dst, ds, count, levels, row_bytes_of(op, count[0]), hdl))
        return COMEX_SUCCESS;
    // the direct-source route is a direct (SMP) route: COMEX_ENABLE_ACC_SMP=0 sends
    // same-node accumulates down the packed route, as the reference (comex.c:6911-6915)
    if (kind == X_ACC && world != r.rank && r.direct_src && r.acc_smp_direct && r.same_node(world)) {
        const int64_t rbd = row_bytes_of(op, count[0]);
        int64_t slo = 0, shi = 0;
        side_span_host(ss, count, levels, rbd, &slo, &shi);
        if (rbd > 0 && payload_bytes(rbd, count, levels) >= kDirectSrcMin &&
            src_segment_shared(src, slo, shi, world)) {
            // the owner reads the patch from our segment through its IPC mapping:
            // one pass instead of pack + unpack-acc (5 -> 3 x payload)
            int64_t dlo = 0, dhi = 0;
            side_span_host(ds, count, levels, rbd, &dlo, &dhi);
            check_remote(world, dst, dlo, dhi);
            drain_target(world);   // earlier packed chunks to world are posted first (inbox order)
            {
                // the owner's kernel must see every write of ours to the source
                // (and our IPC puts into world's memory): our streams drain first
                std::lock_guard<std::mutex> g(r.launch_mu);
                sched_sync_all();
            }
            int cnt[8];
            for (int k = 0; k <= levels; ++k) cnt[k] = count[k];
            cnt[0] = (int)rbd;   // whole elements only (acc.h:122)
            post_request_direct(world, op, scale, (uint64_t)(uintptr_t)dst, ds, (uint64_t)(uintptr_t)src, ss, cnt,
                                levels);
            const uint64_t seq = ++r.posted[world];
            if (g_direct_last.size() != (size_t)r.size) g_direct_last.assign(r.size, 0);
            g_direct_last[world] = seq;
            if (hdl) {
                nb_complete_now(hdl);
                g_nb_rt[*hdl] = world;
                g_nb_rseq[*hdl] = seq;
            } else {
                wait_done(world, seq);   // local completion = the owner has read the source
            }
            return COMEX_SUCCESS;
        }
    }
    // a get through the owner (COMEX_ENABLE_GET_SELF/SMP=0) from a rank on this GPU or
    // ourselves; from another GPU the get stays a direct read (system-scope loads):
    // the owner could only answer by writing our HBM
    if (kind == X_GET && !self_smp_route(X_GET, world) && !r.peer_src(world)) {
        get_via_owner(world, (char *)src, ss, (char *)dst, ds, count, levels);
        if (hdl) nb_complete_now(hdl);
        return COMEX_SUCCESS;
    }
    // the packed route: remote accumulates on this node, and -- under the
    // COMEX_ENABLE_* toggles -- accumulates / puts to self or same-node puts
    // a put into another GPU's memory is applied by its owner too (no rank writes
    // another GPU's HBM: runtime.hpp same_dev / DESIGN.md §6)
    const bool packed = (kind == X_ACC && (world != r.rank || !r.acc_self_direct)) ||
                        (kind == X_PUT && (world == r.rank ? !r.put_self_direct
                                                           : (!r.put_smp_direct || r.peer_src(world))));
    if (packed) {
        int id = 0;
        const int64_t rbp = row_bytes_of(cop, count[0]);
        if (rbp > 0 && (uint64_t)rbp > sub_ring_bytes() && levels < kMaxLevels &&
            (levels == 0 || dst_rows_disjoint(ds, count, levels, rbp))) {
            // a row longer than the staging sub-ring (a 1-D accumulate of tens of MiB;
            // the reference sends such a message in chunks, comex.c:6263-6338): the
            // row is cut into pieces that become one more stride level (a row's
            // pieces lie back to back on both sides), plus the rows' tails as a
            // second patch.  Rows share no dst byte, so the order of the two parts
            // changes no result.  The first part completes locally here.
            // pieces of whole 16-byte units: whole elements of every type (1..16 B)
            const uint64_t unit = 16;
            uint64_t piece = (sub_ring_bytes() / 2) / unit * unit;
            if (piece == 0) piece = unit;
            const uint64_t k = (uint64_t)rbp / piece, tail = (uint64_t)rbp - k * piece;
            int cb[8], ssb[8], dsb[8];
            cb[0] = (int)piece;
            cb[1] = (int)k;
            ssb[0] = dsb[0] = (int)piece;
            for (int j = 0; j < levels; ++j) {
                cb[j + 2] = count[j + 1];
                ssb[j + 1] = ss[j];
                dsb[j + 1] = ds[j];
            }
            const int body = remote_acc_start(world, cop, scale, src, ssb, dst, dsb, cb, levels + 1);
            if (tail) {
                if (body) run_job(body);
                int ct[8];
                for (int j = 0; j <= levels; ++j) ct[j] = count[j];
                ct[0] = (int)tail;
                id = remote_acc_start(world, cop, scale, (char *)src + k * piece, ss, (char *)dst + k * piece, ds, ct,
                                      levels);
            } else {
                id = body;
            }
        } else {
            id = remote_acc_start(world, cop, scale, src, ss, dst, ds, count, levels);
        }
        if (hdl) {
            nb_complete_now(hdl);
            g_nb_job[*hdl] = id;
        } else if (id) {
            run_job(id);
        }
        return COMEX_SUCCESS;
    }

    const int64_t rb = row_bytes_of(cop, count[0]);
    int64_t slo = 0, shi = 0, dlo = 0, dhi = 0;
    side_span_host(ss, count, levels, rb, &slo, &shi);
    side_span_host(ds, count, levels, rb, &dlo, &dhi);
    View sv, dv;
    if (world == r.rank) fence_self_if_pending();
    if (world != r.rank) {
        // put: remote dst / get: remote src, through the owner's IPC mapping
        fence_target(world);   // order after our own pending accumulates to it
        if (kind == X_PUT) {
            sv = local_view(src, slo, shi);
            dv.dev = remote_view(world, dst, dlo, dhi);
        } else {
            sv.dev = remote_view(world, src, slo, shi);
            dv = local_view(dst, dlo, dhi, true);
        }
    } else {
        local_views(src, slo, shi, dst, dlo, dhi, sv, dv);
    }
    const bool host_side = needs_sync(sv) || needs_sync(dv);
    // a get from another GPU's memory reads it with system-scope loads
    const bool peer = kind == X_GET && world != r.rank && r.peer_src(world);
    int si = 0;
    hipStream_t st;
    {
        std::lock_guard<std::mutex> g(r.launch_mu);
        stamp(1);
        if (host_side) sched_join();   // staged copies sit on stream 0: run there, after everything
        else si = sched_pick(span_of(sv.dev, slo, shi), span_of(dv.dev, dlo, dhi), payload_bytes(rb, count, levels));
        st = r.streams[si];
        stamp(2);
        int rc = launch_strided(cop, scale, sv.dev, ss, dv.dev, ds, count, levels, st, last_launch_info(), 0, ~0ull,
                                false, peer);
        stamp(3);
        if (rc == kErrPeerOrdered) rc = get_via_scratch(sv.dev, ss, dv.dev, ds, count, levels, st);
        if (rc) fatal("strided %s launch failed (code %d): misaligned elements or bad descriptor",
                      kind == X_ACC ? "acc" : (kind == X_PUT ? "put" : "get"), rc);
        if (host_side) sched_sync_all();
    }
    // blocking call: local completion before returning (src reusable, a get's
    // dst filled) -- the stream the op went to holds it and its dependencies
    const bool synced = host_side || (!hdl && r.blocking_sync);
    if (!host_side && synced) GA_HIP(hipStreamSynchronize(st));
    if (world != r.rank && !synced && !r.direct_pending.empty()) r.direct_pending[world] = 1;
    if (r.debug)
        fprintf(stderr, "[ga_amd %d] %s -> %d levels %d count0 %d rows %d: src %s dst %s stream %d\n", r.rank,
                kind == X_ACC ? "acc" : (kind == X_PUT ? "put" : "get"), world, levels, count[0],
                levels ? count[levels] : 1, sv.registered ? "registered" : (sv.staged ? "staged" : "device"),
                dv.registered ? "registered" : (dv.staged ? "staged" : "device"), si);
    if (host_side) {
        release_view(sv);
        release_view(dv);
    }
    if (hdl) nb_complete_now(hdl, si, true);
    stamp(4);
    return COMEX_SUCCESS;
}

static int xfer_contig(Xfer kind, int op, void *scale, void *src, void *dst, int bytes, int proc, int group,
                       comex_request_t *hdl) {
    int count[1] = {bytes};
    if (bytes <= 0) fatal("contiguous transfer of %d bytes", bytes);   // nb_acc/nb_put assert bytes > 0
    return xfer(kind, op, scale, src, nullptr, dst, nullptr, count, 0, proc, group, hdl);
}

// ---- vector (io-vector) transfers: comex_accv/putv/getv --------------------
// Reference: comex.c:7327-7400 (nb_accv: per-pair nb_acc, or the iov message to
// the progress rank), _acc_iov_handler 4284-4397.  Here one kernel applies all
// n pairs of a descriptor (k_iov); pairs whose destinations overlap (GA
// scatter-acc duplicates) run one by one in order.
static char *g_iov_scratch = nullptr;
static size_t g_iov_scratch_bytes = 0;
// gaamd_iov_path_counts: local io-vector launches with repeated-destination
// ordering, by path: hashed, hashed + radix fallback (conflicts overflowed), radix
static std::atomic<unsigned long long> g_iov_path[3];

static char *g_iov_host = nullptr;
static size_t g_iov_host_bytes = 0;

static char *iov_host_scratch(size_t bytes) {   // pinned upload staging; caller holds launch_mu
    if (bytes <= g_iov_host_bytes) return g_iov_host;
    if (g_iov_host) GA_HIP(hipHostFree(g_iov_host));
    g_iov_host_bytes = std::max<size_t>(bytes, 1 << 20);
    GA_HIP(hipHostMalloc((void **)&g_iov_host, g_iov_host_bytes, hipHostMallocMapped));
    return g_iov_host;
}

static char *g_riov_pin = nullptr;   // remote io-vector request upload (pinned)
static size_t g_riov_pin_bytes = 0;
static char *remote_iov_pinned(size_t bytes) {   // caller holds launch_mu; no upload from it in flight
    if (bytes <= g_riov_pin_bytes) return g_riov_pin;
    if (g_riov_pin) GA_HIP(hipHostFree(g_riov_pin));
    g_riov_pin_bytes = std::max<size_t>(bytes, 1 << 20);
    GA_HIP(hipHostMalloc((void **)&g_riov_pin, g_riov_pin_bytes, hipHostMallocMapped));
    return g_riov_pin;
}

// copy `bytes` of the pinned (device-mapped) upload buffer into staging with the
// copy kernel on `st` (one launch, no runtime staging of the host bytes)
static void upload_pinned(char *stage, const char *pin, size_t bytes, hipStream_t st) {
    void *dev = nullptr;
    GA_HIP(hipHostGetDevicePointer(&dev, (void *)pin, 0));
    int count[1] = {(int)bytes};
    const int rc = launch_strided(kOpCopy, nullptr, (const char *)dev, nullptr, stage, nullptr, count, 0, st, nullptr);
    if (rc) fatal("io-vector upload failed (%d)", rc);
}

static char *iov_scratch(size_t bytes) {   // caller holds launch_mu
    if (bytes <= g_iov_scratch_bytes) return g_iov_scratch;
    sched_sync_all();
    if (g_iov_scratch) GA_HIP(hipFree(g_iov_scratch));
    g_iov_scratch_bytes = std::max<size_t>(bytes, 1 << 20);
    GA_HIP(hipMalloc((void **)&g_iov_scratch, g_iov_scratch_bytes));
    return g_iov_scratch;
}

static bool ranges_overlap(std::vector<std::pair<uint64_t, uint64_t>> v) {
    std::sort(v.begin(), v.end());
    for (size_t i = 1; i < v.size(); ++i)
        if (v[i].first < v[i - 1].second) return true;
    return false;
}

static bool any_cross_overlap(std::vector<std::pair<uint64_t, uint64_t>> a, std::vector<std::pair<uint64_t, uint64_t>> b) {
    std::sort(a.begin(), a.end());
    std::sort(b.begin(), b.end());
    size_t i = 0, j = 0;
    while (i < a.size() && j < b.size()) {
        if (a[i].first < b[j].second && b[j].first < a[i].second) return true;
        if (a[i].second <= b[j].second) ++i; else ++j;
    }
    return false;
}

// Device views of the listed addresses, resolved through a small cache of the
// allocations already seen (one hipPointerGetAttributes per allocation instead of
// per pair: a GA scatter-acc lists up to millions of addresses in a few buffers).
struct ViewCache {
    struct Range { uint64_t lo = 0, hi = 0; int64_t delta = 0; };
    Range r[4];
    uint64_t neg[4] = {~0ull, ~0ull, ~0ull, ~0ull};   // pages known not to be device-accessible
    int next = 0, next_neg = 0;
    bool view(void *p, int bytes, uint64_t *out) {
        const uint64_t a = (uint64_t)(uintptr_t)p;
        for (const Range &x : r)
            if (a >= x.lo && a + (uint64_t)bytes <= x.hi) { *out = (uint64_t)((int64_t)a + x.delta); return true; }
        const uint64_t pg = a & ~(uint64_t)(kPage - 1);
        for (uint64_t q : neg)
            if (q == pg && a + (uint64_t)bytes <= pg + kPage) return false;
        char *d = nullptr;
        if (!direct_view(p, &d)) {
            neg[next_neg] = pg;
            next_neg = (next_neg + 1) % 4;
            return false;
        }
        *out = (uint64_t)(uintptr_t)d;
        hipDeviceptr_t base = nullptr;
        size_t size = 0;
        if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)d) == hipSuccess && size) {
            Range &x = r[next];
            next = (next + 1) % 4;
            x.delta = (int64_t)(uintptr_t)d - (int64_t)a;
            x.lo = (uint64_t)((int64_t)(uintptr_t)base - x.delta);
            x.hi = x.lo + size;
        } else {
            (void)hipGetLastError();
        }
        return true;
    }
    // the allocation holding address a: its range [lo, hi) and device-view offset
    bool range_of(uint64_t a, uint64_t *lo, uint64_t *hi, int64_t *delta) {
        uint64_t d = 0;
        if (!view((void *)(uintptr_t)a, 1, &d)) return false;
        for (const Range &x : r)
            if (a >= x.lo && a < x.hi) { *lo = x.lo; *hi = x.hi; *delta = x.delta; return true; }
        return false;
    }
    // one allocation holding every byte of [lo, hi): its (uniform) device-view offset
    bool span(uint64_t lo, uint64_t hi, int64_t *delta) {
        uint64_t d = 0;
        if (!view((void *)(uintptr_t)lo, 1, &d)) return false;
        for (const Range &x : r)
            if (lo >= x.lo && hi <= x.hi) { *delta = x.delta; return true; }
        return false;
    }
};

// Host passes over io-vector lists (tens of MiB at GA scatter sizes) split into
// contiguous ranges over a few threads: fn(t, i0, i1) for t < T, T = one thread
// per 256 Ki pairs, at most 8.  Each range's results are combined by the caller
// in range order, so the outcome does not depend on T.
static int par_threads(long n) {
    static const long cap = [] {   // COMEX_AMD_HOST_THREADS: at most this many (1..8, default 8)
        const char *e = getenv("COMEX_AMD_HOST_THREADS");
        const long v = e ? atol(e) : 8;
        return v < 1 ? 1L : (v > 8 ? 8L : v);
    }();
    return (int)std::max(1L, std::min(cap, n >> 18));
}
template <class F> static void par_for(long n, int T, F fn) {
    if (T <= 1) { fn(0, 0L, n); return; }
    std::vector<std::thread> th;
    th.reserve((size_t)T - 1);
    for (int t = 1; t < T; ++t) th.emplace_back([&, t] { fn(t, n * t / T, n * (t + 1) / T); });
    fn(0, 0L, n / T);
    for (std::thread &x : th) x.join();
}

// Is every byte of [lo, hi) ordinary CPU memory of this process (one readable,
// and if `write` writable, mapping that is not a device file)?  One lookup in
// /proc/self/maps replaces a device-view query per page when a whole io-vector
// side lies in pageable host memory (GA's MA buffer `v` of a scatter/gather):
// device allocations are either PROT_NONE reservations or /dev/dri mappings, so
// a side that passes is safe to gather/scatter on the host.  Any address not
// covered (or a line that does not parse) answers false and the per-pair
// classification decides as before.  COMEX_AMD_IOV_MAPS=0 disables it.
static bool host_cpu_range(uint64_t lo, uint64_t hi, bool write) {
    static const bool on = [] {
        const char *e = getenv("COMEX_AMD_IOV_MAPS");
        return !(e && atoi(e) == 0);
    }();
    if (!on || hi <= lo) return false;
    FILE *f = fopen("/proc/self/maps", "r");
    if (!f) return false;
    char line[512];
    bool ok = false;
    while (fgets(line, sizeof(line), f)) {
        const bool whole = strchr(line, '\n') != nullptr;
        unsigned long long a = 0, b = 0;
        char perms[8] = {0};
        int path_at = 0;
        if (sscanf(line, "%llx-%llx %7s %*s %*s %*s %n", &a, &b, perms, &path_at) < 3) break;
        if (lo >= a && lo < b) {
            const char *path = path_at > 0 ? line + path_at : "";
            ok = hi <= b && perms[0] == 'r' && (!write || perms[1] == 'w') && strncmp(path, "/dev/", 5) != 0;
            break;
        }
        while (!whole && fgets(line, sizeof(line), f) && !strchr(line, '\n')) {}   // rest of a long line
    }
    fclose(f);
    return ok;
}

// host-side packing of pageable io-vector runs, in pair order (fixed-size copies
// for the element sizes GA scatters, so the compiler emits plain loads/stores)
template <int B> static void gather_fixed(char *out, void *const *p, int n) {
    for (int i = 0; i < n; ++i) memcpy(out + (size_t)i * B, p[i], B);
}
template <int B> static void scatter_fixed(void *const *p, const char *in, int n) {
    for (int i = 0; i < n; ++i) memcpy(p[i], in + (size_t)i * B, B);
}
static void gather_runs(char *out, void *const *p, int n, int bytes) {
    switch (bytes) {
    case 4: return gather_fixed<4>(out, p, n);
    case 8: return gather_fixed<8>(out, p, n);
    case 16: return gather_fixed<16>(out, p, n);
    }
    for (int i = 0; i < n; ++i) memcpy(out + (size_t)i * bytes, p[i], (size_t)bytes);
}
static void scatter_runs(void *const *p, const char *in, int n, int bytes) {
    switch (bytes) {
    case 4: return scatter_fixed<4>(p, in, n);
    case 8: return scatter_fixed<8>(p, in, n);
    case 16: return scatter_fixed<16>(p, in, n);
    }
    for (int i = 0; i < n; ++i) memcpy(p[i], in + (size_t)i * bytes, (size_t)bytes);
}

// One pass of an io-vector address list: the device-view address of every entry
// into the upload staging, and their OR, OR of XOR with the first, min and max.
// Host-bound at GA scatter sizes (64 Ki pairs: ~85 us per list on one core with
// baseline x86-64 code), so it is built for AVX-512 and AVX2 as well and the
// loader picks the best the host has (GCC function multiversioning).
__attribute__((optimize("O3"), target_clones("avx512f", "avx2", "default")))
static void translate_range(const uint64_t *in, int64_t delta, uint64_t *u, long n, uint64_t a0, uint64_t *or_out,
                            uint64_t *xor_out, uint64_t *lo_out, uint64_t *hi_out) {
    uint64_t ot = 0, lt = ~0ull, ht = 0, xt = 0;
    for (long i = 0; i < n; ++i) {
        const uint64_t a = in[i] + (uint64_t)delta;
        u[i] = a;
        ot |= a;
        xt |= a ^ a0;
        lt = a < lt ? a : lt;
        ht = a > ht ? a : ht;
    }
    *or_out = ot;
    *xor_out = xt;
    *lo_out = lt;
    *hi_out = ht;
}

// io-vector pairs from this many up use the GPU-sorted run kernel (launch_iov_runs)
// instead of a host-side overlap check
constexpr int kIovRunsMin = 4096;
// io-vectors from this many pairs try the whole-side host test (host_cpu_range)
constexpr int kIovMapsMin = 65536;

// One descriptor on this GPU.  `src` lists device addresses, or is empty when
// `host_src` holds the n source runs packed on the host (gathered from pageable
// memory by the caller); `dst` lists device addresses, or is empty when the
// results go packed to `host_dst` (getv into pageable memory: the caller
// scatters them).  Reference: nb_accv / nb_putv / nb_getv to a self/SMP target,
// comex.c:7327-7400 (one _acc / memcpy per pair, in order).
// `bounds` (the fast path of xfer_vec): {src lo, src hi, dst lo, dst hi} of the
// allocations the first pair's addresses lie in, with sdelta / ddelta their device-view
// offsets; when some listed address falls outside them the call returns false before
// anything is uploaded or launched (the caller classifies per address instead).
// `src_peer`: the listed sources lie in another GPU's memory (getv): system-scope loads.
static bool iov_local(int cop, const void *scale, const uint64_t *src, const uint64_t *dst, int bytes, int n,
                      const char *host_src = nullptr, char *host_dst = nullptr, int64_t sdelta = 0,
                      int64_t ddelta = 0, void *const *gather_src = nullptr, const uint64_t *bounds = nullptr,
                      bool src_peer = false) {
    Runtime &r = rt();
    const bool src_listed = src != nullptr, dst_listed = dst != nullptr;
    // device scratch: [dst list | src list or packed sources | packed results | run-sort work],
    // uploaded from pinned staging; the lists are copied there in the same pass that
    // takes their spans
    const size_t nb = (size_t)n * 8, pk = ((size_t)n * (size_t)bytes + 15) & ~(size_t)15;
    const size_t o_dst = 0, o_src = dst_listed ? nb : 0;
    const size_t o_res = o_src + (src_listed ? nb : pk);
    std::unique_lock<std::mutex> g(r.launch_mu);
    sched_sync_all();   // the previous io-vector kernel and its upload are done with both scratches
    char *up = iov_host_scratch(o_res);
    uint64_t align_or = 0, slo = ~0ull, shi = 0, dlo = ~0ull, dhi = 0, dxor = 0;
    // translate a list into the staging, taking its OR / min / max and the OR of every
    // address XOR the first one (per range, then combined)
    auto translate = [&](const uint64_t *in, int64_t delta, uint64_t *u, uint64_t *lo_out, uint64_t *hi_out,
                         uint64_t *xor_out) {
        const int T = par_threads(n);
        uint64_t o[8] = {0}, lo[8], hi[8] = {0}, xo[8] = {0};
        for (int t = 0; t < 8; ++t) lo[t] = ~0ull;
        const uint64_t a0 = in[0] + (uint64_t)delta;
        par_for(n, T, [&](int t, long i0, long i1) {
            translate_range(in + i0, delta, u + i0, i1 - i0, a0, &o[t], &xo[t], &lo[t], &hi[t]);
        });
        for (int t = 0; t < T; ++t) {
            align_or |= o[t];
            *xor_out |= xo[t];
            *lo_out = std::min(*lo_out, lo[t]);
            *hi_out = std::max(*hi_out, hi[t]);
        }
    };
    uint64_t sxor = 0;
    if (src_listed) {
        translate(src, sdelta, (uint64_t *)(up + o_src), &slo, &shi, &sxor);
        shi += (uint64_t)bytes;
    } else if (gather_src) {
        // pageable sources gathered straight into the pinned staging, in pair order, on
        // one thread: split over 8 threads it measured no faster on the boxes' shared
        // host cores (profiles/r01/iov_host_threads.jsonl)
        gather_runs(up + o_src, gather_src, n, bytes);
    } else {
        memcpy(up + o_src, host_src, (size_t)n * (size_t)bytes);
    }
    if (dst_listed) {
        translate(dst, ddelta, (uint64_t *)(up + o_dst), &dlo, &dhi, &dxor);
        dhi += (uint64_t)bytes;
    }
    if (bounds && src_listed && dst_listed &&
        (slo - (uint64_t)sdelta < bounds[0] || shi - (uint64_t)sdelta > bounds[1] ||
         dlo - (uint64_t)ddelta < bounds[2] || dhi - (uint64_t)ddelta > bounds[3]))
        return false;   // an address outside the first pair's allocations: nothing enqueued yet
    // from here on the lists are the translated (device-view) copies in the staging
    if (src_listed) src = (const uint64_t *)(up + o_src);
    if (dst_listed) dst = (const uint64_t *)(up + o_dst);
    bool serial = false, runs = false;
    if (dst_listed) {
        // a source inside a destination: the reference order matters across pairs
        bool cross = false;
        if (src_listed && slo < dhi && dlo < shi) {
            std::vector<std::pair<uint64_t, uint64_t>> sr((size_t)n), dr((size_t)n);
            for (int i = 0; i < n; ++i) {
                sr[i] = {src[i], src[i] + (uint64_t)bytes};
                dr[i] = {dst[i], dst[i] + (uint64_t)bytes};
            }
            cross = any_cross_overlap(sr, dr);
        }
        // every destination a whole number of pairs from dlo (no partial overlaps)
        bool congruent = true;
        if ((bytes & (bytes - 1)) == 0) {
            // all dst[i] == dst[0] (mod bytes), dlo being one of them: from the translate pass
            congruent = (dxor & (uint64_t)(bytes - 1)) == 0;
        } else {
            const FastDiv fd = make_fastdiv((uint32_t)bytes);   // no 64-bit divide per pair
            for (int i = 0; i < n && congruent; ++i) {
                const uint64_t off = dst[i] - dlo;
                congruent = off < (1ull << 32) ? (uint64_t)fd.div((uint32_t)off) * (uint64_t)bytes == off
                                               : off % (uint64_t)bytes == 0;
            }
        }
        const uint64_t units = (dhi - dlo) / (uint64_t)bytes + 1;
        if (cross) {
            serial = true;
        } else if (n >= kIovRunsMin && congruent && bytes <= kIovRunsMaxBytes && units <= (1ull << 32)) {
            runs = true;   // repeated destinations are ordered on the GPU
        } else {
            std::vector<std::pair<uint64_t, uint64_t>> dr((size_t)n);
            for (int i = 0; i < n; ++i) dr[i] = {dst[i], dst[i] + (uint64_t)bytes};
            serial = ranges_overlap(dr);
        }
    }
    const size_t o_work = (o_res + (dst_listed ? 0 : pk) + 255) & ~(size_t)255;   // sort work: 256-aligned
    const size_t work = runs ? iov_runs_work_bytes((uint32_t)n) : 0;
    char *dev = iov_scratch(o_work + work);
    IovDesc d;
    memset(&d, 0, sizeof(d));
    if (src_listed) d.src_list = (const uint64_t *)(dev + o_src);
    else d.src_base = dev + o_src;
    if (dst_listed) d.dst_list = (const uint64_t *)(dev + o_dst);
    else d.dst_base = dev + o_res;
    d.bytes = bytes;
    d.n = (uint32_t)n;
    Span ss, ds;
    ss.lo = src_listed ? (int64_t)slo : (int64_t)(uintptr_t)(dev + o_src);
    ss.hi = src_listed ? (int64_t)shi : ss.lo + (int64_t)pk;
    ds.lo = dst_listed ? (int64_t)dlo : (int64_t)(uintptr_t)(dev + o_res);
    ds.hi = dst_listed ? (int64_t)dhi : ds.lo + (int64_t)pk;
    const int si = sched_pick(ss, ds);
    // the upload: the copy kernel reading the mapped pinned buffer (no DMA engine
    // round trip before the first io-vector kernel), or the runtime's copy
    static const bool kernel_upload = [] {
        const char *e = getenv("COMEX_AMD_IOV_KERNEL_UPLOAD");
        return !e || atoi(e) != 0;
    }();
    if (kernel_upload) upload_pinned(dev, up, o_res, r.streams[si]);
    else GA_HIP(hipMemcpyAsync(dev, up, o_res, hipMemcpyHostToDevice, r.streams[si]));
    const uint64_t units = runs ? (dhi - dlo) / (uint64_t)bytes + 1 : 0;
    int rc;
    if (runs) {
        // repeated destinations: the hashed path (sorts only the pairs that share a
        // destination), or the radix path above 2^19 pairs / with COMEX_AMD_IOV_HASH=0
        static const bool hash_on = [] {
            const char *e = getenv("COMEX_AMD_IOV_HASH");
            return !e || atoi(e) != 0;
        }();
        static IovHash *g_hash = nullptr;
        rc = 1;
        if (hash_on) {
            if (!g_hash) g_hash = iov_hash_create();
            rc = launch_iov_hashed(g_hash, cop, scale, d, align_or, dlo, units, r.streams[si], src_peer);
            if (rc == 0) {
                // more repeated destinations than the hashed launch orders in LDS: after
                // it completed, the radix path applies the pairs it left (the rest masked)
                GA_HIP(hipStreamSynchronize(r.streams[si]));
                const bool over = iov_hash_overflowed(g_hash);
                g_iov_path[over ? 1 : 0].fetch_add(1, std::memory_order_relaxed);
                if (over)
                    rc = launch_iov_runs(cop, scale, d, align_or, dlo, units, dev + o_work, work, r.streams[si],
                                         src_peer, g_hash);
            }
        }
        if (rc == 1) {
            g_iov_path[2].fetch_add(1, std::memory_order_relaxed);
            rc = launch_iov_runs(cop, scale, d, align_or, dlo, units, dev + o_work, work, r.streams[si], src_peer);
        }
    } else {
        rc = launch_iov(cop, scale, d, align_or, serial, r.streams[si], src_peer);
    }
    if (rc) fatal("io-vector launch failed (%d): misaligned elements?", rc);
    if (!dst_listed) {
        GA_HIP(hipStreamSynchronize(r.streams[si]));
        GA_HIP(hipMemcpy(host_dst, dev + o_res, (size_t)n * (size_t)bytes, hipMemcpyDeviceToHost));
    }
    // completion (blocking call) or the handle (non-blocking) is taken by xfer_vec
    return true;
}

static int xfer_vec(Xfer kind, int op, void *scale, comex_giov_t *darr, int len, int proc, int group,
                    comex_request_t *hdl) {
    ensure_init();
    Runtime &r = rt();
    const int world = translate_world(group, proc);
    const int cop = (kind == X_ACC) ? op : kOpCopy;
    if (kind == X_ACC && (!elem_size(op) || op == kOpCopy || !scale)) fatal("bad accumulate op/scale");
    for (int k = 0; k < len; ++k) {
        const int n = darr[k].count, bytes = darr[k].bytes;
        if (n <= 0) continue;
        if (bytes <= 0) fatal("io-vector of %d bytes", bytes);
        if (!(kind == X_ACC ? r.acc_iov : (kind == X_PUT ? r.put_iov : r.get_iov)) && !self_smp_route(kind, world)) {
            // COMEX_ENABLE_*_IOV=0: pair by pair as contiguous operations (nb_accv's
            // loop, comex.c:7342-7351)
            ContigWindow w;
            for (int i = 0; i < n; ++i) w.issue(kind, op, scale, darr[k].src[i], darr[k].dst[i], bytes, proc, group);
            w.flush();
            g_toggle[1].fetch_add(1, std::memory_order_relaxed);
            continue;
        }
        const bool remote_side_is_dst = (kind != X_GET);
        // the owner applies it (staging + inbox request): every remote accumulate, and
        // a put into another GPU's memory (no rank writes another GPU's HBM)
        const bool remote_apply = world != r.rank && (kind == X_ACC || (kind == X_PUT && r.peer_src(world)));
        // a getv from another GPU's memory reads it with system-scope loads
        const bool getv_peer = kind == X_GET && world != r.rank && r.peer_src(world);
        // address lists in buffers kept across calls: fresh ones cost a page fault per
        // 512 entries, more than the classification itself at scatter-acc sizes
        static std::vector<uint64_t> g_sv, g_dv;
        if (g_sv.size() < (size_t)n) {
            g_sv.resize((size_t)n);
            g_dv.resize((size_t)n);
        }
        uint64_t *sv = g_sv.data(), *dv = g_dv.data();
        bool host_bounce = false;
        if (world == r.rank) fence_self_if_pending();
        if (world != r.rank && !r.same_node(world)) {
            // another node: one io-vector message per descriptor chunk (wire.cpp)
            for (int i = 0; i < n && !host_bounce; ++i) {
                void *sp = darr[k].src[i], *dp = darr[k].dst[i];
                char *d = nullptr;
                if (remote_side_is_dst) {
                    check_remote(world, dp, 0, bytes);
                    dv[i] = (uint64_t)(uintptr_t)dp;
                    if (direct_view(sp, &d)) sv[i] = (uint64_t)(uintptr_t)d;
                    else host_bounce = true;
                } else {
                    check_remote(world, sp, 0, bytes);
                    sv[i] = (uint64_t)(uintptr_t)sp;
                    if (direct_view(dp, &d)) dv[i] = (uint64_t)(uintptr_t)d;
                    else host_bounce = true;
                }
            }
            if (host_bounce) {
                for (int i = 0; i < n; ++i)
                    xfer_contig(kind, op, scale, darr[k].src[i], darr[k].dst[i], bytes, proc, group, nullptr);
            } else if (kind == X_GET) {
                wire_get_iov(sv, dv, n, bytes, world);
            } else {
                std::vector<std::pair<uint64_t, uint64_t>> dr((size_t)n);
                for (int i = 0; i < n; ++i) dr[i] = {dv[i], dv[i] + (uint64_t)bytes};
                wire_send_iov(cop, scale, sv, dv, n, bytes, ranges_overlap(dr), world);
            }
            continue;
        }
        ViewCache vc;
        if (world == r.rank && n >= 1024) {
            // fast path: each side's addresses all inside one device-accessible allocation
            // (GA's `v` buffer and array block): one range lookup per side, the lists go to
            // the staging translated in the same pass that takes their spans
            const uint64_t *rs = (const uint64_t *)darr[k].src, *rd = (const uint64_t *)darr[k].dst;
            {
                // the allocations of the first pair, checked against every address in the
                // translate pass (no separate min/max pass over both lists)
                uint64_t b[4];
                int64_t sd0 = 0, dd0 = 0;
                if (vc.range_of(rs[0], &b[0], &b[1], &sd0) && vc.range_of(rd[0], &b[2], &b[3], &dd0) &&
                    iov_local(cop, scale, rs, rd, bytes, n, nullptr, nullptr, sd0, dd0, nullptr, b))
                    continue;
            }
            uint64_t smin = ~0ull, smax = 0, dmin = ~0ull, dmax = 0;
            {
                const int T = par_threads(n);
                uint64_t mm[8][4];
                par_for(n, T, [&](int t, long i0, long i1) {
                    uint64_t a0 = ~0ull, a1 = 0, b0 = ~0ull, b1 = 0;
                    for (long i = i0; i < i1; ++i) {
                        a0 = rs[i] < a0 ? rs[i] : a0;
                        a1 = rs[i] > a1 ? rs[i] : a1;
                        b0 = rd[i] < b0 ? rd[i] : b0;
                        b1 = rd[i] > b1 ? rd[i] : b1;
                    }
                    mm[t][0] = a0; mm[t][1] = a1; mm[t][2] = b0; mm[t][3] = b1;
                });
                for (int t = 0; t < T; ++t) {
                    smin = std::min(smin, mm[t][0]);
                    smax = std::max(smax, mm[t][1]);
                    dmin = std::min(dmin, mm[t][2]);
                    dmax = std::max(dmax, mm[t][3]);
                }
            }
            int64_t sdel = 0, ddel = 0;
            const bool sdev = vc.span(smin, smax + (uint64_t)bytes, &sdel);
            const bool ddev = vc.span(dmin, dmax + (uint64_t)bytes, &ddel);
            if (sdev && ddev) {
                iov_local(cop, scale, rs, rd, bytes, n, nullptr, nullptr, sdel, ddel);
                continue;
            }
            // one side wholly in pageable host memory (GA's `v`): packed on the host in
            // pair order, as the per-pair classification below would, without it
            if (n >= kIovMapsMin && ddev && !sdev && host_cpu_range(smin, smax + (uint64_t)bytes, false)) {
                iov_local(cop, scale, nullptr, rd, bytes, n, nullptr, nullptr, 0, ddel, darr[k].src);
                continue;
            }
            if (n >= kIovMapsMin && sdev && !ddev && cop == kOpCopy &&
                host_cpu_range(dmin, dmax + (uint64_t)bytes, true)) {
                static std::vector<char> g_hpack;
                if (g_hpack.size() < (size_t)n * (size_t)bytes) g_hpack.resize((size_t)n * (size_t)bytes);
                iov_local(cop, scale, rs, nullptr, bytes, n, nullptr, g_hpack.data(), sdel, 0);
                scatter_runs(darr[k].dst, g_hpack.data(), n, bytes);
                continue;
            }
        }
        bool src_host = false, dst_host = false;   // a whole side in pageable host memory
        bool classified = false;
        if (remote_apply && n >= kIovMapsMin) {
            // remote accumulate from GA's `v`: a source side in one ordinary host mapping is
            // recognised with one lookup (host_cpu_range) instead of a query per page
            const uint64_t *rs = (const uint64_t *)darr[k].src;
            uint64_t smin = ~0ull, smax = 0;
            for (int i = 0; i < n; ++i) {
                smin = rs[i] < smin ? rs[i] : smin;
                smax = rs[i] > smax ? rs[i] : smax;
            }
            if (host_cpu_range(smin, smax + (uint64_t)bytes, false)) {
                src_host = classified = true;
                memcpy(dv, darr[k].dst, (size_t)n * 8);   // owner addresses, checked per chunk below
            }
        }
        for (int i = 0; i < n && !host_bounce && !classified; ++i) {
            void *sp = darr[k].src[i], *dp = darr[k].dst[i];
            uint64_t v = 0;
            if (world != r.rank && !remote_side_is_dst) {
                sv[i] = (uint64_t)(uintptr_t)remote_view(world, sp, 0, bytes);
            } else if (vc.view(sp, bytes, &v)) {
                if (src_host) host_bounce = true;   // mixed host and device sources
                sv[i] = v;
            } else if (i == 0 || src_host) {
                src_host = true;
            } else {
                host_bounce = true;
            }
            if (world != r.rank && remote_side_is_dst) {
                if (remote_apply) dv[i] = (uint64_t)(uintptr_t)dp;   // owner's address, checked below
                else dv[i] = (uint64_t)(uintptr_t)remote_view(world, dp, 0, bytes);
            } else if (vc.view(dp, bytes, &v)) {
                if (dst_host) host_bounce = true;
                dv[i] = v;
            } else if (i == 0 || dst_host) {
                dst_host = true;
            } else {
                host_bounce = true;
            }
        }
        // packed host side: sources of an accumulate/put (local or same-node put), or the
        // results of a copy (get/put into host memory); an accumulate into host memory
        // needs the old values and stays per pair
        if (src_host && dst_host) host_bounce = true;
        if (dst_host && cop != kOpCopy) host_bounce = true;
        if (!host_bounce && (src_host || dst_host) && !remote_apply) {
            // pageable host runs on one side (GA's MA buffer `v` of a scatter/gather): the
            // sources are gathered on the host and uploaded packed, or the results come
            // back packed and are scattered on the host, in pair order
            if (world != r.rank) fence_target(world);
            if (src_host) {   // gathered straight into the pinned upload staging
                iov_local(cop, scale, nullptr, dv, bytes, n, nullptr, nullptr, 0, 0, darr[k].src);
            } else {
                static std::vector<char> g_packed;   // kept across calls (no page faults per call)
                if (g_packed.size() < (size_t)n * (size_t)bytes) g_packed.resize((size_t)n * (size_t)bytes);
                iov_local(cop, scale, sv, nullptr, bytes, n, nullptr, g_packed.data(), 0, 0, nullptr, nullptr,
                          getv_peer);
                scatter_runs(darr[k].dst, g_packed.data(), n, bytes);
            }
            continue;
        }
        if (dst_host) host_bounce = true;   // (a remote accumulate from host sources is gathered below)
        if (host_bounce) {
            // pageable host pairs: per-pair transfers (each maps its pages)
            for (int i = 0; i < n; ++i)
                xfer_contig(kind, op, scale, darr[k].src[i], darr[k].dst[i], bytes, proc, group, nullptr);
            continue;
        }
        if (!remote_apply) {
            if (world != r.rank) fence_target(world);
            iov_local(cop, scale, sv, dv, bytes, n, nullptr, nullptr, 0, 0, nullptr, nullptr, getv_peer);
            continue;
        }
        // remote io-vector accumulate (or put into another GPU): pack the sources + the
        // owner addresses into staging, the owner's progress thread applies them (k_iov)
        drain_target(world);   // its staging ring is allocated and posted in order
        const uint64_t sub = sub_ring_bytes();
        const uint64_t per_pair = (uint64_t)bytes + 8;
        const int pairs_per_req = (int)std::max<uint64_t>(1, (sub - 32) / per_pair);
        for (int i0 = 0; i0 < n; i0 += pairs_per_req) {
            const int m = std::min(pairs_per_req, n - i0);
            uint64_t align_or = 0, dlo = ~0ull, dhi = 0;
            for (int i = 0; i < m; ++i) {
                const uint64_t a = dv[(size_t)i0 + i];
                align_or |= a;
                dlo = std::min(dlo, a);
                dhi = std::max(dhi, a + (uint64_t)bytes);
            }
            // reg_cache_find: one lookup when the chunk's destinations lie in one segment
            // of the owner (a GA block), else one per pair (aborting on a stray address)
            if (segment_of_rank(world, dlo, 0, (int64_t)(dhi - dlo))) {
                (void)remote_view(world, (void *)(uintptr_t)dlo, 0, (int64_t)(dhi - dlo));
            } else {
                for (int i = 0; i < m; ++i)
                    (void)remote_view(world, (void *)(uintptr_t)dv[(size_t)i0 + i], 0, bytes);
            }
            // repeated destinations: the owner orders them on its GPU when every destination
            // is a whole number of pairs from dlo, else a host check picks the serial kernel
            int mode = 0;
            bool congruent = m >= kIovRunsMin && bytes <= kIovRunsMaxBytes &&
                             (dhi - dlo) / (uint64_t)bytes < (1ull << 32);
            for (int i = 0; i < m && congruent; ++i) congruent = (dv[(size_t)i0 + i] - dlo) % (uint64_t)bytes == 0;
            if (congruent) {
                mode = 2;
            } else {
                std::vector<std::pair<uint64_t, uint64_t>> dr((size_t)m);
                for (int i = 0; i < m; ++i) dr[i] = {dv[(size_t)i0 + i], dv[(size_t)i0 + i] + (uint64_t)bytes};
                mode = ranges_overlap(dr) ? 1 : 0;
            }
            const uint64_t loff = iov_list_off(m, bytes);
            const uint64_t len_b = loff + (uint64_t)m * 8;
            const uint64_t off = stage_alloc(world, ring_len(len_b));
            char *stage = r.staging + (size_t)world * sub + off;
            {
                std::lock_guard<std::mutex> g(r.launch_mu);
                // the request's bytes (packed host sources, owner addresses) go up from
                // pinned memory; the previous request's upload from this buffer
                // completed before its post
                char *pin = remote_iov_pinned((size_t)len_b);
                memcpy(pin + loff, dv + i0, (size_t)m * 8);
                if (src_host) {
                    // pageable sources (GA's MA buffer): gathered on the host, one upload
                    gather_runs(pin, darr[k].src + i0, m, bytes);
                    sched_join();
                    upload_pinned(stage, pin, (size_t)len_b, r.streams[0]);
                } else {
                    char *dev = iov_scratch((size_t)m * 8);
                    sched_sync_all();
                    GA_HIP(hipMemcpy(dev, sv + i0, (size_t)m * 8, hipMemcpyHostToDevice));
                    uint64_t salign = 0;
                    for (int i = 0; i < m; ++i) salign |= sv[(size_t)i0 + i];
                    IovDesc d;
                    memset(&d, 0, sizeof(d));
                    d.src_list = (const uint64_t *)dev;
                    d.dst_base = stage;
                    d.bytes = bytes;
                    d.n = (uint32_t)m;
                    sched_join();
                    const int rc = launch_iov(kOpCopy, nullptr, d, salign, false, r.streams[0]);
                    if (rc) fatal("io-vector pack failed (%d)", rc);
                }
                if (!src_host) upload_pinned(stage + loff, pin + loff, (size_t)m * 8, r.streams[0]);
                GA_HIP(hipStreamSynchronize(r.streams[0]));
            }
            const uint64_t seq = ++r.posted[world];
            g_pend[world].push_back({seq, off, ring_len(len_b)});
            r.stage_head[world] = off + ring_len(len_b);
            post_request_iov(world, op, scale, bytes, m, (uint64_t)world * sub + off, len_b, dlo, dhi, align_or,
                             mode);
        }
    }
    // io-vector kernels may sit on any library stream (sched_pick per descriptor):
    // a handle is recorded after a join, so it covers all of them; a blocking call
    // completes locally before returning
    const bool blocking = !hdl && r.blocking_sync;
    {
        std::lock_guard<std::mutex> g(r.launch_mu);
        if (hdl) sched_join();
        else if (blocking) sched_sync_all();
    }
    if (world != r.rank && r.same_node(world) && kind != X_ACC && !blocking && !r.direct_pending.empty())
        r.direct_pending[world] = 1;
    if (hdl) nb_complete_now(hdl, 0, true);
    return COMEX_SUCCESS;
}

// ---- read-modify-write and mutexes -----------------------------------------
// comex_rmw (comex.h:670): the reference sends OP_FETCH_AND_ADD / OP_SWAP to the
// target's progress rank (comex.c:2120-2200), which applies it after every earlier
// message from that source.  Here: on this rank's own memory a one-lane kernel on
// the library stream that last touched those bytes; on a rank of this node a
// request in its inbox (after our earlier requests to it), applied by its progress
// thread on its GPU, the old value coming back through the node shm; on another
// node a wire frame.
static void post_request_rmw(int t, int swap, uint64_t addr, int bytes, uint64_t val) {
    Runtime &r = rt();
    Inbox *ib = inbox_of(r.shm, r.li(t));
    const uint64_t ticket = ib->tail.fetch_add(1, std::memory_order_acq_rel);
    Request &q = ib->slot[ticket % kInboxSlots];
    for (unsigned spins = 0; ib->head.load(std::memory_order_acquire) + kInboxSlots <= ticket; ++spins)
        if (spins > 256) sched_yield();
    for (unsigned spins = 0;; ++spins) {
        uint32_t expect = 0;
        if (q.state.compare_exchange_weak(expect, 1, std::memory_order_acq_rel)) break;
        if (spins > 256) sched_yield();
    }
    q.src_rank = r.rank;
    q.op = swap;
    q.levels = 0;
    memset(q.count, 0, sizeof(q.count));
    memset(q.dst_stride, 0, sizeof(q.dst_stride));
    q.dst_addr = addr;
    q.staging_off = 0;
    q.bytes = (uint64_t)bytes;
    q.seq = 0;
    memset(q.scale, 0, sizeof(q.scale));
    memcpy(q.scale, &val, 8);
    q.kind = 2;
    g_route[3].fetch_add(1, std::memory_order_relaxed);
    q.iov_serial = 0;
    q.iov_align = 0;
    q.dst_hi = 0;
    q.state.store(2, std::memory_order_release);
}

uint64_t rmw_local(int swap, void *addr, int bytes, uint64_t val) {
    Runtime &r = rt();
    // one pinned result word per calling thread (user thread, wire server thread)
    static thread_local uint64_t *host = nullptr, *dev = nullptr;
    if (!host) {
        GA_HIP(hipHostMalloc((void **)&host, sizeof(uint64_t), hipHostMallocMapped));
        GA_HIP(hipHostGetDevicePointer((void **)&dev, host, 0));
    }
    char *d = nullptr;
    if (!direct_view(addr, &d)) fatal("comex_rmw: %p is not device-accessible memory", addr);
    hipStream_t st;
    {
        std::lock_guard<std::mutex> g(r.launch_mu);
        const int si = sched_pick(Span(), span_of(d, 0, bytes));
        st = r.streams[si];
        const int rc = launch_rmw(swap, d, bytes, val, dev, st);
        if (rc) fatal("comex_rmw: launch failed (%d): misaligned word?", rc);
    }
    GA_HIP(hipStreamSynchronize(st));
    return *(volatile uint64_t *)host;
}

// comex_create_mutexes / lock / unlock (comex.h:607-643; the reference keeps the
// lock queues at each node's progress rank, comex.c:2225-2357): every rank's
// mutexes are words in its node's shm (kMaxMutexes per rank); a rank of the same
// node takes one with a compare-and-swap, a rank of another node through a
// try-lock frame served by the owner's wire thread.
static std::vector<int> g_mutex_count;   // mutexes created by every rank

bool mutex_try_local(int owner, int mutex) {
    Runtime &r = rt();
    std::atomic<uint32_t> &w = mutex_words(r.shm, r.node_size, r.li(owner))[mutex];
    uint32_t expect = 0;
    return w.compare_exchange_strong(expect, 1, std::memory_order_acquire);
}

void mutex_release_local(int owner, int mutex) {
    Runtime &r = rt();
    mutex_words(r.shm, r.node_size, r.li(owner))[mutex].store(0, std::memory_order_release);
}

static void check_mutex(int mutex, int proc) {
    if (g_mutex_count.empty()) fatal("comex_lock/unlock before comex_create_mutexes");
    if (mutex < 0 || mutex >= g_mutex_count[proc])
        fatal("mutex %d out of range on rank %d (%d created)", mutex, proc, g_mutex_count[proc]);
}

}  // namespace gaamd

using namespace gaamd;

// ============================================================================
// C ABI
extern "C" {

// a process that exits without comex_finalize (an error path) must not die in
// std::thread's destructor: let the helper threads go with the process
static void exit_without_finalize() {
    Runtime &r = rt();
    if (!r.initialized) return;
    if (r.progress.joinable()) r.progress.detach();
    wire_detach();
}

static void export_alloc(void **p, size_t bytes, hipIpcMemHandle_t *h, const char *what);

int comex_init() {
    Runtime &r = rt();
    if (r.initialized) return COMEX_SUCCESS;
    static bool hook = false;
    if (!hook) {
        atexit(exit_without_finalize);
        hook = true;
    }
    boot_init();
    {
        // a torch wheel bundles a libamdhip64 with the same SONAME: imported
        // before this library it serves our HIP calls, and that build hangs in
        // hipIpcOpenMemHandle of a 2 GiB segment while another is mapped
        // (profiles/r02/README.md)
        const char *rt_path = gaamd_hip_runtime();
        if (strstr(rt_path, "/torch/lib/") && r.rank == 0)
            fprintf(stderr, "ga_amd: HIP calls resolve to %s (loaded before libga_amd); load libga_amd first "
                    "(import ga_amd before torch) to use /opt/rocm's runtime\n", rt_path);
    }
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0)
        fatal("no HIP device visible (%s): libga_amd runs its kernels on an MI355X and has no CPU path",
              hipGetErrorString(e));
    const char *dv = getenv("COMEX_AMD_DEVICE");
    r.device = dv ? atoi(dv) : r.local_rank % ndev;
    GA_HIP(hipSetDevice(r.device));
    // COMEX_AMD_WAIT: how host waits (stream/event synchronisation) wait for the
    // GPU -- spin (lowest wake-up latency, a busy core), yield, or blocking
    // (sleep until the interrupt); unset: the HIP runtime's default
    if (const char *w = getenv("COMEX_AMD_WAIT")) {
        const unsigned f = !strcmp(w, "spin") ? hipDeviceScheduleSpin
                         : !strcmp(w, "yield") ? hipDeviceScheduleYield
                         : !strcmp(w, "blocking") ? hipDeviceScheduleBlockingSync : hipDeviceScheduleAuto;
        if (hipSetDeviceFlags(f) != hipSuccess) {
            (void)hipGetLastError();
            fprintf(stderr, "ga_amd: COMEX_AMD_WAIT=%s not applied (device already active)\n", w);
        }
    }
    GA_HIP(hipStreamCreateWithFlags(&r.stream, hipStreamDefault));
    {
        // which ranks share this physical GPU (PCI bus id): another GPU's memory is
        // read with system-scope loads and never written by this rank (runtime.hpp)
        struct Dev { char bus[32]; int32_t node; } mine_dev;
        memset(&mine_dev, 0, sizeof(mine_dev));
        if (hipDeviceGetPCIBusId(mine_dev.bus, (int)sizeof(mine_dev.bus) - 1, r.device) != hipSuccess) {
            (void)hipGetLastError();
            snprintf(mine_dev.bus, sizeof(mine_dev.bus), "device-%d", r.device);
        }
        mine_dev.node = r.node;
        std::vector<Dev> devs(r.size);
        if (r.size > 1) boot_allgather(&mine_dev, devs.data(), sizeof(Dev));
        else devs[0] = mine_dev;
        r.same_dev.assign(r.size, 0);
        for (int q = 0; q < r.size; ++q)
            r.same_dev[q] = devs[q].node == r.node && !strcmp(devs[q].bus, mine_dev.bus);
        const char *pl = getenv("COMEX_AMD_PEER_LOADS");
        r.peer_loads = (pl && !strcmp(pl, "all")) ? 1 : ((pl && !strcmp(pl, "off")) ? 2 : 0);
        int peers = 0;   // same-node ranks whose memory is read as another GPU's
        for (int q = 0; q < r.size; ++q)
            if (r.same_node(q) && r.peer_src(q)) ++peers;
        // owner pulls from peer GPUs: one stream per source rank, so the chunks of
        // different peers (different xGMI links) are applied side by side
        const char *ps = getenv("COMEX_AMD_PULL_STREAMS");
        const int pull = std::min(peers, ps ? atoi(ps) : 6);
        const char *ns = getenv("COMEX_AMD_STREAMS");
        sched_init(ns ? atoi(ns) : 2, pull);   // 2: independent ops overlap kernel edges
        const char *op1 = getenv("COMEX_AMD_ONE_PASS");
        r.one_pass = false;
        if (!op1 || atoi(op1) != 0)
            for (int q = 0; q < r.size; ++q)
                if (q != r.rank && r.same_node(q) && !r.peer_src(q)) r.one_pass = true;
        r.own_holds = false;
    }
    const char *bs = getenv("COMEX_AMD_BLOCKING_SYNC");
    r.blocking_sync = !bs || atoi(bs) != 0;
    {
        const char *ds = getenv("COMEX_AMD_DIRECT_SRC");
        r.direct_src = !ds || atoi(ds) != 0;
        auto flag = [](const char *name) {
            const char *v = getenv(name);
            return !v || atoi(v) != 0;
        };
        r.acc_smp_direct = flag("COMEX_ENABLE_ACC_SMP");
        r.acc_self_direct = flag("COMEX_ENABLE_ACC_SELF") || r.acc_smp_direct;
        r.put_smp_direct = flag("COMEX_ENABLE_PUT_SMP");
        r.put_self_direct = flag("COMEX_ENABLE_PUT_SELF") || r.put_smp_direct;
        r.get_smp_direct = flag("COMEX_ENABLE_GET_SMP");
        r.get_self_direct = flag("COMEX_ENABLE_GET_SELF") || r.get_smp_direct;
        r.acc_packed = flag("COMEX_ENABLE_ACC_PACKED");
        r.put_packed = flag("COMEX_ENABLE_PUT_PACKED");
        r.get_packed = flag("COMEX_ENABLE_GET_PACKED");
        r.acc_iov = flag("COMEX_ENABLE_ACC_IOV");
        r.put_iov = flag("COMEX_ENABLE_PUT_IOV");
        r.get_iov = flag("COMEX_ENABLE_GET_IOV");
    }
    const char *dbg = getenv("COMEX_AMD_DEBUG");
    r.debug = dbg ? atoi(dbg) : 0;
    if (r.size > 1 || !r.acc_self_direct || !r.put_self_direct || !r.get_self_direct) {
        // staging HBM for remote accumulates, exported to every local rank
        const char *mb = getenv("COMEX_AMD_STAGING_MB");
        r.staging_bytes = (size_t)(mb ? atol(mb) : 256) << 20;
        GA_HIP(hipMalloc((void **)&r.staging, r.staging_bytes));
        addr_event('a', r.staging, r.staging_bytes, -1);
        struct { hipIpcMemHandle_t h; uint64_t bytes; } mine, *all;
        memset(&mine, 0, sizeof(mine));
        export_alloc((void **)&r.staging, r.staging_bytes, &mine.h, "staging buffer");
        mine.bytes = r.staging_bytes;
        {
            const uint64_t t = seg_tag(r.rank, 0, 0);   // checked by every peer below
            GA_HIP(hipMemcpy(r.staging, &t, 8, hipMemcpyHostToDevice));
        }
        std::vector<char> buf(sizeof(mine) * (size_t)r.size);
        boot_allgather(&mine, buf.data(), sizeof(mine));
        all = reinterpret_cast<decltype(all)>(buf.data());
        r.peer_staging.assign(r.size, nullptr);
        for (int q = 0; q < r.size; ++q) {
            if (q == r.rank) { r.peer_staging[q] = r.staging; continue; }
            if (!r.same_node(q)) continue;   // another node: reached through wire.cpp
            r.peer_staging[q] = (char *)ipc_open(all[q].h, q, "staging buffer");
        }
        // as for segments (do_malloc): every staging mapping must read its owner's tag
        // (written before the exchange below the allgather's barrier) -- a mapping of
        // the wrong allocation would hand the owners other bytes to accumulate
        boot_barrier();
        for (int q = 0; q < r.size; ++q) {
            if (q == r.rank || !r.peer_staging[q] || all[q].bytes < 8) continue;
            uint64_t t = 0;
            GA_HIP(hipMemcpy(&t, r.peer_staging[q], 8, hipMemcpyDeviceToHost));
            if (t != seg_tag(q, 0, 0))
                fatal("the IPC mapping of rank %d's staging buffer reads %#llx, not its tag: another allocation's "
                      "memory", q, (unsigned long long)t);
        }
        boot_barrier();   // nobody reads a tag any more: the rings may be written
        r.posted.assign(r.size, 0);
        r.stage_head.assign(r.size, 0);
        r.direct_pending.assign(r.size, 0);
        g_pend.assign(r.size, {});
        r.stop.store(false);
        r.progress = std::thread(progress_loop);
        wire_init();
    }
    r.initialized = true;
    boot_barrier();
    // the ARMCI_VERBOSE dump of the reference (comex.c:545-572): this run's configuration
    const char *vb = getenv("COMEX_AMD_VERBOSE");
    if (vb && atoi(vb) && r.rank == 0) {
        hipDeviceProp_t prop;
        const bool okp = hipGetDeviceProperties(&prop, r.device) == hipSuccess;
        const char *async = getenv("COMEX_AMD_ASYNC_ACC");
        const char *seg = getenv("COMEX_AMD_SEGMENT");
        fprintf(stderr,
                "%s: ranks %d on %d node(s), device %d (%s, %d CUs), library streams %d, "
                "staging %zu MiB/rank, remote acc %s, segments in %s, blocking sync %d, "
                "acc to self %s, put to self %s, same-node put %s\n",
                gaamd_version(), r.size, r.nnodes, r.device, okp ? prop.gcnArchName : "?",
                okp ? prop.multiProcessorCount : 0, (int)r.streams.size(), r.staging_bytes >> 20,
                (async && !atoi(async)) ? "synchronous" : "asynchronous jobs", (seg && !strcmp(seg, "host")) ? "host" : "HBM",
                r.blocking_sync ? 1 : 0, r.acc_self_direct ? "direct" : "packed",
                r.put_self_direct ? "direct" : "packed", r.put_smp_direct ? "IPC" : "packed");
    }
    return COMEX_SUCCESS;
}

int comex_init_args(int *argc, char ***argv) {
    (void)argc;
    (void)argv;
    return comex_init();
}

int comex_initialized() { return rt().initialized ? 1 : 0; }

int comex_finalize() {
    Runtime &r = rt();
    if (!r.initialized) return COMEX_SUCCESS;
    comex_barrier(COMEX_GROUP_WORLD);   // drains every remote accumulate job
    {
        std::lock_guard<std::mutex> g(g_op_mu);   // one-pass locks were handed back by the barrier's fence
        for (OnePassHold &h : g_op_hold)
            for (hipEvent_t e : h.evs) (void)hipEventDestroy(e);
        g_op_hold.clear();
        for (hipEvent_t e : g_op_pool) (void)hipEventDestroy(e);
        g_op_pool.clear();
    }
    for (hipEvent_t e : g_chunk_ev) (void)hipEventDestroy(e);
    g_chunk_ev.clear();
    g_out.clear();
    wire_finalize();
    if (r.progress.joinable()) {
        r.stop.store(true, std::memory_order_release);
        r.progress.join();
    }
    boot_barrier();
    for (Segment &s : r.segs) {
        if (!s.live) continue;
        for (int q = 0; q < (int)s.peer.size(); ++q)
            if (q != r.rank && s.peer[q].mapped) ipc_close(s.peer[q].mapped, q);
        if (s.local && s.device) addr_event('f', s.local, s.peer[r.rank].bytes, -1);
        if (s.local) (void)(s.device ? hipFree(s.local) : hipHostFree(s.local));
        s.live = false;
    }
    r.segs.clear();
    for (int q = 0; q < (int)r.peer_staging.size(); ++q)
        if (q != r.rank && r.peer_staging[q]) ipc_close(r.peer_staging[q], q);
    r.peer_staging.clear();
    boot_barrier();
    if (r.staging) addr_event('f', r.staging, r.staging_bytes, -1);
    if (r.staging) (void)hipFree(r.staging);
    r.staging = nullptr;
    segment_cache_flush();
    for (void *q : g_quarantine) (void)hipFree(q);
    g_quarantine.clear();
    sched_sync_all();
    sched_fini();
    if (g_get_scratch) (void)hipFree(g_get_scratch);
    g_get_scratch = nullptr;
    g_get_scratch_bytes = 0;
    if (g_get_scratch_ev) (void)hipEventDestroy(g_get_scratch_ev);
    g_get_scratch_ev = nullptr;
    if (g_iov_scratch) (void)hipFree(g_iov_scratch);
    g_iov_scratch = nullptr;
    if (g_iov_host) (void)hipHostFree(g_iov_host);
    g_iov_host = nullptr;
    g_iov_host_bytes = 0;
    g_iov_scratch_bytes = 0;
    (void)hipStreamDestroy(r.stream);
    r.stream = nullptr;
    r.initialized = false;
    boot_finalize();
    return COMEX_SUCCESS;
}

void comex_error(const char *msg, int code) { fatal("comex_error: %s (code %d)", msg, code); }

int comex_group_create(int n, int *pid_list, comex_group_t group, comex_group_t *new_group) {
    ensure_init();
    std::vector<int> g;
    for (int i = 0; i < n; ++i) g.push_back(translate_world(group, pid_list[i]));
    g_groups.push_back(g);
    *new_group = (comex_group_t)g_groups.size();
    return COMEX_SUCCESS;
}

int comex_group_free(comex_group_t group) {
    if (group >= 1 && group <= (int)g_groups.size()) g_groups[group - 1].clear();
    return COMEX_SUCCESS;
}

int comex_group_rank(comex_group_t group, int *rank) {
    Runtime &r = rt();
    if (group == COMEX_GROUP_WORLD) { *rank = r.rank; return COMEX_SUCCESS; }
    const std::vector<int> &g = g_groups.at(group - 1);
    *rank = -1;
    for (int i = 0; i < (int)g.size(); ++i) if (g[i] == r.rank) *rank = i;
    return COMEX_SUCCESS;
}

int comex_group_size(comex_group_t group, int *size) {
    *size = (group == COMEX_GROUP_WORLD) ? rt().size : (int)g_groups.at(group - 1).size();
    return COMEX_SUCCESS;
}

int comex_group_translate_world(comex_group_t group, int group_rank, int *world_rank) {
    *world_rank = translate_world(group, group_rank);
    return COMEX_SUCCESS;
}

int comex_fence_proc(int proc, comex_group_t group) {
    ensure_init();
    fence_target(translate_world(group, proc));
    {
        std::lock_guard<std::mutex> g(rt().launch_mu);
        sched_sync_all();
    }
    one_pass_reap(true);   // our one-pass kernels are done: hand the owners' locks back
    return COMEX_SUCCESS;
}

int comex_fence_all(comex_group_t group) {
    ensure_init();
    (void)group;
    Runtime &r = rt();
    drain_all_jobs();   // every target's chunks posted (side by side), then wait for each
    for (int t = 0; t < r.size; ++t) fence_target(t);
    {
        std::lock_guard<std::mutex> g(r.launch_mu);
        sched_sync_all();
    }
    one_pass_reap(true);
    return COMEX_SUCCESS;
}

int comex_barrier(comex_group_t group) {
    ensure_init();
    comex_fence_all(group);
    if (group == COMEX_GROUP_WORLD) boot_barrier();
    else members_barrier(group_members(group), group);   // the group's members only (groups.c barrier)
    return COMEX_SUCCESS;
}

// ---- put ----
int comex_put(void *src, void *dst, int bytes, int proc, comex_group_t group) {
    return xfer_contig(X_PUT, 0, nullptr, src, dst, bytes, proc, group, nullptr);
}
int comex_puts(void *src, int *src_stride, void *dst, int *dst_stride, int *count, int stride_levels, int proc,
               comex_group_t group) {
    return xfer(X_PUT, 0, nullptr, src, src_stride, dst, dst_stride, count, stride_levels, proc, group, nullptr);
}
int comex_putv(comex_giov_t *darr, int len, int proc, comex_group_t group) {
    return xfer_vec(X_PUT, 0, nullptr, darr, len, proc, group, nullptr);
}
int comex_nbput(void *src, void *dst, int bytes, int proc, comex_group_t group, comex_request_t *h) {
    return xfer_contig(X_PUT, 0, nullptr, src, dst, bytes, proc, group, h);
}
int comex_nbputs(void *src, int *src_stride, void *dst, int *dst_stride, int *count, int stride_levels, int proc,
                 comex_group_t group, comex_request_t *h) {
    return xfer(X_PUT, 0, nullptr, src, src_stride, dst, dst_stride, count, stride_levels, proc, group, h);
}
int comex_nbputv(comex_giov_t *darr, int len, int proc, comex_group_t group, comex_request_t *h) {
    return xfer_vec(X_PUT, 0, nullptr, darr, len, proc, group, h);
}

// ---- accumulate ----
int comex_acc(int op, void *scale, void *src, void *dst, int bytes, int proc, comex_group_t group) {
    return xfer_contig(X_ACC, op, scale, src, dst, bytes, proc, group, nullptr);
}
int comex_accs(int op, void *scale, void *src, int *src_stride, void *dst, int *dst_stride, int *count,
               int stride_levels, int proc, comex_group_t group) {
    return xfer(X_ACC, op, scale, src, src_stride, dst, dst_stride, count, stride_levels, proc, group, nullptr);
}
int comex_accv(int op, void *scale, comex_giov_t *darr, int len, int proc, comex_group_t group) {
    return xfer_vec(X_ACC, op, scale, darr, len, proc, group, nullptr);
}
int comex_nbacc(int op, void *scale, void *src, void *dst, int bytes, int proc, comex_group_t group,
                comex_request_t *h) {
    return xfer_contig(X_ACC, op, scale, src, dst, bytes, proc, group, h);
}
int comex_nbaccs(int op, void *scale, void *src, int *src_stride, void *dst, int *dst_stride, int *count,
                 int stride_levels, int proc, comex_group_t group, comex_request_t *h) {
    return xfer(X_ACC, op, scale, src, src_stride, dst, dst_stride, count, stride_levels, proc, group, h);
}
int comex_nbaccv(int op, void *scale, comex_giov_t *darr, int len, int proc, comex_group_t group,
                 comex_request_t *h) {
    return xfer_vec(X_ACC, op, scale, darr, len, proc, group, h);
}

// ---- get ----
int comex_get(void *src, void *dst, int bytes, int proc, comex_group_t group) {
    return xfer_contig(X_GET, 0, nullptr, src, dst, bytes, proc, group, nullptr);
}
int comex_gets(void *src, int *src_stride, void *dst, int *dst_stride, int *count, int stride_levels, int proc,
               comex_group_t group) {
    return xfer(X_GET, 0, nullptr, src, src_stride, dst, dst_stride, count, stride_levels, proc, group, nullptr);
}
int comex_getv(comex_giov_t *darr, int len, int proc, comex_group_t group) {
    return xfer_vec(X_GET, 0, nullptr, darr, len, proc, group, nullptr);
}
int comex_nbget(void *src, void *dst, int bytes, int proc, comex_group_t group, comex_request_t *h) {
    return xfer_contig(X_GET, 0, nullptr, src, dst, bytes, proc, group, h);
}
int comex_nbgets(void *src, int *src_stride, void *dst, int *dst_stride, int *count, int stride_levels, int proc,
                 comex_group_t group, comex_request_t *h) {
    return xfer(X_GET, 0, nullptr, src, src_stride, dst, dst_stride, count, stride_levels, proc, group, h);
}
int comex_nbgetv(comex_giov_t *darr, int len, int proc, comex_group_t group, comex_request_t *h) {
    return xfer_vec(X_GET, 0, nullptr, darr, len, proc, group, h);
}

// ---- completion ----
int comex_wait(comex_request_t *h) {
    ensure_init();
    Runtime &r = rt();
    if (!h || *h < 0 || *h >= kMaxNb) return COMEX_SUCCESS;
    if (r.nb_used[*h]) {
        if (g_nb_job[*h]) run_job(g_nb_job[*h]);
        g_nb_job[*h] = 0;
        if (g_nb_rseq[*h]) wait_done(g_nb_rt[*h], g_nb_rseq[*h]);
        g_nb_rseq[*h] = 0;
        (void)sched_complete(r.nb_stream[*h], r.nb_seq[*h], true);
        r.nb_used[*h] = false;
    }
    *h = -1;
    return COMEX_SUCCESS;
}

int comex_test(comex_request_t *h, int *status) {
    ensure_init();
    Runtime &r = rt();
    *status = 0;   // 0 = complete (reference returns status 0 when done)
    if (!h || *h < 0 || *h >= kMaxNb || !r.nb_used[*h]) return COMEX_SUCCESS;
    if (g_nb_job[*h]) {
        progress_jobs();
        if (find_job(g_nb_job[*h])) { *status = 1; return COMEX_SUCCESS; }
        g_nb_job[*h] = 0;
    }
    if (g_nb_rseq[*h]) {
        if (r.shm->done[r.li(r.rank)][r.li(g_nb_rt[*h])].load(std::memory_order_acquire) < g_nb_rseq[*h]) {
            *status = 1;
            return COMEX_SUCCESS;
        }
        g_nb_rseq[*h] = 0;
    }
    if (!sched_complete(r.nb_stream[*h], r.nb_seq[*h], false)) { *status = 1; return COMEX_SUCCESS; }
    r.nb_used[*h] = false;
    *h = -1;
    return COMEX_SUCCESS;
}

int comex_wait_all(comex_group_t group) {
    stamp(5);
    ensure_init();
    (void)group;
    Runtime &r = rt();
    drain_all_jobs();
    for (int t = 0; t < (int)g_direct_last.size(); ++t)
        if (g_direct_last[t]) wait_done(t, g_direct_last[t]);
    for (int i = 0; i < kMaxNb; ++i) {
        g_nb_job[i] = 0;
        g_nb_rseq[i] = 0;
    }
    {
        std::lock_guard<std::mutex> g(r.launch_mu);
        stamp(6);
        sched_sync_all();
        stamp(7);
    }
    one_pass_reap(true);
    for (int i = 0; i < kMaxNb; ++i) r.nb_used[i] = false;
    return COMEX_SUCCESS;
}

int comex_wait_proc(int proc, comex_group_t group) {
    (void)proc;
    return comex_wait_all(group);
}

// ---- memory ----
// IPC handle of a fresh hipMalloc block `*p`.  Round 2 saw the runtime refuse,
// once in 6 two-rank C5 runs, to export a fresh 64 MiB segment whose base and size
// were exactly the allocation's (invalid argument).  tools/ipc_export_probe.py
// drove the candidate sequences -- re-export after the peer closed, after a free
// while the peer still maps, an importer's VA reused for its own export, double
// export, the bench's mixed 64 MiB / 1 GiB pattern -- 96 rounds, 0 refusals
// (profiles/r03/): the cause is not identified.  A refusal now prints every
// export, IPC map/unmap, alloc and free this process made over that address range
// (addr_history), then allocates another block while holding the refused one, up
// to 4 times; COMEX_AMD_IPC_RETRY=0 makes the first refusal fatal instead.
static void *device_alloc(size_t bytes);

static void export_alloc(void **p, size_t bytes, hipIpcMemHandle_t *h, const char *what) {
    Runtime &r = rt();
    static const bool retry = [] {
        const char *e = getenv("COMEX_AMD_IPC_RETRY");
        return !e || atoi(e) != 0;
    }();
    std::vector<void *> held;
    hipError_t e = hipIpcGetMemHandle(h, *p);
    for (int tries = 0; e != hipSuccess && tries < 4; ++tries) {
        (void)hipGetLastError();
        fprintf(stderr, "[ga_amd %d] hipIpcGetMemHandle of a %zu-byte %s at %p failed (%s)\n", r.rank, bytes, what, *p,
                hipGetErrorString(e));
        addr_history(*p, bytes);
        if (!retry) break;
        fprintf(stderr, "[ga_amd %d]   allocating another block (COMEX_AMD_IPC_RETRY=0: abort instead)\n", r.rank);
        held.push_back(*p);
        *p = device_alloc(bytes);
        addr_event('a', *p, bytes, -1);
        e = hipIpcGetMemHandle(h, *p);
    }
    // a refused block is kept, not freed, until comex_finalize: freed, its address
    // would come back from hipMalloc and be refused again
    for (void *q : held) g_quarantine.push_back(q);
    if (e != hipSuccess) fatal("hipIpcGetMemHandle of a %zu-byte %s failed: %s", bytes, what, hipGetErrorString(e));
    addr_event('x', *p, bytes, -1);
}

// Freed device segments are kept for the next comex_malloc of the same size, with
// their IPC export, instead of going back to hipFree (COMEX_AMD_SEGMENT_CACHE_MB,
// default 16 GiB per rank; 0 disables).  GA creates and destroys arrays of the same
// shapes over and over; every hipFree + hipMalloc + export cycle recycles addresses
// and descriptors, and the runtime refuses, now and then, to export a fresh block at
// a recycled address (profiles/r03/s19, s20, s27-s29: 1-4 refusals in most runs of
// eight ranks on one GPU).  A cached block is exported once, for good, and a reused
// one is opened again by the peers from the same handle.
struct CachedBlock {
    void *p;
    size_t bytes;
    bool exported;
    hipIpcMemHandle_t h;
};
static std::deque<CachedBlock> g_blocks;   // oldest first
static size_t g_blocks_bytes = 0;
static std::atomic<unsigned long long> g_block_reuse{0};
static std::atomic<unsigned long long> g_remapped{0};   // segments replaced after a stale peer mapping

static size_t block_cache_cap() {
    static const size_t v = [] {
        const char *e = getenv("COMEX_AMD_SEGMENT_CACHE_MB");
        return (size_t)(e ? atof(e) : 16384.0) << 20;
    }();
    return v;
}

static void block_free_one(const CachedBlock &b) {
    addr_event('f', b.p, b.bytes, -1);
    GA_HIP(hipFree(b.p));
}

static void block_flush() {
    for (const CachedBlock &b : g_blocks) block_free_one(b);
    g_blocks.clear();
    g_blocks_bytes = 0;
}



extern "C" unsigned long long gaamd_segment_cache_reuse(void) { return g_block_reuse.load(); }
extern "C" unsigned long long gaamd_segment_remaps(void) { return g_remapped.load(); }

static void block_put(void *p, size_t bytes, bool exported, const hipIpcMemHandle_t &h) {
    const size_t cap = block_cache_cap();
    if (bytes > cap) {
        block_free_one({p, bytes, exported, h});
        return;
    }
    while (g_blocks_bytes + bytes > cap && !g_blocks.empty()) {
        block_free_one(g_blocks.front());
        g_blocks_bytes -= g_blocks.front().bytes;
        g_blocks.pop_front();
    }
    g_blocks.push_back({p, bytes, exported, h});
    g_blocks_bytes += bytes;
}

// a cached block of exactly `bytes`; its export in *h when it has one
static bool block_take(size_t bytes, void **p, bool *exported, hipIpcMemHandle_t *h) {
    for (auto it = g_blocks.begin(); it != g_blocks.end(); ++it) {
        if (it->bytes != bytes) continue;
        *p = it->p;
        *exported = it->exported;
        if (it->exported) *h = it->h;
        g_blocks_bytes -= bytes;
        g_blocks.erase(it);
        g_block_reuse.fetch_add(1, std::memory_order_relaxed);
        addr_event('r', *p, bytes, -1);
        return true;
    }
    return false;
}

// hipMalloc, giving the cached blocks back first when the device is full
static void *device_alloc(size_t bytes) {
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipErrorOutOfMemory && !g_blocks.empty()) {
        (void)hipGetLastError();
        block_flush();
        e = hipMalloc(&p, bytes);
    }
    if (e != hipSuccess) fatal("hipMalloc of %zu bytes failed: %s", bytes, hipGetErrorString(e));
    return p;
}

// Every segment gets a per-rank, per-allocation tag in its first and last 8 bytes
// before its handle goes out, and every peer reads both through its fresh mapping.
// Eight ranks on one GPU (profiles/r03/s32), with freed blocks going back to the
// runtime: in 2 of 30 runs, after the runtime had refused an export and a new block
// was exported instead, EVERY peer's mapping of that rank's new block reached other
// memory -- the block later read only its owner's own contribution, nobody else's,
// with no error anywhere.  A mapping that does not read the tags is therefore
// closed, the owner's block set aside (quarantined) and replaced, and the exchange
// repeated (all ranks, collectively), up to 4 times.


static int do_malloc(void **ptr_arr, size_t bytes, comex_group_t group, bool device) {
    ensure_init();
    Runtime &r = rt();
    // collective over the group's members (comex.c comex_malloc): ptr_arr is
    // indexed by group rank; non-members keep no view of the segment
    const std::vector<int> members = group_members(group);
    const bool trace = r.debug >= 2;
    if (trace) fprintf(stderr, "[ga_amd %d] comex_malloc(%zu, group %d): enter\n", r.rank, bytes, group);
    struct Info { uint64_t base, bytes; hipIpcMemHandle_t h; int32_t device, pad; uint64_t gen; } mine;
    memset(&mine, 0, sizeof(mine));
    static uint64_t gen = 0;   // this rank's allocation counter (the tags)
    void *p = nullptr;
    bool exported = false;
    if (bytes) {
        if (device) {
            if (!block_take(bytes, &p, &exported, &mine.h)) {
                p = device_alloc(bytes);
                addr_event('a', p, bytes, -1);
            }
            if (r.debug) {
                void *base = nullptr;
                size_t sz = 0;
                (void)hipMemGetAddressRange((hipDeviceptr_t *)&base, &sz, (hipDeviceptr_t)p);
                fprintf(stderr, "[ga_amd %d] segment %p (%zu B): allocation base %p size %zu\n", r.rank, p,
                        bytes, base, sz);
            }
            if (r.size > 1 && !exported) {
                export_alloc(&p, bytes, &mine.h, "segment");
                exported = true;
            }
        } else {
            GA_HIP(hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocPortable));
        }
    }
    const bool tagged = device && bytes >= 16;
    std::vector<Info> all(r.size);
    std::vector<void *> mapped(r.size, nullptr);
    for (int attempt = 0;; ++attempt) {
        mine.base = (uint64_t)(uintptr_t)p;
        mine.bytes = bytes;
        mine.device = r.device;
        mine.gen = ++gen;
        if (tagged) {
            const uint64_t t0 = seg_tag(r.rank, mine.gen, 0), t1 = seg_tag(r.rank, mine.gen, 1);
            GA_HIP(hipMemcpy(p, &t0, 8, hipMemcpyHostToDevice));
            GA_HIP(hipMemcpy((char *)p + bytes - 8, &t1, 8, hipMemcpyHostToDevice));
        }
        if (trace) fprintf(stderr, "[ga_amd %d] comex_malloc: allocated %p, allgather\n", r.rank, p);
        std::vector<Info> gathered(members.size());
        members_allgather(members, group, &mine, gathered.data(), sizeof(Info));
        if (trace) fprintf(stderr, "[ga_amd %d] comex_malloc: allgather done, opening peers\n", r.rank);
        memset(all.data(), 0, sizeof(Info) * all.size());
        for (size_t k = 0; k < members.size(); ++k) {
            all[members[k]] = gathered[k];
            ptr_arr[k] = (void *)(uintptr_t)gathered[k].base;
        }
        // open, and check that each mapping reads its owner's tags
        std::vector<uint8_t> stale(r.size, 0);
        for (int q = 0; q < r.size; ++q) {
            mapped[q] = nullptr;
            if (q == r.rank || !all[q].bytes || !r.same_node(q)) continue;
            if (!device) fatal("host-memory segments are rank-private (use device segments for remote access)");
            mapped[q] = ipc_open(all[q].h, q, "segment");
            if (!mapped[q] || all[q].bytes < 16) continue;
            uint64_t t[2] = {0, 0};
            GA_HIP(hipMemcpy(&t[0], mapped[q], 8, hipMemcpyDeviceToHost));
            GA_HIP(hipMemcpy(&t[1], (char *)mapped[q] + all[q].bytes - 8, 8, hipMemcpyDeviceToHost));
            if (t[0] != seg_tag(q, all[q].gen, 0) || t[1] != seg_tag(q, all[q].gen, 1)) {
                stale[q] = 1;
                fprintf(stderr, "[ga_amd %d] the IPC mapping of rank %d's new %zu-byte segment (%p in its space) "
                        "reads %#llx / %#llx, not its tags: another allocation's memory\n", r.rank, q,
                        (size_t)all[q].bytes, (void *)(uintptr_t)all[q].base, (unsigned long long)t[0],
                        (unsigned long long)t[1]);
            }
        }
        std::vector<uint8_t> seen(members.size() * (size_t)r.size);
        members_allgather(members, group, stale.data(), seen.data(), (size_t)r.size);
        bool any = false, mine_stale = false;
        for (size_t k = 0; k < members.size(); ++k)
            for (int q = 0; q < r.size; ++q)
                if (seen[k * (size_t)r.size + q]) {
                    any = true;
                    if (q == r.rank) mine_stale = true;
                }
        if (!any) break;
        if (attempt >= 3) fatal("IPC mappings of a new segment keep reaching other memory (4 attempts)");
        for (int q = 0; q < r.size; ++q)
            if (mapped[q]) ipc_close(mapped[q], q);
        if (mine_stale) {
            // set the block aside for good and export a fresh one
            addr_history(p, bytes);
            g_quarantine.push_back(p);
            p = device_alloc(bytes);
            addr_event('a', p, bytes, -1);
            export_alloc(&p, bytes, &mine.h, "segment");
            g_remapped.fetch_add(1, std::memory_order_relaxed);
        }
        members_barrier(members, group);   // every stale mapping closed before the next round
    }
    Segment s;
    s.peer.resize(r.size);
    for (int q : members) s.peer[q].member = true;
    s.live = true;
    s.device = device;
    s.local = p;
    s.local_bytes = bytes;
    s.exported = exported;
    if (exported) s.handle = mine.h;
    for (int q = 0; q < r.size; ++q) {
        s.peer[q].base = all[q].base;
        s.peer[q].bytes = all[q].bytes;
        s.peer[q].mapped = q == r.rank ? (char *)p : (char *)mapped[q];
    }
    {
        std::lock_guard<std::mutex> g(r.seg_mu);
        r.segs.push_back(std::move(s));
    }
    if (trace) fprintf(stderr, "[ga_amd %d] comex_malloc: peers mapped, barrier\n", r.rank);
    members_barrier(members, group);
    if (trace) fprintf(stderr, "[ga_amd %d] comex_malloc: done\n", r.rank);
    return COMEX_SUCCESS;
}

int comex_malloc(void **ptr_arr, size_t bytes, comex_group_t group) {
    const char *where = getenv("COMEX_AMD_SEGMENT");
    const bool host = where && !strcmp(where, "host");
    return do_malloc(ptr_arr, bytes, group, !host);
}

int comex_malloc_mem_dev(void **ptr_arr, size_t bytes, comex_group_t group, const char *device) {
    const bool host = device && (!strcmp(device, "host") || !strcmp(device, "cpu") || !strcmp(device, "dram"));
    return do_malloc(ptr_arr, bytes, group, !host);
}

int comex_free(void *ptr, comex_group_t group) {
    ensure_init();
    Runtime &r = rt();
    const std::vector<int> members = group_members(group);
    comex_fence_all(group);
    std::vector<uint64_t> gathered(members.size()), all(r.size, 0);
    uint64_t mine = (uint64_t)(uintptr_t)ptr;
    members_allgather(members, group, &mine, gathered.data(), sizeof(mine));
    for (size_t k = 0; k < members.size(); ++k) all[members[k]] = gathered[k];
    members_barrier(members, group);   // nobody still reads the segment
    void *local = nullptr;
    bool device = true, found = false, exported = false;
    size_t local_bytes = 0;
    hipIpcMemHandle_t handle;
    memset(&handle, 0, sizeof(handle));
    {
        std::lock_guard<std::mutex> g(r.seg_mu);
        for (Segment &s : r.segs) {
            if (!s.live) continue;
            bool match = true;
            for (int q = 0; q < r.size; ++q) if (s.peer[q].base != all[q]) { match = false; break; }
            if (!match) continue;
            for (int q = 0; q < r.size; ++q)
                if (q != r.rank && s.peer[q].mapped) ipc_close(s.peer[q].mapped, q);
            local = s.local;
            device = s.device;
            local_bytes = s.local_bytes;
            exported = s.exported;
            if (exported) handle = s.handle;
            s.live = false;
            s.local = nullptr;
            found = true;
            break;
        }
    }
    if (!found) fatal("comex_free(%p): not a comex_malloc segment", ptr);
    // every member has closed its mapping of every block before any block is freed:
    // freeing a block a peer still maps leaves its export alive, and the runtime then
    // refuses to export a new allocation it hands out at the same address
    // (hipIpcGetMemHandle: invalid argument in the next comex_malloc)
    members_barrier(members, group);
    if (local && device) {
        if (block_cache_cap()) block_put(local, local_bytes, exported, handle);   // kept for the next comex_malloc
        else block_free_one({local, local_bytes, exported, handle});
    } else if (local) {
        GA_HIP(hipHostFree(local));
    }
    return COMEX_SUCCESS;
}

int comex_free_dev(void *ptr, comex_group_t group) { return comex_free(ptr, group); }

void *comex_malloc_local(size_t bytes) {
    ensure_init();
    void *p = nullptr;
    if (bytes == 0) return nullptr;
    GA_HIP(hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocPortable));
    return p;
}

int comex_free_local(void *ptr) {
    if (ptr) GA_HIP(hipHostFree(ptr));
    return COMEX_SUCCESS;
}

// ---- read-modify-write (comex.h:670) ----
int comex_rmw(int op, void *ploc, void *prem, int extra, int proc, comex_group_t group) {
    ensure_init();
    Runtime &r = rt();
    progress_jobs();
    const int world = translate_world(group, proc);
    int bytes, swap;
    uint64_t val;
    switch (op) {
    case COMEX_FETCH_AND_ADD: bytes = 4; swap = 0; val = (uint64_t)(uint32_t)extra; break;
    case COMEX_FETCH_AND_ADD_LONG: bytes = 8; swap = 0; val = (uint64_t)(int64_t)extra; break;
    case COMEX_SWAP: { int v; memcpy(&v, ploc, 4); bytes = 4; swap = 1; val = (uint64_t)(uint32_t)v; break; }
    case COMEX_SWAP_LONG: { int64_t v; memcpy(&v, ploc, 8); bytes = 8; swap = 1; val = (uint64_t)v; break; }
    default: fatal("comex_rmw: unknown op %d", op);
    }
    if (!ploc || !prem) fatal("comex_rmw: NULL ploc or prem");
    uint64_t old = 0;
    if (world == r.rank) {
        fence_self_if_pending();
        old = rmw_local(swap, prem, bytes, val);
    } else if (!r.same_node(world)) {
        check_remote(world, prem, 0, bytes);
        old = wire_rmw(world, swap, (uint64_t)(uintptr_t)prem, bytes, val);
    } else {
        check_remote(world, prem, 0, bytes);
        // behind our earlier traffic to that rank: pending accumulate chunks posted
        // first (the owner applies its inbox in order), direct put/get kernels done
        drain_target(world);
        if (!r.direct_pending.empty() && r.direct_pending[world]) {
            std::lock_guard<std::mutex> g(r.launch_mu);
            sched_sync_all();
        }
        RmwReply &rp = r.shm->rmw[r.li(r.rank)];
        const uint64_t seq0 = rp.seq.load(std::memory_order_acquire);
        post_request_rmw(world, swap, (uint64_t)(uintptr_t)prem, bytes, val);
        ++r.posted[world];
        for (unsigned spins = 0; rp.seq.load(std::memory_order_acquire) == seq0; ++spins)
            if (spins > 256) sched_yield();
        old = rp.value;
    }
    if (bytes == 4) {
        const uint32_t o = (uint32_t)old;
        memcpy(ploc, &o, 4);
    } else {
        memcpy(ploc, &old, 8);
    }
    return COMEX_SUCCESS;
}

// ---- mutexes (comex.h:607-643) ----
int comex_create_mutexes(int num) {
    ensure_init();
    Runtime &r = rt();
    if (num < 0 || num > kMaxMutexes) fatal("comex_create_mutexes(%d): 0..%d per rank", num, kMaxMutexes);
    if (!g_mutex_count.empty()) fatal("comex_create_mutexes: mutexes exist (comex_destroy_mutexes first)");
    std::atomic<uint32_t> *w = mutex_words(r.shm, r.node_size, r.li(r.rank));
    for (int i = 0; i < num; ++i) w[i].store(0, std::memory_order_relaxed);
    g_mutex_count.assign(r.size, 0);
    boot_allgather(&num, g_mutex_count.data(), sizeof(int));   // exchange of mutex counts
    comex_barrier(COMEX_GROUP_WORLD);
    return COMEX_SUCCESS;
}

int comex_destroy_mutexes() {
    ensure_init();
    if (g_mutex_count.empty()) fatal("comex_destroy_mutexes without comex_create_mutexes");
    comex_barrier(COMEX_GROUP_WORLD);   // no lock request outstanding
    g_mutex_count.clear();
    return COMEX_SUCCESS;
}

int comex_lock(int mutex, int proc) {
    ensure_init();
    Runtime &r = rt();
    const int world = translate_world(COMEX_GROUP_WORLD, proc);
    check_mutex(mutex, world);
    for (unsigned spins = 0;; ++spins) {
        if (r.same_node(world) ? mutex_try_local(world, mutex) : wire_lock(world, mutex, true)) break;
        progress_jobs();
        if (spins > 64) usleep(spins > 4096 ? 200 : 10);
        else sched_yield();
    }
    return COMEX_SUCCESS;
}

int comex_unlock(int mutex, int proc) {
    ensure_init();
    Runtime &r = rt();
    const int world = translate_world(COMEX_GROUP_WORLD, proc);
    check_mutex(mutex, world);
    // the reference's OP_UNLOCK reaches the owner after this rank's earlier messages
    // to it, so the critical section's operations land first: complete them here
    fence_target(world);
    {
        std::lock_guard<std::mutex> g(r.launch_mu);
        sched_sync_all();
    }
    if (r.same_node(world)) mutex_release_local(world, mutex);
    else (void)wire_lock(world, mutex, false);
    return COMEX_SUCCESS;
}

// ---- groups (comex.h:147-172) ----
int comex_group_translate_ranks(int n, comex_group_t group_from, int *ranks_from, comex_group_t group_to,
                                int *ranks_to) {
    ensure_init();
    for (int i = 0; i < n; ++i) {
        const int w = translate_world(group_from, ranks_from[i]);
        int out = -32766;   // MPI_UNDEFINED (MPI_Group_translate_ranks, which the reference calls)
        if (group_to == COMEX_GROUP_WORLD) {
            out = w;
        } else {
            int sz = 0;
            comex_group_size(group_to, &sz);
            for (int k = 0; k < sz; ++k)
                if (translate_world(group_to, k) == w) { out = k; break; }
        }
        ranks_to[i] = out;
    }
    return COMEX_SUCCESS;
}

// comex_group_comm / comex_init_comm: mpi_bridge.cpp

int gaamd_owner_counts(unsigned long long counts[4]) {
    for (int k = 0; k < 4; ++k) counts[k] = g_owned[k].load(std::memory_order_relaxed);
    return 0;
}

int gaamd_peers_unmapped(void) {
    Runtime &r = rt();
    if (!r.initialized) return -1;
    int n = 0;
    for (int q = 0; q < r.size && q < (int)r.peer_staging.size(); ++q)
        if (q != r.rank && r.same_node(q) && !r.peer_staging[q]) ++n;
    return n;
}

int gaamd_stamps(int on, unsigned long long out[8]) {
    if (out)
        for (int k = 0; k < 8; ++k) out[k] = g_stamp[k];
    if (on >= 0) {
        if (on) memset(g_stamp, 0, sizeof(g_stamp));
        g_stamp_on.store(on != 0, std::memory_order_relaxed);
    }
    return 0;
}

int gaamd_iov_path_counts(unsigned long long counts[3]) {
    for (int k = 0; k < 3; ++k) counts[k] = g_iov_path[k].load(std::memory_order_relaxed);
    return 0;
}

int gaamd_toggle_counts(unsigned long long counts[3]) {
    for (int k = 0; k < 3; ++k) counts[k] = g_toggle[k].load(std::memory_order_relaxed);
    return 0;
}

int gaamd_route_counts(unsigned long long counts[4]) {
    for (int k = 0; k < 4; ++k) counts[k] = g_route[k].load(std::memory_order_relaxed);
    return 0;
}

unsigned long long gaamd_one_pass_count(void) { return g_one_pass.load(std::memory_order_relaxed); }

}  // extern "C"

namespace gaamd {
void segment_cache_flush() { block_flush(); }
}  // namespace gaamd
