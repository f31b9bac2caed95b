// onepass.cpp -- the one-pass route between ranks that share one GPU.
//
// The reference's SMP route maps the target's shared memory and runs _acc into it
// under the target's semaphore (comex.c:6241-6260).  Here a same-node accumulate
// into a rank on THIS GPU is one fused kernel of the requester, writing the
// owner's segment through its IPC mapping (same physical HBM) under the owner's
// memory lock in node shared memory (NodeShm::mem_lock / mem_want).  DESIGN.md §6
// "One-pass lock protocol" states the protocol and why it cannot deadlock.
#include "comex_impl.hpp"
#include <chrono>
#include <mutex>
#include <sched.h>
#include <stdlib.h>
#include <string.h>

namespace gaamd {

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

// Caller holds launch_mu (sched_pick).  While a requester holds the lock this
// waits WITHOUT launch_mu: a thread holding launch_mu never waits for a memory
// lock, so lock holders (which need their own launch_mu to launch) always get it
// -- a requester holds one lock and waits only for its launch_mu and its kernel,
// the owner's release needs only its launch_mu: no cycle (with launch_mu held
// across the wait, eight ranks accumulating into each other could close one:
// rank A's progress thread holding A's launch_mu waiting for A's lock held by C,
// C waiting for its launch_mu held by its progress thread waiting for C's lock...).
bool one_pass_reap_try();

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
bool own_release_if_wanted() {
    Runtime &r = rt();
    if (!r.one_pass || !r.shm->mem_want[r.li(r.rank)].load(std::memory_order_acquire)) return false;
    std::lock_guard<std::mutex> g(r.launch_mu);
    if (!r.own_holds) return false;
    sched_sync_all();   // every write of ours into our segments has finished
    r.own_holds = false;
    r.shm->mem_lock[r.li(r.rank)].store(0, std::memory_order_release);
    return true;
}

std::atomic<unsigned long long> g_one_pass{0};   // gaamd_route_counts: one-pass accumulates issued

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
// took it (400 us): requesters streaming accumulates into one
// owner then hand the lock over once per lease instead of once per call, each
// hand-over costing a completion wait and a dispatch (tens of us against a few us
// of enqueue per call); the wait a requester sees stays bounded by the lease.
// Every rank but one accumulating into that one (tools/remote_sweep.py --all-to-one,
// profiles/r03/s26): 3 ranks 37 us per call per requester without a lease, 17.5-19.7
// with 100 us, 16.2-17.6 with 400 us; 5 ranks 77-82 / 36-58 / 36-40.
static double one_pass_lease_s() { return 400e-6; }
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

bool one_pass_reap(bool wait) {
    std::lock_guard<std::mutex> g(g_op_mu);
    return one_pass_reap_locked(wait);
}

// from a memory-lock wait loop: reap what others want unless another thread of this
// process is in the bookkeeping (it reaps then, or it is the one-pass launch that
// holds g_op_mu only across a launch and an event wait)
bool one_pass_reap_try() {
    std::unique_lock<std::mutex> g(g_op_mu, std::try_to_lock);
    if (!g.owns_lock()) return false;
    return one_pass_reap_locked(false);
}

// Mark our launches into t's segment, wait for them WITHOUT g_op_mu (the
// progress thread reaps under it and must not stall behind a long kernel), then
// release t's lock unless another thread of ours released it meanwhile.  `og`
// holds g_op_mu on entry and on return.
static void one_pass_finish_locked(std::unique_lock<std::mutex> &og, int t) {
    OnePassHold &h = g_op_hold[t];
    one_pass_mark(h);
    const std::vector<hipEvent_t> evs = h.evs;
    og.unlock();
    for (hipEvent_t e : evs) GA_HIP(hipEventSynchronize(e));
    og.lock();
    if (h.held && h.evs == evs) one_pass_release(t, h);
}

// true: launched (blocking: complete on return; else `hdl` tracks it);
// false: not eligible (the caller takes another route)
bool one_pass_acc(int t, int op, void *scale, void *src, const int *ss, void *dst, const int *ds,
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
    // HBM segments only: a host segment's owner keeps no memory lock (own_write_guard
    // covers its HBM segments), so accumulates into it go through the owner
    if (segment_kind_of(t, (const char *)dst + dlo) != 1) return false;
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
        one_pass_finish_locked(og, t);
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
        one_pass_finish_locked(og, t);
        og.unlock();
    }
    return true;
}


void one_pass_finalize() {
    std::lock_guard<std::mutex> g(g_op_mu);   // the locks were handed back by comex_barrier's fence
    for (OnePassHold &h : g_op_hold)
        for (hipEvent_t e : h.evs) (void)hipEventDestroy(e);
    g_op_hold.clear();
    for (hipEvent_t e : g_op_pool) (void)hipEventDestroy(e);
    g_op_pool.clear();
}

}  // namespace gaamd
