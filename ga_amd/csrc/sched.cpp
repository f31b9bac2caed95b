// sched.cpp -- dependency-aware assignment of operations to HIP streams.
//
// The reference executes every accumulate synchronously under the target's
// semaphore (comex/src-mpi-pr/comex.c:6228-6260), so two accumulates never
// overlap.  On the GPU a single in-order stream gives the same exclusivity but
// leaves each kernel's ramp-up and tail (≈1.5 µs of a 33 µs launch at the
// headline size) with idle CUs.  Operations whose byte ranges are independent
// (no write of one overlaps a read or write of the other) commute, so they may
// run on different streams and overlap those edges; dependent ones are ordered
// on one stream, with cross-stream event waits where a dependency spans two.
//
//   * history: the ranges (device views) of the ops enqueued since the last
//     join, with their stream; capped at kHist entries, then a join (or, when
//     every entry sits on one stream, dropped with a one-time wait per stream).
//   * join: every stream waits for every other's enqueued work (events), so
//     history can be forgotten.
//   * sync_all: host waits for all streams (fences, barriers, waits).
//   * completion marks: a non-blocking handle is (stream, sequence number of
//     the op on that stream); an event is recorded only every kMarkEvery
//     tracked ops of a stream, or when a wait/test needs one.  A later event
//     on the same in-order stream covers every earlier op, so a wait may wait a
//     little longer than its op, never shorter.  (An event per op put a marker
//     packet between every two kernels: +1.7 us per 33 us launch measured on
//     MI355X, profiles/r02/.)
// Callers hold Runtime::launch_mu around pick + launch.  The completion marks
// have their own lock (g_marks_mu): sched_track / sched_complete run outside
// launch_mu, and a wait on an event is done with the lock released.
#include <atomic>
#include "runtime.hpp"
#include "gaamd_kernels.h"
#include <string.h>
#include <stdlib.h>
#include <deque>
#include <algorithm>

namespace gaamd {

namespace {
constexpr int kHist = 64;
struct Entry {
    int stream;
    Span src, dst;
};
std::vector<Entry> g_hist;
std::vector<hipEvent_t> g_ev;   // one reusable event per stream for cross waits
int g_rr = 0;
// history dropped while every entry sat on one stream: the ops behind it are
// ordered on g_base; a stream not yet in g_base_waited waits for g_base before
// its first new op (cheaper than a full join for runs of one-stream work)
int g_base = -1;
unsigned g_base_waited = 0;

inline bool overlap(const Span &a, const Span &b) { return a.lo < b.hi && b.lo < a.hi && a.lo < a.hi && b.lo < b.hi; }

constexpr uint64_t kMarkEvery = 16;
struct Mark {
    uint64_t seq;
    hipEvent_t ev;
};
struct Marks {
    uint64_t issued = 0, done = 0, marked = 0;   // tracked ops enqueued / known complete / covered by an event
    std::deque<Mark> q;
};
std::vector<Marks> g_marks;
std::vector<hipEvent_t> g_mark_pool;
std::mutex g_marks_mu;   // g_marks, g_mark_pool

void marks_reset_done() {   // caller holds g_marks_mu
    for (Marks &m : g_marks) {
        m.done = m.marked = m.issued;
        for (const Mark &k : m.q) g_mark_pool.push_back(k.ev);
        m.q.clear();
    }
}

void mark_now(int s) {   // caller holds g_marks_mu
    Marks &m = g_marks[s];
    if (m.marked == m.issued) return;
    hipEvent_t e;
    if (g_mark_pool.empty()) GA_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    else { e = g_mark_pool.back(); g_mark_pool.pop_back(); }
    GA_HIP(hipEventRecord(e, rt().streams[s]));
    m.q.push_back({m.issued, e});
    m.marked = m.issued;
}
}  // namespace

uint64_t sched_track(int s) {
    std::lock_guard<std::mutex> g(g_marks_mu);
    if (s < 0 || s >= (int)g_marks.size()) return 0;
    Marks &m = g_marks[s];
    const uint64_t seq = ++m.issued;
    if (seq - m.marked >= kMarkEvery) mark_now(s);
    return seq;
}

bool sched_complete(int s, uint64_t seq, bool wait) {
    std::unique_lock<std::mutex> g(g_marks_mu);
    if (seq == 0 || s < 0 || s >= (int)g_marks.size()) return true;
    Marks &m = g_marks[s];
    if (seq <= m.done) return true;
    if (m.marked < seq) mark_now(s);   // no event covers it yet
    while (!m.q.empty()) {
        const Mark k = m.q.front();
        hipError_t e = hipEventQuery(k.ev);
        if (e == hipErrorNotReady && wait) {
            // wait without the lock; the event is not recycled meanwhile (it stays
            // in the queue until someone sees it complete, under the lock)
            g.unlock();
            e = hipEventSynchronize(k.ev);
            g.lock();
            if (m.q.empty() || m.q.front().ev != k.ev) {   // another thread retired it
                if (m.done >= seq) return true;
                continue;
            }
        }
        if (e == hipErrorNotReady) return false;
        if (e != hipSuccess) fatal("operation failed: %s", hipGetErrorString(e));
        m.done = k.seq;
        g_mark_pool.push_back(k.ev);
        m.q.pop_front();
        if (m.done >= seq) return true;
    }
    return m.done >= seq;
}

static std::atomic<uint64_t> g_epoch{0};
uint64_t sched_epoch() { return g_epoch.load(std::memory_order_relaxed); }

void sched_init(int n, int pull) {
    Runtime &r = rt();
    g_epoch.fetch_add(1, std::memory_order_relaxed);
    if (n < 1) n = 1;
    if (n > 8) n = 8;
    if (pull < 0) pull = 0;
    if (pull > 8) pull = 8;
    r.user_streams = n;
    n += pull;
    r.streams.assign(1, r.stream);
    for (int i = 1; i < n; ++i) {
        hipStream_t s;
        GA_HIP(hipStreamCreateWithFlags(&s, hipStreamDefault));
        r.streams.push_back(s);
    }
    g_ev.assign(n, nullptr);
    for (int i = 0; i < n; ++i) GA_HIP(hipEventCreateWithFlags(&g_ev[i], hipEventDisableTiming));
    std::lock_guard<std::mutex> g(g_marks_mu);
    g_marks.assign(n, Marks());
    g_hist.clear();
    g_rr = 0;
    g_base = -1;
    sched_flag_init();
}

// change the number of library streams at run time (all work drained first)
void sched_resize(int n) {
    Runtime &r = rt();
    const int pull = (int)r.streams.size() - r.user_streams;
    sched_sync_all();
    sched_fini();
    r.streams.clear();
    sched_init(n, pull);
}

static std::vector<hipEvent_t> g_pub_ev;   // sched_publish_all
std::atomic<bool> g_publish_conservative{false};

void sched_fini() {
    Runtime &r = rt();
    for (hipEvent_t e : g_pub_ev) (void)hipEventDestroy(e);
    g_pub_ev.clear();
    for (size_t i = 1; i < r.streams.size(); ++i) (void)hipStreamDestroy(r.streams[i]);
    for (hipEvent_t e : g_ev) (void)hipEventDestroy(e);
    g_ev.clear();
    std::lock_guard<std::mutex> g(g_marks_mu);
    marks_reset_done();
    for (hipEvent_t e : g_mark_pool) (void)hipEventDestroy(e);
    g_mark_pool.clear();
    g_marks.clear();
    r.streams.clear();
    g_hist.clear();
}

static void wait_on(int waiter, int producer) {
    Runtime &r = rt();
    GA_HIP(hipEventRecord(g_ev[producer], r.streams[producer]));
    GA_HIP(hipStreamWaitEvent(r.streams[waiter], g_ev[producer], 0));
}

void sched_join() {
    Runtime &r = rt();
    const int n = (int)r.streams.size();
    if (n > 1) {
        for (int x = 1; x < n; ++x) wait_on(0, x);   // stream 0 after everything
        for (int x = 1; x < n; ++x) wait_on(x, 0);   // everything after stream 0
    }
    g_hist.clear();
    g_base = -1;
}

// A join before a launch on stream 0 that writes `dst` (host-side operands,
// staged copies, wire unpacks): like sched_pick, it first takes this rank's
// memory lock when dst may be one of its segments -- a same-GPU peer's one-pass
// kernel may otherwise be writing the same bytes.
void sched_join_write(const Span &dst) {
    own_write_guard(dst);
    sched_join();
}

void sched_sync_all() {
    Runtime &r = rt();
    // (polling hipStreamQuery instead measured the same ≈13 µs acc + fence
    // latency: the floor is the GPU's launch-to-completion, not the host wake-up)
    for (hipStream_t s : r.streams) GA_HIP(hipStreamSynchronize(s));
    for (uint8_t &p : r.direct_pending) p = 0;   // every put/get kernel has finished
    {
        std::lock_guard<std::mutex> g(g_marks_mu);
        marks_reset_done();                       // every tracked op is complete
    }
    g_hist.clear();
    g_base = -1;
}

// The conservative publication mode (gaamd_diag "publish" 1):
// sched_sync_all behind an event recorded with hipEventReleaseToSystem on every
// library stream -- a system-scope release stated on each stream, then waited for.
// Round 5 measured it on every direct-source post and fence (-33 % on that route,
// profiles/r05/ab/) and took it out of the default path; a cross-GPU check that reads
// MISMATCH runs once more under it, to tell a visibility fault from a logic one.
void sched_publish_all() {
    Runtime &r = rt();
    while (g_pub_ev.size() < r.streams.size()) {
        hipEvent_t e;
        GA_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventReleaseToSystem));
        g_pub_ev.push_back(e);
    }
    for (size_t i = 0; i < r.streams.size(); ++i) GA_HIP(hipEventRecord(g_pub_ev[i], r.streams[i]));
    sched_sync_all();
}

// ---- blocking-call completion through a flag -----------------
// A blocking call whose operands are all device memory (HBM) completes locally when
// its kernel has finished.  hipStreamSynchronize returns some 4 us after the GPU is
// done (the runtime's completion signal and the host wake-up); a one-lane kernel
// behind it storing a sequence number into pinned host memory, which the caller
// spins on, is seen that much sooner.  Only for HBM operands: the CPU never reads
// them, so nothing but the ORDER of the GPU's work matters; a host-memory
// destination keeps hipStreamSynchronize (the runtime's system-scope release at
// the stream's end makes its bytes visible to the CPU).
namespace {
uint64_t *g_flag_host = nullptr, *g_flag_dev = nullptr;
std::vector<uint64_t> g_flag_seq;
}

// the flag page, at comex_init (sched_init) rather than inside the first blocking call
void sched_flag_init() {
    if (g_flag_host) return;
    // coherent (fine-grained) stated, not left to the runtime's default: the GPU's
    // store must reach the host's polling loads without any cache maintenance
    GA_HIP(hipHostMalloc((void **)&g_flag_host, 64 * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent));
    GA_HIP(hipHostGetDevicePointer((void **)&g_flag_dev, g_flag_host, 0));
    memset(g_flag_host, 0, 64 * sizeof(uint64_t));
    g_flag_seq.assign(64, 0);
    // one flag launch into the spare last slot, waited for: it loads the library's
    // code object (all its kernels, gaamd_all.hip) onto the GPU here, in comex_init,
    // instead of in the first operation that launches a kernel (≈ 15 ms, profiles/r05/s5)
    const int rc = launch_flag(g_flag_dev + 63, 0, rt().stream);
    if (rc) fatal("completion flag launch failed (%d)", rc);
    GA_HIP(hipStreamSynchronize(rt().stream));
}

void sched_wait_flag(int s) {
    Runtime &r = rt();
    uint64_t v;
    volatile uint64_t *f;
    {
        std::lock_guard<std::mutex> g(r.launch_mu);
        sched_flag_init();
        if (s < 0 || s >= 64) fatal("stream index %d out of range", s);
        v = ++g_flag_seq[s];
        const int rc = launch_flag(g_flag_dev + s, v, r.streams[s]);
        if (rc) fatal("completion flag launch failed (%d)", rc);
        f = g_flag_host + s;
    }
    for (unsigned long spins = 0; __atomic_load_n(f, __ATOMIC_ACQUIRE) < v; ++spins) {
        if ((spins & 0xfffff) == 0xfffff) {
            // every ~1M polls: a failed stream reports its error instead of spinning on,
            // and an idle stream ends the wait -- the flag kernel behind the call has
            // finished, so the call has, whether or not its store was seen
            const hipError_t e = hipStreamQuery(r.streams[s]);
            if (e == hipSuccess) break;
            if (e != hipErrorNotReady) fatal("stream failed: %s", hipGetErrorString(e));
        }
        __builtin_ia32_pause();
    }
}

void sched_flag_fini() {
    if (g_flag_host) (void)hipHostFree(g_flag_host);
    g_flag_host = g_flag_dev = nullptr;
    g_flag_seq.clear();
}

// Launches that move at least this many payload bytes stay on the stream of the
// previous operation even when independent: two such kernels running side by
// side lost 3 % against running them back to back (C4, 256 MiB of double
// complex per launch: profiles/r01/sweep_streams.jsonl), while the edge overlap
// they would buy is < 1 % of their length.  Smaller launches alternate.
constexpr uint64_t kBigPayload = 192ull << 20;
// Below this, launches are host-bound (≈3 µs of enqueue against a shorter
// kernel): alternating streams only added ≈1-2 µs per call up to 4 MiB and
// gained from 16 MiB on (tools/perf_strided.cpp, profiles/r01/perf_strided.jsonl).
constexpr uint64_t kSmallPayload = 8ull << 20;

int sched_pick(const Span &src, const Span &dst, uint64_t payload, int prefer) {
    Runtime &r = rt();
    own_write_guard(dst);
    const int n = (int)r.streams.size();
    if (n <= 1) return 0;
    const int nu = std::max(1, std::min(r.user_streams, n));   // round robin over the user streams
    if ((int)g_hist.size() >= kHist) {
        const int s0 = g_hist.front().stream;
        bool one = g_base < 0 || g_base == s0;
        for (const Entry &e : g_hist) one = one && e.stream == s0;
        if (one) {   // drop the history; remember the stream it is ordered on
            g_hist.clear();
            if (g_base != s0) g_base_waited = 1u << s0;
            g_base = s0;
        } else {
            sched_join();
        }
    }
    unsigned mask = 0;
    int last = -1;
    for (const Entry &e : g_hist) {
        if (overlap(dst, e.dst) || overlap(dst, e.src) || overlap(src, e.dst)) {
            mask |= 1u << e.stream;
            last = e.stream;
        }
    }
    int s;
    if (!mask) {
        if (prefer >= 0 && prefer < n) {
            s = prefer;
        } else {
            if (payload == 0 || (payload >= kSmallPayload && payload < kBigPayload)) g_rr = (g_rr + 1) % nu;
            s = g_rr % nu;
        }
    } else {
        s = last;   // the most recent dependency's stream; wait for the others
        for (int x = 0; x < n; ++x)
            if (x != s && (mask & (1u << x))) wait_on(s, x);
    }
    if (g_base >= 0 && !(g_base_waited & (1u << s))) {
        wait_on(s, g_base);
        g_base_waited |= 1u << s;
        if (g_base_waited == (1u << n) - 1) g_base = -1;
    }
    g_hist.push_back({s, src, dst});
    return s;
}

}  // namespace gaamd
