// remote.cpp -- operations applied by the owner: the staging ring, the owner's
// inbox, its progress thread, and the asynchronous remote-accumulate jobs.
//
// Reference: the MPI-PR progress rank (_progress_server, comex.c:3379-3565) and its
// handlers (_acc_packed_handler 4133-4281, _acc_iov_handler 4284-4397,
// _put_packed_handler 3605-3677, OP_GET 6188-6214, OP_FETCH_AND_ADD / OP_SWAP),
// fed by nb_accs_packed (6965-7109).  Here every rank exports one staging buffer
// (HBM) cut into a FIFO sub-ring per target; a requester packs into it and posts a
// Request into the owner's 256-slot inbox in node shared memory; the owner's
// progress thread applies requests in ticket order on its own streams (a pull
// stream per source GPU) and counts them done[src][owner].
#include "comex_impl.hpp"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <sched.h>
#include <time.h>
#include <algorithm>
#include <deque>
#include <mutex>
#include <thread>

namespace gaamd {

// Events the owner's progress thread records behind the kernels it applies (their
// completion bumps done[src][owner], or frees a staging slice): a system-scope
// release, stated rather than left to HIP's default, so what the owner wrote is
// visible to a requester on another GPU that reads it after its fence (§6)
constexpr unsigned kOwnerEventFlags = hipEventDisableTiming | hipEventReleaseToSystem;

static const char *peer_staging_or_die(int src) {
    const char *p = rt().peer_staging[src];
    if (!p) fatal("rank %d's staging buffer is not mapped here (IPC open failed at comex_init)", src);
    return p;
}

// ---- staging ring + owner inbox ----------------------------------------------
std::vector<std::deque<Pending>> g_pend;   // per target

uint64_t sub_ring_bytes() {
    Runtime &r = rt();
    return (r.staging_bytes / (size_t)r.size) & ~(size_t)255;
}

static void reap(int t) {
    Runtime &r = rt();
    const uint64_t done = r.shm->done[r.li(r.rank)][r.li(t)].load(std::memory_order_acquire);
    while (!g_pend[t].empty() && g_pend[t].front().seq <= done) g_pend[t].pop_front();
}

void wait_done(int t, uint64_t seq) {
    Runtime &r = rt();
    for (unsigned spins = 0; r.shm->done[r.li(r.rank)][r.li(t)].load(std::memory_order_acquire) < seq; ++spins)
        if (spins > 256) sched_yield();
    reap(t);
}

// reserve `len` bytes in the staging sub-ring for target t (FIFO release)
uint64_t stage_alloc(int t, uint64_t len) {
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

std::atomic<unsigned long long> g_route[4];   // gaamd_route_counts
std::atomic<unsigned long long> g_owned[4];   // gaamd_owner_counts: requests applied, by kind

// Reserve rank t's next inbox slot (ticket order) and claim it for writing: the
// slot belongs to our lap once the previous lap's ticket is consumed.  The caller
// fills the request and publishes it (publish: state 2, release).
static Request &inbox_claim(int t) {
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
    // every field a kind does not use reads zero
    q.src_rank = r.rank;
    q.op = 0;
    q.levels = 0;
    memset(q.count, 0, sizeof(q.count));
    memset(q.dst_stride, 0, sizeof(q.dst_stride));
    memset(q.src_stride, 0, sizeof(q.src_stride));
    q.dst_addr = q.src_addr = q.staging_off = q.bytes = q.seq = q.iov_align = q.dst_hi = 0;
    memset(q.scale, 0, sizeof(q.scale));
    q.iov_serial = 0;
    return q;
}

static void publish(Request &q, int kind) {
    q.kind = kind;
    q.state.store(2, std::memory_order_release);
}

static void set_scale(Request &q, int op, const void *scale) {
    q.op = op;
    if (scale) memcpy(q.scale, scale, (size_t)elem_size(op));
}

// kind 0: a packed strided chunk, rows rb..re of the patch at `off` of our staging
static void post_request(int t, int op, const void *scale, uint64_t dst_addr, const int *dst_stride,
                         const int *count, int levels, uint64_t off, uint64_t len, uint64_t rb, uint64_t re) {
    Request &q = inbox_claim(t);
    set_scale(q, op, scale);
    q.levels = levels;
    for (int j = 0; j <= levels; ++j) q.count[j] = count[j];
    for (int j = 0; j < levels; ++j) q.dst_stride[j] = dst_stride[j];
    q.dst_addr = dst_addr;
    q.staging_off = off;
    q.bytes = len;
    q.seq = (rb << 32) | (re & 0xffffffffull);   // row range travels in seq
    g_route[0].fetch_add(1, std::memory_order_relaxed);
    publish(q, 0);
}

// kind 1: io-vector; staging holds n packed source runs, then the n owner
// addresses (8-byte aligned); mode: 0 parallel, 1 in order on one lane
// (destinations overlap), 2 GPU-sorted runs
void post_request_iov(int t, int op, const void *scale, int bytes, int n, uint64_t off, uint64_t len, uint64_t dlo,
                      uint64_t dhi, uint64_t align_or, int mode) {
    Request &q = inbox_claim(t);
    set_scale(q, op, scale);
    q.count[0] = bytes;
    q.count[1] = n;
    q.dst_addr = dlo;
    q.dst_hi = dhi;
    q.staging_off = off;
    q.bytes = len;
    q.iov_serial = mode;
    q.iov_align = align_or;
    g_route[2].fetch_add(1, std::memory_order_relaxed);
    publish(q, 1);
}

// kind 3: the owner reads the source patch from this rank's segment directly
void post_request_direct(int t, int op, const void *scale, uint64_t dst_addr, const int *dst_stride,
                         uint64_t src_addr, const int *src_stride, const int *count, int levels) {
    Request &q = inbox_claim(t);
    set_scale(q, op, scale);
    q.levels = levels;
    for (int j = 0; j <= levels; ++j) q.count[j] = count[j];
    for (int j = 0; j < levels; ++j) {
        q.dst_stride[j] = dst_stride[j];
        q.src_stride[j] = src_stride[j];
    }
    q.dst_addr = dst_addr;
    q.src_addr = src_addr;
    g_route[1].fetch_add(1, std::memory_order_relaxed);
    publish(q, 3);
}

// kind 4: a get through the owner (COMEX_ENABLE_GET_SELF/SMP=0): the owner packs
// rows rb..re of its patch into our staging at `off` (nb_get's OP_GET message to the
// progress rank, comex.c:6188-6214)
void post_request_get(int t, uint64_t src_addr, const int *src_stride, const int *count, int levels, uint64_t off,
                      uint64_t len, uint64_t rb, uint64_t re) {
    Request &q = inbox_claim(t);
    q.op = kOpCopy;
    q.levels = levels;
    for (int j = 0; j <= levels; ++j) q.count[j] = count[j];
    for (int j = 0; j < levels; ++j) q.src_stride[j] = src_stride[j];
    q.src_addr = src_addr;
    q.staging_off = off;
    q.bytes = len;
    q.seq = (rb << 32) | (re & 0xffffffffull);
    publish(q, 4);
}

// kind 2: comex_rmw on a rank of this node (the progress rank's OP_FETCH_AND_ADD /
// OP_SWAP, comex.c:2120-2200): applied after every earlier request from us
void post_request_rmw(int t, int swap, uint64_t addr, int bytes, uint64_t val) {
    Request &q = inbox_claim(t);
    q.op = swap;
    q.dst_addr = addr;
    q.bytes = (uint64_t)bytes;
    memcpy(q.scale, &val, 8);
    g_route[3].fetch_add(1, std::memory_order_relaxed);
    publish(q, 2);
}

// owner side: drain the inbox in ticket order
static std::atomic<bool> g_progress_exited{false};
std::atomic<long long> g_diag_drop_chunk{0};
static std::atomic<unsigned long long> g_drop_seen{0};

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
    // requesters' staging and fences -- and for 2 ms after the last request, then
    // backs off to short sleeps (+6.5 % on the packed route to self, +20 % on the
    // 2-rank exchange against sleeping once idle, profiles/r02/session_l)
    constexpr double spin_s = 2000e-6;
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
        if (!x.ev) GA_HIP(hipEventCreateWithFlags(&x.ev, kOwnerEventFlags));
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
            if (pool.empty()) GA_HIP(hipEventCreateWithFlags(&ev, kOwnerEventFlags));
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
                int rc = 1;
                const uint64_t units = (q.dst_hi - q.dst_addr) / (uint64_t)d.bytes + 1;
                if (q.iov_serial == 2 && d.n < kIovLdsRoute && tuning().iov_lds)
                    // below 1 Ki pairs: ordered and applied by one workgroup, in LDS
                    rc = launch_iov_lds(q.op, q.scale, d, q.iov_align, q.dst_addr, units, r.streams[si]);
                if (q.iov_serial == 2 && rc == 1) {
                    // repeated destinations ordered on the GPU: up to kIovPartWindowMax pairs
                    // by hash partitions in LDS, above by the radix path; the progress thread's
                    // own scratch, free once its previous apply has finished (which also
                    // orders the partition counters, zero at rest, between its calls)
                    const bool part = d.n <= kIovPartWindowMax && tuning().iov_lds;
                    const size_t need = std::max(iov_runs_work_bytes(d.n), part ? iov_lds_scratch_bytes(d.n) : 0);
                    if (prog_work_ev) GA_HIP(hipEventSynchronize(prog_work_ev));
                    if (need > prog_work_bytes) {
                        if (prog_work) GA_HIP(hipFree(prog_work));
                        prog_work_bytes = std::max<size_t>(need, 1 << 20);
                        GA_HIP(hipMalloc((void **)&prog_work, prog_work_bytes));
                    }
                    if (!prog_work_ev) GA_HIP(hipEventCreateWithFlags(&prog_work_ev, kOwnerEventFlags));
                    if (part)
                        rc = launch_iov_lds(q.op, q.scale, d, q.iov_align, q.dst_addr, units, r.streams[si], false,
                                            prog_work);
                    if (rc == 1)
                        rc = launch_iov_runs(q.op, q.scale, d, q.iov_align, q.dst_addr, units, prog_work,
                                             prog_work_bytes, r.streams[si]);
                    GA_HIP(hipEventRecord(prog_work_ev, r.streams[si]));
                } else if (rc == 1) {
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
            if (pool.empty()) GA_HIP(hipEventCreateWithFlags(&ev, kOwnerEventFlags));
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
            if (pool.empty()) GA_HIP(hipEventCreateWithFlags(&ev, kOwnerEventFlags));
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
            if (pool.empty()) GA_HIP(hipEventCreateWithFlags(&ev, kOwnerEventFlags));
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
            // test hook (gaamd_diag "drop_chunk" N): every N-th packed chunk is counted
            // applied without its kernel -- a logic fault no publication mode can mend
            const long long dn = g_diag_drop_chunk.load(std::memory_order_relaxed);
            const bool drop = dn > 0 && (g_drop_seen.fetch_add(1, std::memory_order_relaxed) + 1) % dn == 0;
            if (drop)
                fprintf(stderr, "[ga_amd %d] gaamd_diag drop_chunk: rows %llu..%llu of a chunk from rank %d dropped\n",
                        r.rank, (unsigned long long)rb, (unsigned long long)re, src);
            hipEvent_t ev;
            if (pool.empty()) GA_HIP(hipEventCreateWithFlags(&ev, kOwnerEventFlags));
            else { ev = pool.back(); pool.pop_back(); }
            {
                std::lock_guard<std::mutex> g(r.launch_mu);
                const bool peer = r.peer_src(src);
                int64_t dlo = 0, dhi = 0;
                side_span_host(q.dst_stride, q.count, q.levels, q.count[0], &dlo, &dhi);
                const int si = sched_pick(span_of(packed, 0, (int64_t)q.bytes), span_of((void *)q.dst_addr, dlo, dhi),
                                          0, peer ? pull_stream(src) : -1);
                int rc = drop ? 0 : launch_strided(q.op, q.scale, packed0, pstride, (void *)q.dst_addr, q.dst_stride,
                                                   q.count, q.levels, r.streams[si], nullptr, rb, re, false, peer);
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
        // our one-pass kernels into peers' segments (never blocking: a user thread may
        // be waiting for a long kernel under the bookkeeping lock)
        if (one_pass_reap_try()) worked = true;
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
    g_progress_exited.store(true, std::memory_order_release);
}

// a process leaving without comex_finalize (exit_without_finalize, comex.cpp): stop the
// progress thread if it is idle within `wait_s` and join it, so it is not inside a HIP
// call while the runtime tears down; otherwise leave it detached
void progress_stop_at_exit(double wait_s) {
    Runtime &r = rt();
    if (!r.progress.joinable()) return;
    r.stop.store(true, std::memory_order_release);
    auto now_s = [] {
        timespec ts;
        clock_gettime(CLOCK_MONOTONIC, &ts);
        return ts.tv_sec + 1e-9 * ts.tv_nsec;
    };
    const double t0 = now_s();
    while (!g_progress_exited.load(std::memory_order_acquire) && now_s() - t0 < wait_s) sched_yield();
    if (g_progress_exited.load(std::memory_order_acquire)) r.progress.join();
    else r.progress.detach();
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
bool progress_jobs() {
    Runtime &r = rt();
    if (g_jobs.empty()) return false;
    const uint64_t sub = sub_ring_bytes();
    bool any = false;
    // post chunks whose pack finished, per target in allocation order
    bool published = false;
    for (int t = 0; t < (int)g_out.size(); ++t) {
        std::deque<Chunk> &o = g_out[t];
        while (!o.empty()) {
            Chunk &c = o.front();
            const hipError_t e = hipEventQuery(c.ev);
            if (e == hipErrorNotReady) break;
            if (e != hipSuccess) fatal("pack kernel failed: %s", hipGetErrorString(e));
            if (!published && g_publish_conservative.load(std::memory_order_relaxed)) {
                // the conservative publication mode: a system-scope release on every
                // library stream, drained, before the first post of this pass
                std::lock_guard<std::mutex> g(r.launch_mu);
                sched_publish_all();
                published = true;
            }
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
            // the chunk's publication: the owner (possibly on another GPU) reads this
            // slice of our staging with system-scope loads once the request is posted,
            // and the request is posted only after this event completed -- recorded
            // with a system-scope release (hipEventReleaseToSystem, stated rather than
            // left to the default), so the pack kernel's stores are written back past
            // every cache of this GPU before the post
            if (g_chunk_ev.empty())
                GA_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventReleaseToSystem));
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

void run_job(int id) {
    for (unsigned spins = 0; find_job(id); backoff(spins))
        if (progress_jobs()) spins = 0;
}

bool target_busy(int t) {
    for (const RJob &j : g_jobs) if (j.t == t) return true;
    return false;
}

void drain_target(int t) {
    for (unsigned spins = 0; target_busy(t); backoff(spins))
        if (progress_jobs()) spins = 0;
}

void drain_all_jobs() {
    for (unsigned spins = 0; !g_jobs.empty(); backoff(spins))
        if (progress_jobs()) spins = 0;
}

// start a remote accumulate; returns its job id (0: nothing to do)
// Are the rows of one side pairwise byte-disjoint?  Sufficient test: with the
// levels sorted by |stride|, each stride covers the whole extent below it.
bool dst_rows_disjoint(const int *str, const int *count, int levels, int64_t row_bytes) {
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

int remote_acc_start(int t, int op, const void *scale, void *src, const int *ss, void *dst, const int *ds,
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
    // a small pageable source goes through the thread's pinned bounce buffer: such a job
    // completes before the call returns (host_src below), so the buffer is free again
    j.sv = local_view(src, j.slo, j.shi, false, true);
    j.staged_src = j.sv.staged != nullptr;
    if (j.staged_src) {
        std::lock_guard<std::mutex> g(r.launch_mu);
        sched_join();
    }
    const uint64_t sub = sub_ring_bytes();
    if ((uint64_t)row_bytes > sub) fatal("row of %ld bytes exceeds staging ring", (long)row_bytes);
    // One chunk per sub-ring for every target.  Cutting the ring into slices for an
    // owner on another GPU (packing chunk k+1 while it pulls chunk k) measured only
    // slower on the one-GPU proxy (2-rank C3 exchange, profiles/r03/s38: 2950-3140
    // GiB/s with one slice, 2922-2941 with 2, 2607-2637 with 4), so it went.
    j.per_req = std::max<uint64_t>(1, sub / (uint64_t)row_bytes);
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
    const bool host_src = j.sv.registered || j.sv.staged || j.sv.bounce;
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

void fence_target(int t) {
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
void fence_self_if_pending() {
    Runtime &r = rt();
    if (r.posted.empty()) return;
    if (target_busy(r.rank) ||
        r.shm->done[r.li(r.rank)][r.li(r.rank)].load(std::memory_order_acquire) < r.posted[r.rank])
        fence_target(r.rank);
}


// ---- setup / teardown (collective) -------------------------------------------
// The staging HBM for remote operations, exported to every local rank, each
// mapping checked against the tag its owner wrote (as segments are, do_malloc),
// and the progress thread.
void remote_init() {
    Runtime &r = rt();
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
    for (int q = 0; q < r.size; ++q) handle_seen(q, 0, 0, all[q].bytes, all[q].h);   // allocation 0: staging
    for (int q = 0; q < r.size; ++q) {
        if (q == r.rank) { r.peer_staging[q] = r.staging; continue; }
        if (!r.same_node(q)) continue;   // another node: reached through wire.cpp
        r.peer_staging[q] = (char *)ipc_open(all[q].h, q, "staging buffer");
    }
    // every staging mapping must read its owner's tag (written before the exchange,
    // below the allgather's barrier) -- a mapping of the wrong allocation would hand
    // the owners other bytes to accumulate
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
}

// after comex_barrier (every job drained): the progress thread stopped, the peers'
// staging mappings closed, and -- after a barrier -- our staging freed
void remote_finalize() {
    Runtime &r = rt();
    for (hipEvent_t e : g_chunk_ev) (void)hipEventDestroy(e);
    g_chunk_ev.clear();
    g_out.clear();
    if (r.progress.joinable()) {
        r.stop.store(true, std::memory_order_release);
        r.progress.join();
    }
}

void remote_release_staging() {
    Runtime &r = rt();
    for (int q = 0; q < (int)r.peer_staging.size(); ++q)
        if (q != r.rank && r.peer_staging[q]) ipc_close(r.peer_staging[q], q);
    r.peer_staging.clear();
}

void remote_free_staging() {
    Runtime &r = rt();
    if (r.staging) addr_event('f', r.staging, r.staging_bytes, -1);
    if (r.staging) (void)hipFree(r.staging);
    r.staging = nullptr;
}

bool job_pending(int id) { return find_job(id) != nullptr; }

}  // namespace gaamd
