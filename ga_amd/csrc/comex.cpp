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
//   comex_malloc (2359-2605)                 -> segments.cpp
//   comex_accv/putv/getv (7327-7400)         -> iov.cpp
//   comex_fence_* (1074-1191), comex_barrier (1217-1234), comex_wait* (1776-1802).
// This file holds the C ABI, init/finalize, handles and the routing of strided
// operations; comex_impl.hpp lists what the other files of the runtime hold.
//
// Host (non-HBM) buffers are accepted everywhere: pinned memory is used in
// place (device-mapped), pageable memory is registered for the call.  All
// arithmetic runs on the GPU; there is no CPU compute path.
#include "comex_impl.hpp"
#include "../../include/ga_amd.h"
#include <hip/hip_version.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include <sched.h>
#include <deque>
#include <memory>
#include <algorithm>

#ifndef GAAMD_ROCM_PATH
#define GAAMD_ROCM_PATH "/opt/rocm"
#endif

namespace gaamd {

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

// ---- non-blocking handles ------------------------------------------------
static int g_nb_job[kMaxNb];   // nb handle -> its remote accumulate job (0: none; see progress_jobs)
// nb handle -> a direct-source request (target, its posted sequence; 0: none):
// complete once the owner has applied it (the source is read in place)
static int g_nb_rt[kMaxNb];
static uint64_t g_nb_rseq[kMaxNb];
static std::vector<uint64_t> g_direct_last;   // per target: last direct-source request posted

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
void nb_complete_now(comex_request_t *h, int stream_idx, bool on_stream) {
    Runtime &r = rt();
    const int i = nb_alloc();
    g_nb_job[i] = 0;
    g_nb_rseq[i] = 0;
    r.nb_stream[i] = stream_idx;
    r.nb_seq[i] = on_stream ? sched_track(stream_idx) : 0;
    *h = i;
}

// ---- the one transfer routine ---------------------------------------------
// smallest payload sent by the direct-source route: below it the packed route's
// asynchronous pack beats the host drain of our streams the direct route needs
constexpr uint64_t kDirectSrcMin = 1ull << 20;

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
// region edges on a kernel trace.  Off unless gaamd_diag("stamps", 1).
static std::atomic<bool> g_stamp_on{false};
std::atomic<unsigned long long> g_peer_gets{0};   // strided gets read from another GPU (system-scope loads)
static uint64_t g_stamp[8];
static inline void stamp(int i) {
    if (!g_stamp_on.load(std::memory_order_relaxed)) return;
    timespec ts;
    clock_gettime(CLOCK_BOOTTIME, &ts);
    g_stamp[i] = (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

// ---- the reference's route toggles beyond SELF/SMP --------------------------
std::atomic<unsigned long long> g_toggle[3];   // gaamd_toggle_counts: rows, pairs, owner gets

// the reference's self/SMP test (comex.c:6365-6377, 6634-6647, 6910-6913,
// 7120-7122, 7224-7226, 7336-7338): true when the self or SMP route applies to an
// operation on `world`; only otherwise are the PACKED / IOV toggles consulted
bool self_smp_route(Xfer kind, int world) {
    Runtime &r = rt();
    const bool self = kind == X_ACC ? r.acc_self_direct : (kind == X_PUT ? r.put_self_direct : r.get_self_direct);
    const bool smp = kind == X_ACC ? r.acc_smp_direct : (kind == X_PUT ? r.put_smp_direct : r.get_smp_direct);
    return world == r.rank ? self : (smp && r.same_node(world));
}

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
    View dv = local_view(dst, dlo, dhi, true, true);
    if (dv.bounce) view_rows(dv, ds, count, levels, (int64_t)row);
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
        if (host_side) sched_join_write(span_of(dv.dev, dlo, dhi));
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
            View dv = local_view(dst, dlo, dhi, true, true);
            if (dv.bounce) view_rows(dv, ds, count, levels, count[0]);
            wire_get_strided((uint64_t)(uintptr_t)src, ss, dv.dev, ds, count, levels, world);
            release_view(dv);
        } else {
            side_span_host(ss, count, levels, count[0], &slo, &shi);
            side_span_host(ds, count, levels, rb, &dlo, &dhi);
            check_remote(world, dst, dlo, dhi);
            View sv = local_view(src, slo, shi, false, true);
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
                // (and our IPC puts into world's memory): our streams drain first --
                // every kernel's end-of-kernel release (agent scope at least: the XCD
                // L2s written back) has then put its bytes where another GPU's
                // system-scope loads read them
                std::lock_guard<std::mutex> g(r.launch_mu);
                if (g_publish_conservative.load(std::memory_order_relaxed)) sched_publish_all();
                else sched_sync_all();
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
            sv = local_view(src, slo, shi, false, true, hdl != nullptr);
            dv.dev = remote_view(world, dst, dlo, dhi);
            dv.hbm = segment_kind_of(world, (const char *)dst + dlo) == 1;
        } else {
            sv.dev = remote_view(world, src, slo, shi);
            sv.hbm = segment_kind_of(world, (const char *)src + slo) == 1;
            dv = local_view(dst, dlo, dhi, true, true);
        }
    } else {
        local_views(src, slo, shi, dst, dlo, dhi, sv, dv, hdl != nullptr);
    }
    if (dv.bounce) view_rows(dv, ds, count, levels, kind == X_ACC ? rb : count[0]);
    // a pageable side in this thread's pinned bounce buffer, or pinned for this call, is
    // private to the call: the operation is scheduled as any other and completes on its
    // own stream before the views are released (small calls 37 -> 15 us,
    // profiles/r05/lat/); a staged copy (hipMemcpyAsync on stream 0) keeps the ordered
    // path below (stream 0, every stream synced)
    const bool bounce_only = (needs_sync(sv) || needs_sync(dv)) && !sv.staged && !dv.staged;
    const bool host_side = (needs_sync(sv) || needs_sync(dv)) && !bounce_only;
    // a get from another GPU's memory reads it with system-scope loads
    const bool peer = kind == X_GET && world != r.rank && r.peer_src(world);
    if (peer) g_peer_gets.fetch_add(1, std::memory_order_relaxed);
    int si = 0;
    hipStream_t st;
    {
        std::lock_guard<std::mutex> g(r.launch_mu);
        stamp(1);
        // staged copies sit on stream 0: run there, after everything (a dst in one of our
        // segments takes our memory lock first, as sched_pick does: ADVICE r3 high)
        if (host_side) sched_join_write(span_of(dv.dev, dlo, dhi));
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
    const bool synced = host_side || bounce_only || (!hdl && r.blocking_sync);
    if (!host_side && synced) {
        // HBM destination: a completion flag behind the kernel (sched_wait_flag, ~4 us
        // sooner than the runtime's signal; for a bounced source it also says the kernel
        // has read the bounce buffer); otherwise the runtime's sync, whose system-scope
        // release makes a host-memory destination's bytes visible
        if (dv.hbm) sched_wait_flag(si);
        else GA_HIP(hipStreamSynchronize(st));
    }
    if (world != r.rank && !synced && !r.direct_pending.empty()) r.direct_pending[world] = 1;
    if (r.debug)
        fprintf(stderr, "[ga_amd %d] %s -> %d levels %d count0 %d rows %d: src %s dst %s stream %d\n", r.rank,
                kind == X_ACC ? "acc" : (kind == X_PUT ? "put" : "get"), world, levels, count[0],
                levels ? count[levels] : 1, sv.registered ? "registered" : (sv.staged ? "staged" : "device"),
                dv.registered ? "registered" : (dv.staged ? "staged" : "device"), si);
    if (host_side || bounce_only) {
        release_view(sv);
        release_view(dv);
    }
    if (hdl) {
        nb_complete_now(hdl, si, true);
        if (sv.ring) ring_commit(si, r.nb_seq[*hdl]);
    }
    stamp(4);
    return COMEX_SUCCESS;
}

int xfer_contig(Xfer kind, int op, void *scale, void *src, void *dst, int bytes, int proc, int group,
                comex_request_t *hdl) {
    int count[1] = {bytes};
    if (bytes <= 0) fatal("contiguous transfer of %d bytes", bytes);   // nb_acc/nb_put assert bytes > 0
    return xfer(kind, op, scale, src, nullptr, dst, nullptr, count, 0, proc, group, hdl);
}

// ---- read-modify-write and mutexes -----------------------------------------
// comex_rmw (comex.h:670): the reference sends OP_FETCH_AND_ADD / OP_SWAP to the
// target's progress rank (comex.c:2120-2200), which applies it after every earlier
// message from that source.  Here: on this rank's own memory a one-lane kernel on
// the library stream that last touched those bytes; on a rank of this node a
// request in its inbox (after our earlier requests to it), applied by its progress
// thread on its GPU, the old value coming back through the node shm; on another
// node a wire frame.  (post_request_rmw: remote.cpp)
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
    progress_stop_at_exit(0.2);
    wire_detach();
}

// The HIP runtime this library's calls resolve to must be the one it was built
// against.  A torch wheel bundles its own libamdhip64 with the same SONAME
// (torch 2.10 + rocm7.0: HIP 7.0.51831); loaded before this library (torch imported
// first) it serves every HIP call here, and on it the inter-process memory calls of
// comex_malloc fail: hipIpcOpenMemHandle of a 2 GiB segment stalls while a 1 GiB
// one of the same peer is mapped, and hipMemImportFromShareableHandle of the vmm
// allocator's first 1 GiB descriptor kills the process with SIGSEGV
// (profiles/r05/runtime_diag/, phase traces; /opt/rocm 7.2 passes both).  The
// reference aborts with a message on any such condition (COMEX_ASSERT ->
// comex_error, comex_impl.h:52-76); so does this, before any device work, when other
// ranks share this node (their segments will be mapped here, and ours there).  A
// rank alone on its node never opens an inter-process mapping: for it the mismatch
// is a warning.  COMEX_AMD_ALLOW_HIP_MISMATCH=1 makes it a warning always.
static void check_hip_runtime(bool peers_map) {
    const char *path = gaamd_hip_runtime();
    int ver = 0;
    const bool got = hipRuntimeGetVersion(&ver) == hipSuccess;
    if (!got) (void)hipGetLastError();
    const int built = HIP_VERSION;
    trace(1, "HIP runtime %s, version %d (built against %d)", path, ver, built);
    if (got && ver / 100000 == built / 100000) return;   // same major.minor
    const char *allow = getenv("COMEX_AMD_ALLOW_HIP_MISMATCH");
    char msg[768];
    snprintf(msg, sizeof(msg),
             "HIP calls resolve to %s, runtime %d.%d.%d, but libga_amd was built against HIP %d.%d.%d "
             "(%s/lib); comex_malloc's inter-process mappings hang or crash on that runtime. Load libga_amd "
             "before the library that brought it (import ga_amd before torch), or set "
             "COMEX_AMD_ALLOW_HIP_MISMATCH=1 to run on it anyway",
             path, ver / 10000000, ver / 100000 % 100, ver % 100000, built / 10000000, built / 100000 % 100,
             built % 100000, GAAMD_ROCM_PATH);
    if ((allow && atoi(allow)) || !peers_map) {
        fprintf(stderr, "ga_amd warning: %s%s\n", msg,
                peers_map ? "" : " (no other rank on this node: no inter-process mapping, going on)");
        return;
    }
    fatal("%s", msg);
}

int comex_init() {
    Runtime &r = rt();
    if (r.initialized) return COMEX_SUCCESS;
    static bool hook = false;
    if (!hook) {
        atexit(exit_without_finalize);
        hook = true;
    }
    const char *dbg = getenv("COMEX_AMD_DEBUG");
    r.debug = dbg ? atoi(dbg) : 0;
    boot_init();   // host shm rendezvous only, no HIP call
    check_hip_runtime(r.node_size > 1);
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
        r.node_gpus = 0;   // distinct bus ids among this node's ranks
        for (int q = 0; q < r.size; ++q) {
            if (devs[q].node != r.node) continue;
            bool first = true;
            for (int k = 0; k < q && first; ++k)
                first = !(devs[k].node == r.node && !strcmp(devs[k].bus, devs[q].bus));
            if (first) ++r.node_gpus;
        }
        const char *pl = getenv("COMEX_AMD_PEER_LOADS");
        r.peer_loads = (pl && !strcmp(pl, "all")) ? 1 : ((pl && !strcmp(pl, "off")) ? 2 : 0);
        int peers = 0;   // same-node ranks whose memory is read as another GPU's
        for (int q = 0; q < r.size; ++q)
            if (r.same_node(q) && r.peer_src(q)) ++peers;
        // owner pulls from peer GPUs: one stream per source rank, so the chunks of
        // different peers (different xGMI links) are applied side by side
        // (at most 6: GPU_MAX_HW_QUEUES is 4 here, more streams share hardware queues;
        // the former COMEX_AMD_PULL_STREAMS knob, settled)
        const int pull = std::min(peers, 6);
        // 2 library streams: independent ops overlap kernel edges; 1 when
        // other ranks of the job share this GPU: their processes fill it anyway, and two
        // streams per process made a small blocking call wait 55-80 us for its kernel
        // instead of 13-15 and lowered the aggregate rate by 2-8 % (2 and 4 ranks on one
        // GPU, profiles/r05/lat7/)
        // (ranks read as another GPU's, COMEX_AMD_PEER_LOADS=all, are counted as such: the
        // one-GPU proxy of a multi-GPU node keeps that node's two streams)
        int sharing = 0;
        for (int q = 0; q < r.size; ++q)
            if (q != r.rank && r.same_dev[q] && !r.peer_src(q)) ++sharing;
        const char *ns = getenv("COMEX_AMD_STREAMS");
        sched_init(ns ? atoi(ns) : (sharing ? 1 : 2), pull);
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
        // the direct-source route is always on (the former COMEX_AMD_DIRECT_SRC knob:
        // its A/B settled in round 2; COMEX_ENABLE_ACC_SMP=0 still turns it off, as the
        // reference's SMP toggle does)
        r.direct_src = true;
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
    if (r.size > 1 || !r.acc_self_direct || !r.put_self_direct || !r.get_self_direct) {
        remote_init();   // staging HBM + inbox + progress thread (remote.cpp)
        wire_init();
    }
    r.initialized = true;
    boot_barrier();
    // the ARMCI_VERBOSE dump of the reference (comex.c:545-572): this run's configuration
    const char *vb = getenv("COMEX_AMD_VERBOSE");
    if (vb && atoi(vb) && r.rank == 0) {
        hipDeviceProp_t prop;
        const bool okp = hipGetDeviceProperties(&prop, r.device) == hipSuccess;
        const char *seg = getenv("COMEX_AMD_SEGMENT");
        fprintf(stderr,
                "%s: ranks %d on %d node(s), device %d (%s, %d CUs), library streams %d, "
                "staging %zu MiB/rank, segments in %s, blocking sync %d, "
                "acc to self %s, put to self %s, same-node put %s\n",
                gaamd_version(), r.size, r.nnodes, r.device, okp ? prop.gcnArchName : "?",
                okp ? prop.multiProcessorCount : 0, (int)r.streams.size(), r.staging_bytes >> 20,
                (seg && !strcmp(seg, "host")) ? "host" : "HBM",
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
    one_pass_finalize();                // the one-pass locks were handed back by the barrier's fence
    wire_finalize();
    remote_finalize();                  // progress thread stopped
    boot_barrier();
    segments_finalize();                // every mapping closed, every block freed
    remote_release_staging();
    boot_barrier();
    remote_free_staging();
    segments_release_blocks();          // the freed-segment cache and quarantined blocks
    vmm_finalize();                     // the reserved address ranges
    sched_sync_all();
    sched_fini();
    sched_flag_fini();
    if (g_get_scratch) (void)hipFree(g_get_scratch);
    g_get_scratch = nullptr;
    g_get_scratch_bytes = 0;
    if (g_get_scratch_ev) (void)hipEventDestroy(g_get_scratch_ev);
    g_get_scratch_ev = nullptr;
    iov_finalize();
    views_finalize();
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
        if (g_publish_conservative.load(std::memory_order_relaxed)) sched_publish_all();
        else sched_sync_all();
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
        if (job_pending(g_nb_job[*h])) { *status = 1; return COMEX_SUCCESS; }
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

// Test and diagnostic hooks: one entry point, not used by GA (include/ga_amd.h
// section 7).  "stamps": the bench's value-region stamps (value 1: clear and start,
// 0: stop, -1: leave as is; out[0..7] gets them when nout >= 8).  "stale_gen" /
// "stale_granule": the segment tests' stale-mapping hooks (segments.cpp).
int gaamd_diag(const char *key, long long value, unsigned long long *out, int nout) {
    if (!key) return -1;
    if (!strcmp(key, "stamps")) {
        if (out && nout >= 8)
            for (int k = 0; k < 8; ++k) out[k] = g_stamp[k];
        if (value >= 0) {
            if (value) memset(g_stamp, 0, sizeof(g_stamp));
            g_stamp_on.store(value != 0, std::memory_order_relaxed);
        }
        return 0;
    }
    if (!strcmp(key, "stale_gen")) {
        g_diag_stale_gen.store(value);
        return 0;
    }
    if (!strcmp(key, "stale_granule")) {
        g_diag_stale_granule.store(value);
        return 0;
    }
    if (!strcmp(key, "host_range")) {   // out[0], out[1] in: [lo, hi); value: 1 = writable; out[0] out: 1/0
        if (!out || nout < 2) return -1;
        out[0] = host_cpu_range_probe(out[0], out[1], value != 0) ? 1 : 0;
        return 0;
    }
    if (!strcmp(key, "publish")) {   // 1: the conservative publication mode, 0: the default; out[0] = old
        if (out && nout >= 1) out[0] = g_publish_conservative.load() ? 1 : 0;
        if (value >= 0) g_publish_conservative.store(value != 0);
        return 0;
    }
    if (!strcmp(key, "drop_chunk")) {   // N > 0: the owner drops every N-th packed chunk (test hook), 0: off
        g_diag_drop_chunk.store(value);
        return 0;
    }
    if (!strcmp(key, "peer_gets")) {   // strided gets this rank read from another GPU's memory
        if (out && nout >= 1) out[0] = g_peer_gets.load(std::memory_order_relaxed);
        return 0;
    }
    if (!strcmp(key, "vmm_window")) {   // out[0] bytes of the vmm private window taken, out[1] left
        if (!out || nout < 2) return -1;
        vmm_window_usage(&out[0], &out[1]);
        return 0;
    }
    if (!strcmp(key, "pinned_threads")) {   // threads holding pinned bounce buffers or an nb ring
        if (out && nout >= 1) out[0] = views_pinned_threads();
        return 0;
    }
    if (!strcmp(key, "iov_host_sides")) {   // io-vector sides found wholly in pageable host memory
        if (out && nout >= 1) out[0] = g_iov_host_sides.load(std::memory_order_relaxed);
        return 0;
    }
    return -1;
}

int gaamd_iov_path_counts(unsigned long long counts[4]) {
    for (int k = 0; k < 4; ++k) counts[k] = g_iov_path[k].load(std::memory_order_relaxed);
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


