// comex_impl.hpp -- internals shared by the files that implement the ComEx C API
// (include/comex.h) on MI355X.  Reference: comex/src-mpi-pr/comex.c.
//
//   comex.cpp     C ABI entry points, comex_init/finalize, non-blocking handles, the
//                 transfer routing of strided operations (xfer: self / one-pass /
//                 direct-source / packed / wire), rmw, mutexes, groups
//   segments.cpp  comex_malloc/free: HBM segments exported by IPC or host segments in
//                 node shared memory, peer mappings and their tag check, the IPC
//                 address history, the freed-segment cache (reg_cache, comex.c:2359-2605)
//   views.cpp     device views of user pointers (segments, HBM, pinned, pageable host)
//   remote.cpp    staging ring, owner inbox, the progress thread (_progress_server,
//                 comex.c:3379-3565) and the asynchronous remote-accumulate jobs
//                 (nb_accs_packed, comex.c:6965-7109)
//   onepass.cpp   the one-pass route between ranks of one GPU and its memory-lock
//                 protocol (the per-target semaphore of comex.c:6241-6260)
//   iov.cpp       io-vector transfers, comex_accv/putv/getv (comex.c:7327-7400)
#pragma once
#include "runtime.hpp"
#include "gaamd_kernels.h"
#include "../../include/comex.h"
#include <stdint.h>
#include <atomic>
#include <deque>
#include <vector>

namespace gaamd {

constexpr long kPage = 4096;

inline void ensure_init() {
    if (!rt().initialized) fatal("comex used before comex_init");
}

// ---- device views of user pointers (views.cpp) ------------------------------
struct View {
    char *dev = nullptr;          // device-accessible address of the user pointer
    void *registered = nullptr;   // page base we registered for this call
    char *staged = nullptr;       // fallback: device copy of [host+lo, host+hi)
    char *bounce = nullptr;       // small pageable span: pinned copy of [host+lo, host+hi)
    // a bounced destination is written back row by row (only the bytes the kernel wrote):
    // wb_host is the user's dst pointer, wb_bounce the matching address in the bounce copy
    char *wb_host = nullptr, *wb_bounce = nullptr;
    const int *wb_stride = nullptr, *wb_count = nullptr;
    int wb_levels = -1;
    int64_t wb_row = 0;
    char *host = nullptr;
    int64_t lo = 0, hi = 0;
    bool copy_back = false;
    bool hbm = false;             // device memory the CPU never touches (HBM segment or hipMalloc)
    bool ring = false;            // a pageable source copied into the thread's nb ring (ring_view)
};
// device-visible without help (our segments, HBM, managed, pinned/registered host);
// *hbm (optional): the memory is HBM (not managed, not host)
bool direct_view(void *p, char **dev, bool *hbm = nullptr);
// src and dst of one local transfer; a pageable pair whose page ranges overlap is
// registered once as a union
// (small pageable spans through a pinned bounce buffer: synchronous callers only)
// ring_src: a non-blocking call -- a small pageable source with a direct destination goes
// through the thread's ring (ring_view), and the call need not wait for its kernel
void local_views(void *src, int64_t slo, int64_t shi, void *dst, int64_t dlo, int64_t dhi, View &sv, View &dv,
                 bool ring_src = false);
// bounce_ok: the caller completes the transfer before release_view and before its next
// transfer (a small pageable span may then use the thread's pinned bounce buffer)
// ring_ok: a non-blocking call's source (ring_view)
View local_view(void *p, int64_t lo, int64_t hi, bool is_dst = false, bool bounce_ok = false, bool ring_ok = false);
// a small pageable source [p + lo, p + hi) copied into this thread's pinned ring (false: too
// large); ring_commit then names the operation that reads it (stream, sched_track sequence)
bool ring_view(View &v, void *p, int64_t lo, int64_t hi);
void ring_commit(int stream, uint64_t seq);
size_t views_pinned_threads();   // threads holding pinned bounce/ring buffers now
void views_finalize();    // every thread's pinned bounce buffers and ring (comex_finalize)
inline bool needs_sync(const View &v) { return v.registered || v.staged || v.bounce; }
// the rows a bounced destination view's kernel writes (dst strides, count, levels, row
// bytes): release_view copies back those rows only; without it, nothing but the view's
// own span [lo, hi)
void view_rows(View &v, const int *stride, const int *count, int levels, int64_t row_bytes);
// after the kernel: copy a staged dst back, then unpin / free (stream synced by caller)
void release_view(View &v);

inline Span span_of(const void *base, int64_t lo, int64_t hi) {
    Span s;
    s.lo = (int64_t)(uintptr_t)base + lo;
    s.hi = (int64_t)(uintptr_t)base + hi;
    return s;
}

enum Xfer { X_ACC, X_PUT, X_GET };

inline uint64_t payload_bytes(int64_t row_bytes, const int *count, int levels) {
    uint64_t n = (uint64_t)row_bytes;
    for (int j = 1; j <= levels; ++j) n *= (uint64_t)count[j];
    return n;
}

inline int64_t row_bytes_of(int op, int count0) {
    const int esz = elem_size(op);
    return (op == kOpCopy) ? count0 : (int64_t)(count0 / esz) * esz;
}

// ---- segments (segments.cpp) ------------------------------------------------
bool find_segment_local(const void *p, int64_t lo, int64_t hi);   // caller holds seg_mu
void check_remote(int owner, const void *p, int64_t lo, int64_t hi);
// address of rank `owner`'s byte `p` (owner's address space) in this process
char *remote_view(int owner, const void *p, int64_t lo, int64_t hi);
// [p+lo, p+hi) inside one of our HBM segments that rank t mapped at comex_malloc
bool src_segment_shared(const void *p, int64_t lo, int64_t hi, int t);
// d meets one of our segments that same-GPU ranks may write (one-pass route)
bool in_own_segment(const Span &d);
// rank `owner`'s segment holding p (owner's address space): 0 none, 1 HBM, 2 host
int segment_kind_of(int owner, const void *p);
// the tag a rank writes into a new exported block (segments, the staging buffer)
uint64_t seg_tag(int rank, uint64_t gen, int end);
// the IPC handle table a stale mapping is reported against (rank, allocation number)
void handle_seen(int rank, uint64_t gen, uint64_t base, uint64_t bytes, const hipIpcMemHandle_t &h);
void *ipc_open(hipIpcMemHandle_t h, int q, const char *what);
void ipc_close(void *mapped, int peer);
// IPC handle of a fresh hipMalloc block *p (another block if the export is refused)
void export_alloc(void **p, size_t bytes, hipIpcMemHandle_t *h, const char *what);
// test hooks (gaamd_diag): every peer treats its first mapping of each rank's N-th
// allocation as stale (stale_gen = N, stale_granule < 0), or the owner writes a
// foreign tag into granule G of it (stale_granule = G) for the check to find
extern std::atomic<long long> g_diag_stale_gen, g_diag_stale_granule;
extern std::atomic<long long> g_diag_drop_chunk;   // gaamd_diag("drop_chunk"): remote.cpp
extern std::atomic<unsigned long long> g_peer_gets;   // gaamd_diag("peer_gets"): comex.cpp
void segments_finalize();         // every live segment: peer mappings closed, block freed
void segments_release_blocks();   // the freed-segment cache and the quarantined blocks

// ---- HBM segments through the virtual-memory API (vmm.cpp) ---------------------
bool vmm_enabled();                       // COMEX_AMD_SEGMENT_ALLOC=vmm
void vmm_window_usage(unsigned long long *used, unsigned long long *left);   // private window bytes
size_t vmm_round(size_t bytes);           // to the allocation granularity
void *vmm_alloc(size_t bytes, VmmBlock *b);                  // this GPU's HBM, exported (b->fd)
void vmm_listen();                        // this process's descriptor socket (before the allgather)
void vmm_exchange(int fd, int rank, uint64_t gen, const std::vector<int> &to_pids,
                  const std::vector<std::pair<int, uint64_t>> &from, int *fds);   // SCM_RIGHTS both ways
void *vmm_import(int myfd, size_t bytes, int q, VmmBlock *b);   // rank q's block
void vmm_quarantine(VmmBlock *b);        // a block whose peers' mappings read other memory: set aside
void vmm_free(VmmBlock *b);               // unmap + release + the virtual range back
void vmm_finalize();

// ---- remote operations through the owner (remote.cpp) -----------------------
void remote_init();             // staging buffer, peer mappings, progress thread (collective)
void remote_finalize();
void progress_stop_at_exit(double wait_s);   // exit without comex_finalize: join an idle progress thread         // after comex_barrier: job bookkeeping freed, progress thread stopped
void remote_release_staging();  // the peers' staging mappings closed
void remote_free_staging();     // our staging freed (after a barrier: nobody maps it)
uint64_t sub_ring_bytes();
inline uint64_t ring_len(uint64_t len) { return (len + 255) & ~255ull; }   // 256-byte aligned requests
struct Pending { uint64_t seq, off, len; };
extern std::vector<std::deque<Pending>> g_pend;   // per target: staging slices the owner still reads
void wait_done(int t, uint64_t seq);
uint64_t stage_alloc(int t, uint64_t len);
// io-vector request layout in staging: n packed runs, then the n owner addresses
inline uint64_t iov_list_off(int n, int bytes) { return (((uint64_t)n * (uint64_t)bytes) + 15) & ~15ull; }
void post_request_iov(int t, int op, const void *scale, int bytes, int n, uint64_t off, uint64_t len, uint64_t dlo,
                      uint64_t dhi, uint64_t align_or, int mode);
void post_request_direct(int t, int op, const void *scale, uint64_t dst_addr, const int *dst_stride,
                         uint64_t src_addr, const int *src_stride, const int *count, int levels);
void post_request_get(int t, uint64_t src_addr, const int *src_stride, const int *count, int levels, uint64_t off,
                      uint64_t len, uint64_t rb, uint64_t re);
void post_request_rmw(int t, int swap, uint64_t addr, int bytes, uint64_t val);
bool progress_jobs();        // one non-blocking pass over the remote-accumulate jobs
bool job_pending(int id);
void run_job(int id);
void drain_target(int t);
void drain_all_jobs();
bool target_busy(int t);
bool dst_rows_disjoint(const int *str, const int *count, int levels, int64_t row_bytes);
// start a remote accumulate (or owner-applied put); returns its job id (0: nothing left)
int remote_acc_start(int t, int op, const void *scale, void *src, const int *ss, void *dst, const int *ds,
                     const int *count, int levels);
void fence_target(int t);
void fence_self_if_pending();
extern std::atomic<unsigned long long> g_route[4];   // gaamd_route_counts
extern std::atomic<unsigned long long> g_owned[4];   // gaamd_owner_counts

// ---- one-pass route between ranks of one GPU (onepass.cpp) ------------------
// true: launched (blocking: complete on return; else `hdl` tracks it); false: not eligible
bool one_pass_acc(int t, int op, void *scale, void *src, const int *ss, void *dst, const int *ds, const int *count,
                  int levels, int64_t rbd, comex_request_t *hdl);
bool own_release_if_wanted();     // progress thread: hand our memory lock to a waiting requester
bool one_pass_reap(bool wait);    // release the owners' locks our kernels no longer need
bool one_pass_reap_try();         // the same without waiting for the bookkeeping lock (never blocks)
void one_pass_finalize();
extern std::atomic<unsigned long long> g_one_pass;

// ---- io-vector transfers (iov.cpp) -------------------------------------------
int xfer_vec(Xfer kind, int op, void *scale, comex_giov_t *darr, int len, int proc, int group, comex_request_t *hdl);
void iov_finalize();
extern std::atomic<unsigned long long> g_iov_path[4];   // gaamd_iov_path_counts
extern std::atomic<unsigned long long> g_iov_host_sides;   // gaamd_diag("iov_host_sides")
bool host_cpu_range_probe(uint64_t lo, uint64_t hi, bool write);   // gaamd_diag("host_range")

// ---- comex.cpp ----------------------------------------------------------------
// handle of an op just enqueued on library stream `stream_idx` (`on_stream`), or of
// one with nothing left on a stream
void nb_complete_now(comex_request_t *h, int stream_idx = 0, bool on_stream = false);
// the reference's self/SMP test: true when the self or SMP route applies to `world`
bool self_smp_route(Xfer kind, int world);
int xfer_contig(Xfer kind, int op, void *scale, void *src, void *dst, int bytes, int proc, int group,
                comex_request_t *hdl);
extern std::atomic<unsigned long long> g_toggle[3];   // gaamd_toggle_counts: rows, pairs, owner gets

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

}  // namespace gaamd
