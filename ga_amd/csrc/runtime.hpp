// runtime.hpp -- process-wide state of the ComEx/ARMCI runtime on MI355X.
//
// Reference counterparts (comex/src-mpi-pr/comex.c):
//   g_state (rank/size/host table)        -> Runtime::{rank,size,local_rank}
//   reg_cache (reg_cache.c:380-409)       -> Runtime::segs (owner base -> mapped ptr)
//   nb_state[COMEX_MAX_NB_OUTSTANDING]    -> Runtime::nb_* (stream + sequence, sched.cpp marks)
//   per-rank POSIX semaphores (2812-2908) -> none: every write into rank t's
//       HBM is issued on rank t's stream (its own ops, or requests its progress
//       thread drains), so stream order serialises accumulates per target.
//   progress rank (_progress_server 3379-3565, _acc_packed_handler 4133-4281)
//       -> a progress thread per process draining a node-shared inbox.
#pragma once
#include <stdint.h>
#include <stddef.h>
#include <atomic>
#include <vector>
#include <mutex>
#include <thread>
#include <hip/hip_runtime_api.h>
#include "../../include/ga_amd.h"

namespace gaamd {

[[noreturn]] void fatal(const char *fmt, ...);
// a line on stderr when COMEX_AMD_DEBUG >= level (phase traces of init / comex_malloc)
void trace(int level, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

#define GA_HIP(call)                                                                  \
    do {                                                                              \
        hipError_t e_ = (call);                                                       \
        if (e_ != hipSuccess)                                                         \
            ::gaamd::fatal("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_),     \
                           __FILE__, __LINE__);                                       \
    } while (0)

#define GA_ASSERT(cond, msg)                                                          \
    do {                                                                              \
        if (!(cond)) ::gaamd::fatal("assertion `%s` failed: %s (%s:%d)", #cond, msg,  \
                                    __FILE__, __LINE__);                              \
    } while (0)

constexpr int kMaxNb = 256;          // COMEX_MAX_NB_OUTSTANDING default
constexpr int kMaxRanks = 64;        // ranks per node
constexpr int kInboxSlots = 256;     // requests in flight per target
constexpr size_t kBootSlot = 64 * 1024;
constexpr int kMaxMutexes = 4096;    // comex_create_mutexes: locks per rank (node shm words)

// ---- node-shared memory (one mapping per node, created at init) ----------
struct alignas(64) Request {
    std::atomic<uint32_t> state;     // 0 free, 1 writing, 2 ready
    int32_t src_rank;
    int32_t op;                      // COMEX_ACC_* (or 0 = copy)
    int32_t levels;
    int32_t count[8];
    int32_t dst_stride[8];
    uint64_t dst_addr;               // owner's address space
    uint64_t staging_off;            // offset into src_rank's staging buffer
    uint64_t bytes;                  // packed bytes
    uint64_t seq;                    // strided: row range (begin << 32 | end)
    uint8_t scale[16];
    int32_t kind;                    // 0 strided (count/dst_stride), 1 io-vector, 2 rmw,
                                     // 3 strided read straight from src_rank's segment,
                                     // 4 get: our patch (src_addr/src_stride) packed into
                                     //   src_rank's staging at staging_off (row range in seq)
    int32_t iov_serial;              // io-vector: destinations overlap -> in order
    uint64_t iov_align;              // io-vector: OR of the destination addresses
    uint64_t dst_hi;                 // io-vector: [dst_addr, dst_hi) covers every pair
    int32_t src_stride[8];           // kind 3: the source patch in src_rank's segment; kind 4: ours
    uint64_t src_addr;               // kind 3: src_rank's address space; kind 4: ours
};

struct alignas(64) Inbox {
    std::atomic<uint64_t> tail;      // producers reserve slots
    char pad0[56];
    std::atomic<uint64_t> head;      // consumer position
    char pad1[56];
    Request slot[kInboxSlots];
};

// comex_rmw reply to one requester (requests are blocking: one in flight per rank)
struct alignas(64) RmwReply {
    std::atomic<uint64_t> seq;       // replies delivered so far
    uint64_t value;                  // the old remote value (4 or 8 bytes)
};

struct alignas(64) NodeShm {
    std::atomic<uint32_t> magic;
    int32_t size;
    std::atomic<uint64_t> bar_count;
    std::atomic<uint64_t> bar_gen;
    char pad[40];
    // done[s][t]: requests from s applied by t (monotonic); s, t = positions on the node
    std::atomic<uint64_t> done[kMaxRanks][kMaxRanks];
    RmwReply rmw[kMaxRanks];         // indexed by the requester's position on the node
    // one-pass accumulates between ranks sharing a GPU (comex.cpp one_pass_acc):
    // mem_lock[t] = 0 free, 1 + p held by node position p (the owner t itself while
    // its own writes into its segments may be in flight, or a requester while its
    // kernel writing t's segment runs); mem_want[t] = requesters waiting for it
    std::atomic<uint32_t> mem_lock[kMaxRanks];
    std::atomic<uint32_t> mem_want[kMaxRanks];
    Inbox inbox[1];                  // [size] follows; then boot data area
};

size_t node_shm_bytes(int size);
Inbox *inbox_of(NodeShm *s, int rank);
char *boot_area(NodeShm *s, int size);
// lock words of the comex mutexes of the rank at node position `rank`
std::atomic<uint32_t> *mutex_words(NodeShm *s, int size, int rank);

// a device-view byte range [lo, hi) touched by one operation (lo == hi: none)
struct Span {
    int64_t lo = 0, hi = 0;
};

struct PeerMap {
    uintptr_t base = 0;   // segment address in the owner's address space
    size_t bytes = 0;
    char *mapped = nullptr;   // same bytes as seen from this process (device-accessible)
    bool member = false;      // the rank took part in the segment's comex_malloc
    // host segments: this process's mapping of the owner's node shm object (page-
    // rounded bytes), registered with HIP; `mapped` is its device view (the same
    // address: do_malloc checks it)
    char *host_map = nullptr;
    size_t map_bytes = 0;
};

// an HBM block of the virtual-memory allocator (vmm.cpp): its mapping here, the
// physical handle and its dmabuf descriptor (an owner's export or a peer's import)
struct VmmBlock {
    char *va = nullptr;
    size_t bytes = 0;                    // mapped bytes (granularity-rounded)
    hipMemGenericAllocationHandle_t handle{};
    int fd = -1;
    bool imported = false;
};

struct Segment {
    bool live = false;
    bool vmm = false;            // HBM from vmm.cpp (own block in vmm_local, peers' in vmm_peer)
    VmmBlock vmm_local;
    std::vector<VmmBlock> vmm_peer;
    bool device = true;          // HBM (IPC-exported) or a host segment in node shm
    void *local = nullptr;
    size_t local_bytes = 0;      // bytes of the local block
    bool exported = false;       // `handle` is the local block's IPC export
    hipIpcMemHandle_t handle;
    std::vector<PeerMap> peer;   // indexed by world rank
};

struct Runtime {
    bool initialized = false;
    bool boot_ready = false;
    int rank = 0, size = 1, local_rank = 0, device = 0;
    // nodes (hosts): ranks of one node share the node shm and map each other's HBM
    int nnodes = 1, node = 0, node_size = 1;
    std::vector<int> node_of;                  // node index of every rank
    std::vector<int> node_index;               // every rank's position on its node (node shm slots)
    int li(int q) const { return node_index.empty() ? q : node_index[q]; }
    bool same_node(int q) const { return node_of.empty() || node_of[q] == node; }
    hipStream_t stream = nullptr;              // primary stream (= streams[0])
    std::vector<hipStream_t> streams;          // COMEX_AMD_STREAMS streams (sched.cpp)
    // COMEX_AMD_BLOCKING_SYNC (default 1): a blocking call returns once its kernel
    // has finished, i.e. src is reusable and a get's dst holds the data, as the
    // reference's blocking calls promise; 0 is the documented
    // opt-out where blocking calls are only stream-ordered
    bool blocking_sync = true;
    // COMEX_ENABLE_{ACC,PUT}_{SELF,SMP} (comex.c:438-471, defaults 1): with both
    // SELF and SMP off, an accumulate / put to this rank takes the packed route
    // (pack into staging, the progress thread unpacks) as a remote one does;
    // PUT_SMP off also sends same-node puts that way instead of through the IPC
    // mapping.  (Same-node accumulates always take the packed route here.)
    // ACC_SMP off also turns the direct-source route off (a same-node accumulate
    // then always packs, comex.c:6911-6915)
    bool acc_self_direct = true, acc_smp_direct = true, put_self_direct = true, put_smp_direct = true;
    // COMEX_ENABLE_GET_{SELF,SMP} (comex.c:444-465, nb_get 6157-6214): with both off a
    // get from this rank, with SMP off a get from a rank sharing this GPU, goes
    // through the owner (kind 4: its progress thread packs the patch into our
    // staging, we unpack it) instead of reading the owner's memory directly
    bool get_self_direct = true, get_smp_direct = true;
    // COMEX_ENABLE_{ACC,PUT,GET}_PACKED and _IOV (comex.c:474-531): off, a strided /
    // io-vector operation that does not take the self/SMP route goes row by row /
    // pair by pair as contiguous operations (nb_accs 6918-6961, nb_accv 7342-7351)
    bool acc_packed = true, put_packed = true, get_packed = true;
    bool acc_iov = true, put_iov = true, get_iov = true;
    // COMEX_AMD_DIRECT_SRC (default 1): a same-node accumulate whose source lies
    // in one of this rank's HBM segments is applied by the owner straight from
    // that segment (its IPC mapping) -- no pack pass, no staging
    bool direct_src = true;
    int debug = 0;                  // COMEX_AMD_DEBUG: trace transfers on stderr
    // bootstrap
    gaamd_allgather_fn ag = nullptr;
    gaamd_barrier_fn bar = nullptr;
    void *ctx = nullptr;
    bool hooks = false;
    NodeShm *shm = nullptr;
    size_t shm_bytes = 0;
    // memory
    std::vector<Segment> segs;
    std::mutex seg_mu;
    // non-blocking handles: the op's stream and its sequence number there (sched.cpp
    // completion marks; seq 0 = nothing left on a stream)
    int nb_stream[kMaxNb] = {};
    uint64_t nb_seq[kMaxNb] = {};
    bool nb_used[kMaxNb] = {};
    int nb_next = 0;
    // remote (multi-rank) state
    char *staging = nullptr;            // this rank's exported staging buffer
    size_t staging_bytes = 0;
    std::vector<char *> peer_staging;   // mapped staging of every rank
    std::vector<uint64_t> posted;       // requests posted to each target
    std::vector<uint64_t> stage_head;   // per-target staging ring write cursor
    // per target: a put/get kernel addressing that rank's HBM through its IPC
    // mapping may still run on one of our streams; a following remote
    // accumulate (applied by the owner's progress thread) must wait for it
    std::vector<uint8_t> direct_pending;
    std::thread progress;
    std::atomic<bool> stop{false};
    std::mutex launch_mu;
    // devices: same_dev[q] = rank q's HIP device is this rank's physical GPU (PCI
    // bus id), so its HBM is local memory here.  Another GPU's memory is only ever
    // READ by this rank's kernels, with system-scope loads (peer_src), and every
    // write into it is made by its owner: puts to it take the packed route.
    // COMEX_AMD_PEER_LOADS: auto (default: per device), all (every other rank's
    // memory as if on another GPU -- exercises that path on one GPU), off.
    std::vector<uint8_t> same_dev;
    int node_gpus = 1;                  // distinct physical GPUs among this node's ranks
    int peer_loads = 0;                 // 0 auto, 1 all, 2 off
    bool peer_src(int q) const {
        if (q == rank || peer_loads == 2) return false;
        return peer_loads == 1 || q >= (int)same_dev.size() || !same_dev[q];
    }
    int user_streams = 2;               // streams[0, user_streams): every operation; the rest: owner pulls
    // one-pass accumulate into a segment of a rank on THIS GPU (COMEX_AMD_ONE_PASS,
    // default on when such a rank exists): the requester's fused kernel writes the
    // owner's segment, under the owner's node-shm memory lock (NodeShm::mem_lock)
    bool one_pass = false;
    bool own_holds = false;             // this process holds its own mem_lock (launch_mu)
};

Runtime &rt();

// bootstrap.cpp
void boot_init();                                  // rank/size + node shm
void boot_allgather(const void *send, void *recv, size_t bytes);
void boot_barrier();
void boot_finalize();

// sched.cpp (callers hold launch_mu)
// give the freed device segments kept for reuse (comex.cpp) back to the runtime
void segment_cache_flush();
void sched_init(int nstreams, int pull_streams = 0);
void sched_fini();
void sched_resize(int nstreams);
// comex.cpp: before a launch that writes `dst` (caller holds launch_mu): a write
// into one of this rank's segments takes this rank's memory lock when a rank on the
// same GPU may write them too (one-pass accumulates); a no-op otherwise
void own_write_guard(const Span &dst);
// stream index for an op; payload = its bytes (0: unknown); prefer = stream for an
// op with no dependency (owner pulls from a peer GPU: one stream per source rank)
int sched_pick(const Span &src, const Span &dst, uint64_t payload = 0, int prefer = -1);
void sched_join();
// blocking-call completion with HBM operands: a flag kernel behind stream s's work,
// the host spinning on it (caller does NOT hold launch_mu); sched_flag_fini at finalize
void sched_wait_flag(int s);
void sched_flag_init();   // the flag page (sched_init)
void sched_flag_fini();
// sched_join before a launch that writes `dst` (own_write_guard first); a span of
// unknown extent is Span{0, INT64_MAX}
void sched_join_write(const Span &dst);
void sched_sync_all();
// sched_sync_all behind a system-scope release on every library stream (the
// conservative publication mode, g_publish_conservative)
void sched_publish_all();
extern std::atomic<bool> g_publish_conservative;   // gaamd_diag("publish")
// completion marks (user thread): sequence number of an op just enqueued on
// stream s; whether op `seq` of stream s has completed (waiting for it if `wait`)
uint64_t sched_track(int s);
bool sched_complete(int s, uint64_t seq, bool wait);
// bumped by sched_init: sequence numbers of an earlier epoch were drained (finalize, resize)
uint64_t sched_epoch();

// wire.cpp: the host fallback between nodes (MPI-PR message protocol over TCP)
void wire_init();                                   // collective; no-op on one node
void wire_finalize();                               // collective
void wire_detach();                                 // process exit without finalize
bool wire_active();
// put (op == 0) / accumulate of a local strided patch into rank t's `dst`
void wire_send_strided(int op, const void *scale, const char *src_dev, const int *ss, uint64_t dst,
                       const int *ds, const int *count, int levels, int t);
// get of rank t's strided patch at `src` into a local patch
void wire_get_strided(uint64_t src, const int *ss, char *dst_dev, const int *ds, const int *count, int levels,
                      int t);
// io-vector put (op == 0) / accumulate: n local device sources -> n addresses of rank t
void wire_send_iov(int op, const void *scale, const uint64_t *src_dev, const uint64_t *dst, int n, int bytes,
                   bool serial, int t);
// io-vector get: n addresses of rank t -> n local device destinations
void wire_get_iov(const uint64_t *src, const uint64_t *dst_dev, int n, int bytes, int t);
void wire_fence(int t);                             // remote completion of everything sent to t
// armci_msg transport (every multi-rank job): tagged byte messages, in send order per sender
void msg_send(int to, int tag, const void *buf, size_t len);
size_t msg_recv(int from, int tag, void *buf, size_t buflen, int *src);   // from < 0: any sender
// comex_rmw / comex_lock on a rank of another node
uint64_t wire_rmw(int t, int swap, uint64_t addr, int bytes, uint64_t val);
bool wire_lock(int t, int mutex, bool acquire);   // acquire: try once (true = held); else release
// comex.cpp: operations on this rank's (or this node's) memory, for the wire server
uint64_t rmw_local(int swap, void *addr, int bytes, uint64_t val);
bool mutex_try_local(int owner, int mutex);
void mutex_release_local(int owner, int mutex);
bool segment_of_rank(int owner, uint64_t p, int64_t lo, int64_t hi);   // comex.cpp (reg_cache_find)
bool segment_local(const void *p, int64_t lo, int64_t hi);              // segments.cpp
// 0: not in one of our segments, 1: in an HBM segment, 2: in a host (node shm) segment
int segment_kind(const void *p);
// comex.cpp: the device-address history a refused IPC export prints (kind: a alloc,
// f free, x export, o IPC map, c IPC unmap; peer = the other rank, -1 none)
void addr_event(char kind, const void *p, size_t bytes, int peer);
void addr_history(const void *p, size_t bytes);   // the logged events touching a range, to stderr

// comex.cpp helpers shared with armci.cpp / armci_msg.cpp
int translate_world(int group, int proc);
std::vector<int> group_members(int group);   // world ranks in group-rank order
// armci_msg.cpp: collectives over a member list (world ranks), by messages
// (msg_send/msg_recv); `key` separates the traffic of different groups
void members_allgather(const std::vector<int> &members, int key, const void *send, void *recv, size_t bytes);
void members_barrier(const std::vector<int> &members, int key);
void members_bcast(const std::vector<int> &members, int key, void *buf, size_t bytes, int root_index);

}  // namespace gaamd
