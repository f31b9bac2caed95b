/*
 * ga_amd.h -- framework-level C ABI of libga_amd.so beyond comex.h/armci.h.
 *
 *  1. Bootstrap hooks.  The reference exchanges segment registrations and
 *     semaphore names with MPI_Allgather (comex/src-mpi-pr/comex.c:2461, 2874)
 *     and synchronises with MPI_Barrier (comex.c:1231).  Here the host program
 *     may hand in its own allgather/barrier (torch.distributed, MPI, ...);
 *     without hooks comex_init() uses RANK/WORLD_SIZE/LOCAL_RANK (or the
 *     OMPI_/PMI_ equivalents) and a node-local shared-memory rendezvous.
 *  2. Kernel-level entry points: the gfx950 kernels that comex_accs/puts/gets
 *     enqueue, callable directly on device pointers with an explicit stream.
 *     They replace, element for element:
 *       gaamd_strided(op=COMEX_ACC_*) : nb_accs per-row _acc  comex.c:6890-6962,
 *                                       acc.h:106-154
 *       gaamd_strided(op=GAAMD_OP_COPY): nb_puts/nb_gets       comex.c:6342-6427, 6617-6696
 *       gaamd_pack                     : pack                   comex.c:1267-1328
 *       gaamd_unpack                   : unpack                 comex.c:1331-1384
 *       gaamd_unpack_acc               : _acc_packed_handler    comex.c:4238-4268
 *  3. Device plumbing used by tests and bench.py (allocation, copies,
 *     synthetic inputs, HIP-event timing, tuning knobs).
 *
 * All functions return 0 on success and a negative code on failure unless
 * stated otherwise; `stream` arguments are hipStream_t passed as void*
 * (NULL = the library's own stream).
 */
#ifndef GA_AMD_H
#define GA_AMD_H

#include <stddef.h>

#if defined(__cplusplus)
extern "C" {
#endif

#define GAAMD_OP_COPY 0

/* ---- 1. bootstrap ------------------------------------------------------ */
typedef int (*gaamd_allgather_fn)(const void *send, void *recv, size_t bytes, void *ctx);
typedef int (*gaamd_barrier_fn)(void *ctx);
int gaamd_set_bootstrap(int rank, int size, int local_rank,
                        gaamd_allgather_fn allgather, gaamd_barrier_fn barrier, void *ctx);
#ifdef MPI_VERSION
/* hooks over an MPI communicator (the bootstrap half of comex_init_comm, no GPU) */
int gaamd_set_bootstrap_comm(MPI_Comm comm);
#endif
/* exercise the bootstrap alone (no GPU): allgather of ranks + barriers */
int gaamd_bootstrap_selftest(int rounds);
int gaamd_rank(void);
int gaamd_size(void);
/* HIP device of this rank after comex_init (COMEX_AMD_DEVICE or local rank mod devices) */
int gaamd_device(void);
/* after comex_init: ranks (this one included) whose HIP device is this rank's physical
   GPU (PCI bus id), distinct GPUs among the ranks of this node, and the peer-load mode
   (COMEX_AMD_PEER_LOADS: 0 auto -- peers on other GPUs read with system-scope loads,
   1 all -- every peer treated as another GPU, 2 off).  Lets a caller say whether its
   remote traffic crossed xGMI. */
int gaamd_device_topology(int *ranks_on_gpu, int *gpus_on_node, int *peer_loads);
/* nodes: ranks sharing a host (or the same COMEX_AMD_NODE value) map each other's
   HBM; ranks on different nodes exchange the MPI-PR messages over TCP (wire.cpp).
   After bootstrap: this rank's node index, the node count, ranks on this node. */
int gaamd_node_info(int *node, int *nnodes, int *node_size);
/* exercise the cross-node transport alone (no GPU): PING frames between all ranks */
int gaamd_wire_selftest(int rounds);

/* ---- 2. kernels -------------------------------------------------------- */
int gaamd_strided(int op, const void *scale, const void *src, const int *src_stride,
                  void *dst, const int *dst_stride, const int *count, int stride_levels,
                  void *stream);
long gaamd_packed_size(const int *count, int stride_levels);
int gaamd_pack(const void *src, const int *src_stride, const int *count, int stride_levels,
               void *packed, void *stream);
int gaamd_unpack(const void *packed, void *dst, const int *dst_stride, const int *count,
                 int stride_levels, void *stream);
int gaamd_unpack_acc(int op, const void *scale, const void *packed, void *dst,
                     const int *dst_stride, const int *count, int stride_levels, void *stream);
/* The launch plan of a strided operation without launching anything (no GPU
 * needed): plan[0..7] = {kind (1 rows, 2 flat, 3 serial, 4 ordered), vector width, unroll
 * (for kind 4: 0 one workgroup, 1 column slices with src prefetch, 2 column slices in
 * place), threads per block, launches, blocks, stride levels after merging, chunk grid
 * aligned}; row_end = ~0 for all rows.  Returns 0 or the launcher's error code. */
int gaamd_plan_strided(int op, const void *src, const int *src_stride, const void *dst, const int *dst_stride,
                       const int *count, int stride_levels, unsigned long long row_begin,
                       unsigned long long row_end, long long plan[8]);
/* kind / vector width / unroll / launches / blocks of the last kernel-level call */
int gaamd_last_launch(int *kind, int *width, int *unroll, int *launches,
                      unsigned long long *blocks);
/* kernel launches since start, by kind: counts[0..4] = {unused, rows, flat,
 * serial, ordered}, every caller of this process (user calls, progress thread, wire) */
int gaamd_kernel_counts(unsigned long long counts[5]);
/* requests this rank posted to same-node owners, by route: counts[0..3] =
 * {packed chunks (pack -> staging -> owner unpack), direct-source (owner reads
 * our segment), io-vector, rmw} */
int gaamd_route_counts(unsigned long long counts[4]);
/* Operations that took the reference's route toggles beyond SELF/SMP, since init:
 * [0] strided operations split row by row (COMEX_ENABLE_{ACC,PUT,GET}_PACKED=0),
 * [1] io-vector descriptors split pair by pair (COMEX_ENABLE_{ACC,PUT,GET}_IOV=0),
 * [2] gets through the owner (COMEX_ENABLE_GET_SELF/SMP=0). */
int gaamd_toggle_counts(unsigned long long counts[3]);
/* Local io-vector launches whose destinations may repeat (>= 2048 pairs, or fewer
 * with a repeat), by path: [0] hashed (only pairs sharing a destination sorted, in
 * LDS), [1] hashed, then the radix path for the pairs it could not order (more than
 * 8192 such pairs), [2] the radix path (above the other paths' range, or for the
 * partitions [3] deferred), [3] ordered in LDS: one workgroup below 1 Ki pairs, hash
 * partitions up to 4 Mi pairs (tuning iov_lds=0 routes to [0]-[2] instead). */
int gaamd_iov_path_counts(unsigned long long counts[4]);
/* runs fn(t, ctx) for t = 0 .. T-1 (1 <= T <= 16) on the library's persistent host worker
 * pool, t = 0 on the calling thread, and returns when all have; -1 on bad arguments.
 * One job at a time (concurrent callers wait); fn must not call back into this function. */
int gaamd_host_parallel(int T, void (*fn)(int t, void *ctx), void *ctx);
/* one-pass accumulates this rank applied into the segment of a rank on the same GPU */
unsigned long long gaamd_one_pass_count(void);
/* comex_malloc calls served by a freed segment block kept for reuse (with its IPC export) */
unsigned long long gaamd_segment_cache_reuse(void);
/* segments this rank replaced because a peer's fresh IPC mapping did not read their tags */
unsigned long long gaamd_segment_remaps(void);
/* times the freed-segment cache was given back under device-memory pressure */
unsigned long long gaamd_segment_cache_trims(void);
/* the kind of this rank's segment holding p: 0 none, 1 HBM, 2 host (node shm,
   COMEX_AMD_SEGMENT=host: the host may read and write it directly) */
int gaamd_segment_kind(const void *p);
/* vmm segment allocator: hipMemSetAccess refusals retried at a fresh range (diagnostic) */
unsigned long long gaamd_vmm_access_retries(void);
/* CPU self-test of the vmm allocator's descriptor exchange over the bootstrap (no GPU):
   wrong or missing descriptors, 0 = pass */
int gaamd_vmm_exchange_selftest(int rounds);
/* same-node peers whose staging buffer this rank could not map by IPC at
 * comex_init (remote accumulates to or from them would abort); -1 before init */
int gaamd_peers_unmapped(void);
/* requests this rank's progress thread applied, by kind: packed, io-vector, rmw, direct-source */
int gaamd_owner_counts(unsigned long long counts[4]);
/* keys: "kind" (0 auto, 1 rows, 2 flat, 3 serial, 4 ordered), "block" (0 auto/64/128),
 * "flat_max_nvec", "align", "flat_line_min", "ordered_cols" (column-sliced ordered
 * kernel), "streams", "iov_lds" (1: io-vectors with repeated destinations ordered in
 * LDS up to 4 Mi pairs; 0: the hashed / radix paths); returns the previous value or -1 */
int gaamd_set_tuning(const char *key, int value);
int gaamd_get_tuning(const char *key);

/* ---- 3. device plumbing ------------------------------------------------ */
int gaamd_device_count(void);
int gaamd_set_device(int dev);
void *gaamd_stream(void);
/* library stream i (0 = gaamd_stream()), or NULL past gaamd_num_streams() */
void *gaamd_stream_at(int i);
void *gaamd_dev_malloc(size_t bytes);
int gaamd_dev_free(void *p);
void *gaamd_host_malloc(size_t bytes);   /* pinned, device-mapped */
int gaamd_host_free(void *p);
int gaamd_memcpy(void *dst, const void *src, size_t bytes);   /* any direction, synchronous */
/* a 2-D patch, any direction, synchronous: `height` rows of `width` bytes, rows
 * `spitch` / `dpitch` bytes apart (hipMemcpy2D) */
int gaamd_memcpy2d(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width, size_t height);
int gaamd_memset(void *dst, int value, size_t bytes);
int gaamd_sync(void *stream);          /* NULL: all library streams */
/* order the primary stream (gaamd_stream()) after everything enqueued on the
 * library's other streams, and them after it (COMEX_AMD_STREAMS > 1) */
int gaamd_join(void);
int gaamd_num_streams(void);
/* synthetic inputs of SURVEY.md 8(d) generated on the device; type:
 * 0 f64, 1 f32, 2 i32, 3 i64 ; n elements from splitmix64(seed) */
int gaamd_fill(void *dst, long n, int type, unsigned long long seed, void *stream);
/* n 8-byte words of one bit pattern (8-byte aligned dst) */
int gaamd_fill_word(void *dst, long n, unsigned long long word, void *stream);
void *gaamd_stream_create(void);       /* an extra blocking HIP stream */
int gaamd_stream_destroy(void *stream);
/* HIP events on the library stream (or `stream`) */
void *gaamd_event_create(void);
int gaamd_event_destroy(void *ev);
int gaamd_event_record(void *ev, void *stream);
int gaamd_event_sync(void *ev);
float gaamd_event_elapsed_ms(void *start, void *stop);
const char *gaamd_version(void);
/* path of the HIP runtime (libamdhip64) this library's calls resolve to */
const char *gaamd_hip_runtime(void);
/* build provenance: sha256 (hex) of the sources this library was compiled from --
 * ga_amd/csrc/ and include/ (ga_amd/provenance.py) -- so a stale prebuilt library is
 * detectable against the tree beside it */
const char *gaamd_build_id(void);

/* ---- test and diagnostic hooks (not used by GA) ------------
 * One entry point; returns 0, or -1 for an unknown key.
 *   "stamps"        host stamps (CLOCK_BOOTTIME ns) of the last strided call and
 *                   the last comex_wait_all: [0] call entry, [1] route decided
 *                   (launch lock held), [2] stream picked, [3] kernel launched,
 *                   [4] call return, [5] wait entry, [6] streams about to be
 *                   synchronised, [7] synchronised.  out (nout >= 8, may be NULL)
 *                   receives them; value 1 clears them and starts stamping, 0
 *                   stops, -1 leaves it.
 *   "stale_gen"     N > 0: every peer treats its first mapping of each rank's N-th
 *                   allocation as stale, so the replace-and-repeat path of
 *                   comex_malloc runs on demand (0: off).
 *   "stale_granule" G >= 0 (with stale_gen): instead, each owner writes a foreign
 *                   tag into granule G (G * 2 MiB bytes in) of its N-th allocation
 *                   on the first exchange, and the peers' check must find it
 *                   (-1: off).
 *   "iov_host_sides" out[0] (nout >= 1): io-vector sides found wholly in pageable
 *                   host memory by one /proc/self/maps pass (value ignored).
 *   "host_range"    that pass on its own: out[0], out[1] (nout >= 2) hold [lo, hi) on
 *                   entry, value 1 asks for writable memory; out[0] is 1 when every
 *                   byte lies in readable (writable) mappings that are not device
 *                   files, else 0.  Needs no GPU.
 *   "pinned_threads" out[0] (nout >= 1): threads that hold pinned bounce buffers or
 *                   a non-blocking ring now (a thread's are freed when it ends, every
 *                   thread's at comex_finalize).
 *   "publish"       1: the conservative publication mode -- every direct-source
 *                   post, every packed-chunk post and every fence first records a
 *                   system-scope release (hipEventReleaseToSystem) on each library
 *                   stream and waits for them (the markers round 5 measured and took
 *                   out of the default path); 0: the default; -1 leaves it.  out[0]
 *                   (nout >= 1) receives the previous setting.  Used to classify a
 *                   cross-GPU mismatch as visibility (clears) or logic (persists).
 *   "drop_chunk"    N > 0: the owner's progress thread counts every N-th packed chunk
 *                   applied without running its kernel (a test hook: a logic fault);
 *                   0: off.
 *   "peer_gets"     out[0] (nout >= 1): strided gets this rank read from another GPU's
 *                   memory with system-scope loads.
 *   "vmm_window"    out[0], out[1] (nout >= 2): bytes of the vmm allocator's private
 *                   address window taken so far and bytes left.  Every mapping (this
 *                   rank's blocks and its imports of peers' blocks) takes
 *                   round_up(bytes, 2 MiB) + 2 MiB of it, never handed out again;
 *                   comex_malloc aborts with a message once it is used up. */
int gaamd_diag(const char *key, long long value, unsigned long long *out, int nout);

#if defined(__cplusplus)
}
#endif

#endif /* GA_AMD_H */
