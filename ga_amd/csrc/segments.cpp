// segments.cpp -- comex_malloc / comex_free: the memory a GA partition lives in.
//
// Reference: comex/src-mpi-pr/comex.c comex_malloc (2359-2605): _comex_malloc_local
// shm_open + mmap (1465-1524), the reg_entry_t MPI_Allgather (2461), every same-node
// segment _shm_attach'ed into the reg cache (2497-2552, reg_cache.c).  Here a
// segment is HBM of the owner's GPU (hipMalloc), exported by IPC and mapped by
// every same-node rank (hipIpcOpenMemHandle), or -- COMEX_AMD_SEGMENT=host /
// comex_malloc_mem_dev(..., "host") -- host memory (see do_malloc).  The IPC
// address history, the tag check of fresh mappings and the freed-segment cache
// answer the runtime's export refusals and stale mappings.
#include "comex_impl.hpp"
#include "../../include/ga_amd.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <errno.h>
#include <fcntl.h>
#include <time.h>
#include <sys/mman.h>
#include <deque>
#include <mutex>
#include <algorithm>

namespace gaamd {

bool find_segment_local(const void *p, int64_t lo, int64_t hi) {
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

void check_remote(int owner, const void *p, int64_t lo, int64_t hi) {
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
uint64_t seg_tag(int rank, uint64_t gen, int end) {
    return 0x67614d4453454700ull ^ ((uint64_t)rank << 40) ^ (gen << 1) ^ (uint64_t)end;
}

static std::vector<void *> g_quarantine;   // blocks whose IPC export was refused (freed at finalize)

void addr_history(const void *p, size_t bytes) {
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

void ipc_close(void *mapped, int peer) {
    if (!mapped) return;
    addr_event('c', mapped, mapped_size(mapped), peer);
    GA_HIP(hipIpcCloseMemHandle(mapped));
}

// Map a same-node peer's HBM (IPC handle).  A failure is not fatal here: a job
// that never touches that peer's memory (owner-aligned accumulates, the weak-
// scaling bench) runs on; the first operation that needs the mapping aborts with
// this diagnosis (remote_view / the progress thread).
void *ipc_open(hipIpcMemHandle_t h, int q, const char *what) {
    void *p = nullptr;
    trace(2, "hipIpcOpenMemHandle of rank %d's %s", q, what);
    const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
    trace(2, "hipIpcOpenMemHandle -> %d (%p)", (int)e, p);
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

// address of rank `owner`'s byte `p` (owner's address space) in this process
char *remote_view(int owner, const void *p, int64_t lo, int64_t hi) {
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

// [p+lo, p+hi) inside one of our HBM segments that rank t mapped at comex_malloc
bool src_segment_shared(const void *p, int64_t lo, int64_t hi, int t) {
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

// d meets one of our HBM segments (which same-GPU ranks may write: one-pass route)
bool in_own_segment(const Span &d) {
    Runtime &r = rt();
    std::lock_guard<std::mutex> g(r.seg_mu);
    for (const Segment &s : r.segs) {
        if (!s.live || !s.device || s.peer.empty()) continue;
        const PeerMap &m = s.peer[r.rank];
        if (m.bytes && d.lo < (int64_t)(m.base + m.bytes) && (int64_t)m.base < d.hi) return true;
    }
    return false;
}

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

void export_alloc(void **p, size_t bytes, hipIpcMemHandle_t *h, const char *what) {
    Runtime &r = rt();
    constexpr bool retry = true;   // the former COMEX_AMD_IPC_RETRY knob (its 0 only aborted sooner)
    std::vector<void *> held;
    trace(2, "hipIpcGetMemHandle of a %zu-byte %s at %p", bytes, what, *p);
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
// their IPC export, instead of going back to hipFree.  GA creates and destroys
// arrays of the same shapes over and over; every hipFree + hipMalloc + export cycle
// recycles addresses and descriptors, and the runtime refuses, now and then, to
// export a fresh block at a recycled address (profiles/r03/s19, s20, s27-s29: 1-4
// refusals in most runs of eight ranks on one GPU).  A cached block is exported
// once, for good, and a reused one is opened again by the peers from the same
// handle.  The cache must not starve other allocators: its default cap
// is an eighth of the device's memory shared among the ranks on that GPU (at most
// 16 GiB; COMEX_AMD_SEGMENT_CACHE_MB overrides, 0 disables), and it is given back
// -- by every rank of the GPU, each seeing the device's free memory -- whenever a
// new segment would leave less than COMEX_AMD_SEGMENT_FREE_MIN_MB free (default
// 1/16 of the device), before a freed block would be cached below that watermark,
// and when any allocation of this library fails.
struct CachedBlock {
    void *p;
    size_t bytes;
    bool exported;
    hipIpcMemHandle_t h;
    bool vmm = false;   // a block of the vmm allocator: kept with its handle, mapping and descriptor
    VmmBlock vb;
};
static std::deque<CachedBlock> g_blocks;   // oldest first
static size_t g_blocks_bytes = 0;
static std::atomic<unsigned long long> g_block_reuse{0};
static std::atomic<unsigned long long> g_remapped{0};   // segments replaced after a stale peer mapping
static std::atomic<unsigned long long> g_cache_trims{0};   // cache given back under memory pressure

static size_t device_total() {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return tot;
}

static size_t device_free() {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return fr;
}

static int ranks_on_this_gpu() {
    int n = 0;
    for (uint8_t d : rt().same_dev) n += d ? 1 : 0;
    return n > 0 ? n : 1;
}

static size_t block_cache_cap() {
    static const size_t v = [] {
        if (const char *e = getenv("COMEX_AMD_SEGMENT_CACHE_MB")) return (size_t)atof(e) << 20;
        const size_t share = device_total() / 8 / (size_t)ranks_on_this_gpu();
        return std::min<size_t>(share, 16ull << 30);
    }();
    return v;
}

static size_t free_watermark() {
    static const size_t v = device_total() / 16;   // the former COMEX_AMD_SEGMENT_FREE_MIN_MB
    return v;
}

static void block_free_one(const CachedBlock &b) {
    if (b.vmm) {
        VmmBlock v = b.vb;
        vmm_free(&v);
        return;
    }
    addr_event('f', b.p, b.bytes, -1);
    GA_HIP(hipFree(b.p));
}

static void block_flush() {
    for (const CachedBlock &b : g_blocks) block_free_one(b);
    g_blocks.clear();
    g_blocks_bytes = 0;
}

static void block_put(const CachedBlock &nb) {
    const size_t bytes = nb.bytes, cap = block_cache_cap();
    if (bytes > cap || device_free() < free_watermark()) {
        // too big to keep, or the device is short of memory: give it back now
        block_free_one(nb);
        if (!g_blocks.empty() && device_free() < free_watermark()) {
            g_cache_trims.fetch_add(1, std::memory_order_relaxed);
            block_flush();
        }
        return;
    }
    while (g_blocks_bytes + bytes > cap && !g_blocks.empty()) {
        block_free_one(g_blocks.front());
        g_blocks_bytes -= g_blocks.front().bytes;
        g_blocks.pop_front();
    }
    g_blocks.push_back(nb);
    g_blocks_bytes += bytes;
}

static void block_put(void *p, size_t bytes, bool exported, const hipIpcMemHandle_t &h) {
    CachedBlock b;
    b.p = p;
    b.bytes = bytes;
    b.exported = exported;
    b.h = h;
    block_put(b);
}

// a cached block of exactly `bytes`; its export in *h when it has one
static bool block_take(size_t bytes, void **p, bool *exported, hipIpcMemHandle_t *h) {
    for (auto it = g_blocks.begin(); it != g_blocks.end(); ++it) {
        if (it->bytes != bytes || it->vmm) continue;
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

// the vmm allocator's counterpart: a cached block of exactly `bytes`, with its handle,
// mapping and descriptor (a reused block is a known-good one: the runtime defect of
// vmm.cpp strikes new blocks, so GA's create/destroy cycles then create none)
static bool block_take_vmm(size_t bytes, VmmBlock *v) {
    for (auto it = g_blocks.begin(); it != g_blocks.end(); ++it) {
        if (it->bytes != bytes || !it->vmm) continue;
        *v = it->vb;
        g_blocks_bytes -= bytes;
        g_blocks.erase(it);
        g_block_reuse.fetch_add(1, std::memory_order_relaxed);
        addr_event('r', v->va, bytes, -1);
        return true;
    }
    return false;
}

// Before a new device segment of `bytes` per rank: every rank of this GPU makes
// the same call at the same point of the collective comex_malloc and sees the
// same device-wide free memory, so when the GPU's ranks together would drop below
// the watermark each one gives its cache back -- another rank's allocation (or the
// application's) is not refused for memory this library only keeps for reuse.
static void block_trim_for(size_t bytes) {
    if (g_blocks.empty()) return;
    const size_t need = bytes * (size_t)ranks_on_this_gpu() + free_watermark();
    if (device_free() < need) {
        g_cache_trims.fetch_add(1, std::memory_order_relaxed);
        block_flush();
    }
}

// hipMalloc, giving the cached blocks back first when the device is full
static void *device_alloc(size_t bytes) {
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipErrorOutOfMemory && !g_blocks.empty()) {
        (void)hipGetLastError();
        g_cache_trims.fetch_add(1, std::memory_order_relaxed);
        block_flush();
        e = hipMalloc(&p, bytes);
    }
    if (e != hipSuccess) fatal("hipMalloc of %zu bytes failed: %s", bytes, hipGetErrorString(e));
    return p;
}

// ---- IPC handle table ------------------------------------
// Every IPC handle this process exported or was handed (a segment's, a staging
// buffer's): whose, which allocation (the tag number), the owner's base and size,
// and the handle's 64 bytes.  A mapping that fails its tag check is reported with
// its handle and every earlier handle with the same bytes, and with the handle of
// the allocation its tags say it reached -- which earlier export, and whose, it
// really resolved to.
struct HandleSeen {
    int rank;
    uint64_t gen, base, bytes;
    hipIpcMemHandle_t h;
};
static std::mutex g_hs_mu;
static std::deque<HandleSeen> g_handles;   // newest last, at most 4096

static uint64_t handle_hash(const hipIpcMemHandle_t &h) {
    uint64_t x = 1469598103934665603ull;
    const unsigned char *b = reinterpret_cast<const unsigned char *>(&h);
    for (size_t i = 0; i < sizeof(h); ++i) x = (x ^ b[i]) * 1099511628211ull;
    return x;
}

void handle_seen(int rank, uint64_t gen, uint64_t base, uint64_t bytes, const hipIpcMemHandle_t &h) {
    std::lock_guard<std::mutex> g(g_hs_mu);
    g_handles.push_back({rank, gen, base, bytes, h});
    if (g_handles.size() > 4096) g_handles.pop_front();
}

static void print_handle(const char *what, const hipIpcMemHandle_t &h) {
    const uint64_t *w = reinterpret_cast<const uint64_t *>(&h);
    fprintf(stderr, "[ga_amd %d]     %s (hash %016llx):", rt().rank, what, (unsigned long long)handle_hash(h));
    for (size_t i = 0; i < sizeof(h) / 8; ++i) fprintf(stderr, " %016llx", (unsigned long long)w[i]);
    fprintf(stderr, "\n");
}

// a stale mapping of rank q's segment (its handle h, allocation gen) read `tag`
static void report_stale(int q, uint64_t gen, uint64_t base, uint64_t bytes, const hipIpcMemHandle_t &h,
                         uint64_t tag) {
    std::lock_guard<std::mutex> g(g_hs_mu);
    const uint64_t x = tag ^ seg_tag(0, 0, 0);
    const int trank = (int)(x >> 40);
    const uint64_t tgen = (x & ((1ull << 40) - 1)) >> 1;
    const bool is_tag = (x >> 40) < (uint64_t)kMaxRanks * 64 && !(x & 1);
    fprintf(stderr, "[ga_amd %d]   stale mapping of rank %d's allocation %llu (base %#llx, %llu B): it reads ",
            rt().rank, q, (unsigned long long)gen, (unsigned long long)base, (unsigned long long)bytes);
    if (is_tag) fprintf(stderr, "the tag of rank %d's allocation %llu\n", trank, (unsigned long long)tgen);
    else fprintf(stderr, "no tag (%#llx)\n", (unsigned long long)tag);
    print_handle("handle opened", h);
    const uint64_t hh = handle_hash(h);
    int same = 0;
    for (const HandleSeen &e : g_handles) {
        if (handle_hash(e.h) == hh && !(e.rank == q && e.gen == gen)) {
            fprintf(stderr, "[ga_amd %d]     equal to the handle rank %d sent for its allocation %llu (base %#llx, "
                    "%llu B)\n", rt().rank, e.rank, (unsigned long long)e.gen, (unsigned long long)e.base,
                    (unsigned long long)e.bytes);
            ++same;
        }
        if (is_tag && e.rank == trank && e.gen == tgen) print_handle("handle of the allocation it reached", e.h);
    }
    if (!same) fprintf(stderr, "[ga_amd %d]     no earlier handle has the same bytes\n", rt().rank);
}

// ---- host segments in node shared memory ----------------
// COMEX_AMD_SEGMENT=host / comex_malloc_mem_dev(..., "host"): the reference's own
// segment kind -- a POSIX shm object per rank, mmap'ed by every rank of the node
// (_comex_malloc_local / _shm_attach, comex.c:1465-1524, 4968-5290) -- registered
// with HIP in every process that maps it, so kernels on any of the node's GPUs reach
// it through a device pointer and the host can touch it directly: GA's host-side
// local operations (pnga_access_ptr + memset in pnga_zero, global.nalg.c:94-129)
// work on it.  Registered host memory is fine-grained (PCIe / system memory), so it
// needs no cache maintenance between a host write and a peer's kernel.
static size_t page_round(size_t n) { return (n + (size_t)kPage - 1) & ~(size_t)(kPage - 1); }

static char *shm_map_registered(const char *name, size_t map_bytes, bool create) {
    const int fd = shm_open(name, O_RDWR | (create ? (O_CREAT | O_EXCL) : 0), 0600);
    if (fd < 0) fatal("host segment: shm_open(%s) failed: %s", name, strerror(errno));
    if (create && ftruncate(fd, (off_t)map_bytes) != 0) fatal("host segment: ftruncate(%s) failed", name);
    void *p = mmap(nullptr, map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) fatal("host segment: mmap(%s, %zu) failed: %s", name, map_bytes, strerror(errno));
    GA_HIP(hipHostRegister(p, map_bytes, hipHostRegisterMapped));
    void *d = nullptr;
    GA_HIP(hipHostGetDevicePointer(&d, p, 0));
    // every address computation of the library (a rank's own segment addresses,
    // the owner addresses in requests) assumes the device view of this process's
    // mapping is the mapping itself, as it is for registered memory on this runtime
    if (d != p) fatal("host segment: the device view %p of registered memory differs from its address %p", d, p);
    return (char *)p;
}

static void shm_unmap_registered(char *p, size_t map_bytes) {
    if (!p) return;
    (void)hipHostUnregister(p);
    munmap(p, map_bytes);
}

// Every segment gets a per-rank, per-allocation tag at the start of every 2 MiB
// granule and in its last 8 bytes (k_seg_tags) before its handle goes out, and every
// peer checks all of them through its fresh mapping in one kernel (k_seg_check,
// system-scope loads).  Eight ranks on one GPU (profiles/r03/s32), with freed blocks
// going back to the runtime: in 2 of 30 runs, after the runtime had refused an export
// and a new block was exported instead, EVERY peer's mapping of that rank's new block
// reached other memory -- the block later read only its owner's own contribution,
// nobody else's, with no error anywhere -- and tools/vmm_probe.hip reproduced such a
// binding without this library (profiles/r04/s08).  A block is mapped granule by
// granule, so the tags cover every granule, not only the two ends.
// A mapping that does not read them all is closed, the owner's block set aside
// (quarantined) and replaced, and the exchange repeated (all ranks, collectively), up
// to 4 times.  Test hooks (gaamd_diag "stale_gen" / "stale_granule"): every peer
// treats its first mapping of each rank's N-th allocation as stale, or the owner
// writes a foreign tag into granule G of it so that the check must find it.
std::atomic<long long> g_diag_stale_gen{0}, g_diag_stale_granule{-1};

// the tag key of a rank's allocation (granule 0's tag) and its end tag
static uint64_t tag_key(int rank, uint64_t gen) { return seg_tag(rank, gen, 0); }
static uint64_t tag_end(int rank, uint64_t gen) { return seg_tag(rank, gen, 1); }

static double now_us() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return 1e6 * (double)t.tv_sec + 1e-3 * (double)t.tv_nsec;
}

// the owner: every tag of its new block (null stream, waited for before the descriptor
// or handle goes out); the test hook's foreign tag on the first exchange
static void write_tags(void *p, size_t bytes, int rank, uint64_t gen, int attempt) {
    const double t0 = now_us();
    int rc = launch_seg_tags(p, bytes, tag_key(rank, gen), tag_end(rank, gen), nullptr);
    if (rc) fatal("segment tag kernel failed (%d)", rc);
    const long long sg = g_diag_stale_granule.load(), sn = g_diag_stale_gen.load();
    if (attempt == 0 && sn > 0 && (uint64_t)sn == gen && sg >= 0) {
        const uint64_t ngran = seg_granule_count(bytes);
        const uint64_t g = (uint64_t)sg % ngran;
        const uint64_t foreign = seg_granule_tag(tag_key(rank, gen + 1000), (uint32_t)g);
        GA_HIP(hipStreamSynchronize(nullptr));
        GA_HIP(hipMemcpy((char *)p + g * kSegGranule, &foreign, 8, hipMemcpyHostToDevice));
        fprintf(stderr, "[ga_amd %d] gaamd_diag stale_granule: allocation %llu's granule %llu carries a foreign tag\n",
                rt().rank, (unsigned long long)gen, (unsigned long long)g);
    }
    GA_HIP(hipStreamSynchronize(nullptr));
    trace(1, "comex_malloc: tags of %zu bytes (%llu granules) written in %.1f us", bytes,
          (unsigned long long)seg_granule_count(bytes), now_us() - t0);
}

static int do_malloc(void **ptr_arr, size_t bytes, comex_group_t group, bool device) {
    ensure_init();
    Runtime &r = rt();
    // collective over the group's members (comex.c comex_malloc): ptr_arr is
    // indexed by group rank; non-members keep no view of the segment
    const std::vector<int> members = group_members(group);
    const bool tr = r.debug >= 2;
    if (tr) fprintf(stderr, "[ga_amd %d] comex_malloc(%zu, group %d): enter\n", r.rank, bytes, group);
    struct Info {
        uint64_t base, bytes;
        hipIpcMemHandle_t h;
        int32_t device, host;    // host: a node shm segment, `name` below
        uint64_t gen;
        char name[64];
        int32_t vmm, pid, fd, pad;   // vmm: HBM from vmm.cpp; pid: the process its descriptor comes from
        uint64_t vmm_bytes;
    } mine;
    memset(&mine, 0, sizeof(mine));
    static uint64_t gen = 0;   // this rank's allocation counter (the tags, the shm names)
    void *p = nullptr;
    bool exported = false;
    const size_t map_bytes = page_round(bytes);
    const bool vmm = device && vmm_enabled();
    VmmBlock vlocal;
    if (vmm) vmm_listen();
    mine.pid = (int32_t)getpid();
    if (bytes) {
        if (vmm) {
            block_trim_for(bytes);
            p = block_take_vmm(bytes, &vlocal) ? vlocal.va : vmm_alloc(bytes, &vlocal);
            mine.vmm = 1;
            mine.fd = vlocal.fd;
            mine.vmm_bytes = vlocal.bytes;
        } else if (device) {
            block_trim_for(bytes);
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
            const char *job = getenv("COMEX_AMD_JOBID");
            snprintf(mine.name, sizeof(mine.name), "/gaamd_seg_%d_%d_%s_%d_%llu", (int)getuid(), (int)getpid(),
                     job ? job : "0", r.rank, (unsigned long long)(gen + 1));
            p = shm_map_registered(mine.name, map_bytes, true);
            mine.host = 1;
        }
    }
    const bool tagged = device && bytes >= 16;
    std::vector<Info> all(r.size);
    std::vector<void *> mapped(r.size, nullptr);
    std::vector<VmmBlock> vpeer;
    for (int attempt = 0;; ++attempt) {
        mine.base = (uint64_t)(uintptr_t)p;
        mine.bytes = bytes;
        mine.device = r.device;
        mine.gen = ++gen;
        if (tagged) {
            trace(2, "comex_malloc: writing the tags of %p", p);
            write_tags(p, bytes, r.rank, mine.gen, attempt);
        }
        if (tr) fprintf(stderr, "[ga_amd %d] comex_malloc: allocated %p, allgather\n", r.rank, p);
        std::vector<Info> gathered(members.size());
        members_allgather(members, group, &mine, gathered.data(), sizeof(Info));
        if (tr) fprintf(stderr, "[ga_amd %d] comex_malloc: allgather done, opening peers\n", r.rank);
        memset(all.data(), 0, sizeof(Info) * all.size());
        for (size_t k = 0; k < members.size(); ++k) {
            all[members[k]] = gathered[k];
            ptr_arr[k] = (void *)(uintptr_t)gathered[k].base;
            if (gathered[k].bytes && !gathered[k].host && !gathered[k].vmm)
                handle_seen(members[k], gathered[k].gen, gathered[k].base, gathered[k].bytes, gathered[k].h);
        }
        // vmm: each member's descriptor passed to the other members on this node
        std::vector<int> vfd(r.size, -1);
        if (vmm) {
            std::vector<int> to;
            std::vector<std::pair<int, uint64_t>> from;
            std::vector<int> from_rank;
            for (int q : members) {
                if (q == r.rank || !r.same_node(q)) continue;
                if (mine.vmm) to.push_back(all[q].pid);   // zero-byte members map it too
                if (all[q].vmm && all[q].bytes) {
                    from.push_back({q, all[q].gen});
                    from_rank.push_back(q);
                }
            }
            std::vector<int> got(from.size(), -1);
            vmm_exchange(vlocal.fd, r.rank, mine.gen, to, from, got.data());
            for (size_t k = 0; k < from.size(); ++k) vfd[from_rank[k]] = got[k];
        }
        // open, and check that each mapping reads every one of its owner's tags
        std::vector<uint8_t> stale(r.size, 0);
        std::vector<int> checked;   // peers whose tags the check kernel reads
        for (int q = 0; q < r.size; ++q) {
            mapped[q] = nullptr;
            if (q == r.rank || !all[q].bytes || !r.same_node(q)) continue;
            if (all[q].host) {   // a host segment: map the owner's shm object
                all[q].name[sizeof(all[q].name) - 1] = 0;
                mapped[q] = shm_map_registered(all[q].name, page_round(all[q].bytes), false);
                continue;
            }
            if (all[q].vmm) {    // the owner's dmabuf descriptor, mapped at a fresh address here
                if (vpeer.size() != (size_t)r.size) vpeer.assign(r.size, VmmBlock());
                mapped[q] = vmm_import(vfd[q], all[q].vmm_bytes, q, &vpeer[q]);
                if (!mapped[q]) {
                    // the runtime refused this GPU access to the imported block (vmm.cpp): a
                    // broken binding like a stale one -- the owner replaces the block and every
                    // member repeats the exchange, instead of this rank aborting alone
                    stale[q] = 1;
                    continue;
                }
            } else {
                mapped[q] = ipc_open(all[q].h, q, "segment");
            }
            if (!mapped[q] || all[q].bytes < 16) continue;
            const long long sn = g_diag_stale_gen.load();
            if (attempt == 0 && sn > 0 && all[q].gen == (uint64_t)sn && g_diag_stale_granule.load() < 0) {
                // test hook: this round's mappings of allocation N are treated as stale, so the
                // replacement path (set aside, new block, repeated exchange) runs on demand
                fprintf(stderr, "[ga_amd %d] gaamd_diag stale_gen: treating rank %d's allocation %llu as stale\n",
                        r.rank, q, (unsigned long long)all[q].gen);
                stale[q] = 1;
                continue;
            }
            checked.push_back(q);
        }
        if (!checked.empty()) {
            const double t0 = now_us();
            uint32_t *dres = nullptr;
            std::vector<uint32_t> res(2 * checked.size());
            for (size_t k = 0; k < checked.size(); ++k) {
                res[2 * k] = 0;
                res[2 * k + 1] = ~0u;
            }
            GA_HIP(hipMalloc((void **)&dres, res.size() * sizeof(uint32_t)));
            GA_HIP(hipMemcpy(dres, res.data(), res.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
            uint64_t gran = 0;
            for (size_t k = 0; k < checked.size(); ++k) {
                const int q = checked[k];
                trace(2, "comex_malloc: checking rank %d's tags through %p", q, mapped[q]);
                const int rc = launch_seg_check(mapped[q], all[q].bytes, tag_key(q, all[q].gen),
                                                tag_end(q, all[q].gen), dres + 2 * k, nullptr);
                if (rc) fatal("segment tag check kernel failed (%d)", rc);
                gran += seg_granule_count(all[q].bytes);
            }
            GA_HIP(hipMemcpy(res.data(), dres, res.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
            GA_HIP(hipFree(dres));
            trace(1, "comex_malloc: %zu peers' tags (%llu granules) checked in %.1f us", checked.size(),
                  (unsigned long long)gran, now_us() - t0);
            for (size_t k = 0; k < checked.size(); ++k) {
                if (!res[2 * k]) continue;
                const int q = checked[k];
                stale[q] = 1;
                const uint64_t ng = seg_granule_count(all[q].bytes), g = res[2 * k + 1];
                const uint64_t off = g < ng ? g * kSegGranule : seg_end_tag_off(all[q].bytes);
                uint64_t got = 0;
                GA_HIP(hipMemcpy(&got, (char *)mapped[q] + off, 8, hipMemcpyDeviceToHost));
                fprintf(stderr, "[ga_amd %d] the %s mapping of rank %d's new %zu-byte segment (%p in its space) "
                        "reads %u of its %llu tags wrong, the first at byte %llu (%s): %#llx, not %#llx -- another "
                        "allocation's memory\n", r.rank, all[q].vmm ? "vmm" : "IPC", q, (size_t)all[q].bytes,
                        (void *)(uintptr_t)all[q].base, res[2 * k], (unsigned long long)ng + 1,
                        (unsigned long long)off, g < ng ? "a granule tag" : "the end tag", (unsigned long long)got,
                        (unsigned long long)(g < ng ? seg_granule_tag(tag_key(q, all[q].gen), (uint32_t)g)
                                                    : tag_end(q, all[q].gen)));
                if (!all[q].vmm && g == 0) report_stale(q, all[q].gen, all[q].base, all[q].bytes, all[q].h, got);
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
        if (attempt >= 3) fatal("mappings of a new segment keep reaching other memory (4 attempts)");
        if (vmm) {
            // every member drops its imports of this round; the owner of a stale block sets
            // it aside and creates another (vmm.cpp: the runtime can bind a new block's
            // descriptor to another process's block), then the exchange repeats
            for (int q = 0; q < r.size; ++q)
                if (q < (int)vpeer.size() && vpeer[q].va) vmm_free(&vpeer[q]);
            if (mine_stale) {
                fprintf(stderr, "[ga_amd %d]   my new vmm block's mappings were stale; replacing it\n", r.rank);
                vmm_quarantine(&vlocal);
                p = vmm_alloc(bytes, &vlocal);
                mine.fd = vlocal.fd;
                mine.vmm_bytes = vlocal.bytes;
                g_remapped.fetch_add(1, std::memory_order_relaxed);
            }
            members_barrier(members, group);
            continue;
        }
        for (int q = 0; q < r.size; ++q)
            if (mapped[q]) ipc_close(mapped[q], q);
        if (mine_stale) {
            // set the block aside for good and export a fresh one
            fprintf(stderr, "[ga_amd %d]   my new segment's mapping was stale; its handle and address history:\n",
                    r.rank);
            print_handle("handle exported", mine.h);
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
    s.vmm = vmm;
    if (vmm) {
        s.vmm_local = vlocal;
        s.vmm_peer = vpeer;
    }
    s.local = p;
    s.local_bytes = bytes;
    s.exported = exported;
    if (exported) s.handle = mine.h;
    for (int q = 0; q < r.size; ++q) {
        s.peer[q].base = all[q].base;
        s.peer[q].bytes = all[q].bytes;
        s.peer[q].mapped = q == r.rank ? (char *)p : (char *)mapped[q];
        if (all[q].host && s.peer[q].mapped) {
            s.peer[q].host_map = s.peer[q].mapped;
            s.peer[q].map_bytes = page_round(all[q].bytes);
        }
    }
    {
        std::lock_guard<std::mutex> g(r.seg_mu);
        r.segs.push_back(std::move(s));
    }
    if (tr) fprintf(stderr, "[ga_amd %d] comex_malloc: peers mapped, barrier\n", r.rank);
    members_barrier(members, group);
    // every member has mapped the shm object: its name can go (the mappings stay)
    if (!device && bytes) shm_unlink(mine.name);
    if (tr) fprintf(stderr, "[ga_amd %d] comex_malloc: done\n", r.rank);
    return COMEX_SUCCESS;
}

// close this process's view of a segment's peer q (IPC, shm or vmm mapping)
static void close_peer(Segment &s, int q) {
    PeerMap &m = s.peer[q];
    if (m.host_map) shm_unmap_registered(m.host_map, m.map_bytes);
    else if (s.vmm && q < (int)s.vmm_peer.size() && s.vmm_peer[q].va) vmm_free(&s.vmm_peer[q]);
    else if (m.mapped) ipc_close(m.mapped, q);
    m.mapped = m.host_map = nullptr;
}

int segment_kind_of(int owner, const void *p) {
    Runtime &r = rt();
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> g(r.seg_mu);
    for (const Segment &s : r.segs) {
        if (!s.live || s.peer.empty()) continue;
        const PeerMap &m = s.peer[owner];
        if (m.bytes && a >= m.base && a < m.base + m.bytes) return s.device ? 1 : 2;
    }
    return 0;
}

int segment_kind(const void *p) { return segment_kind_of(rt().rank, p); }

// comex_finalize, after the last barrier: every live segment's mappings closed and
// its block freed, then the cached and quarantined blocks
void segments_finalize() {
    Runtime &r = rt();
    for (Segment &s : r.segs) {
        if (!s.live) continue;
        for (int q = 0; q < (int)s.peer.size(); ++q)
            if (q != r.rank) close_peer(s, q);
        if (s.vmm) vmm_free(&s.vmm_local);
        else if (s.local && s.device) {
            addr_event('f', s.local, s.peer[r.rank].bytes, -1);
            (void)hipFree(s.local);
        } else if (s.local) {
            shm_unmap_registered((char *)s.local, s.peer[r.rank].map_bytes);
        }
        s.live = false;
    }
    r.segs.clear();
}

void segments_release_blocks() {
    block_flush();
    for (void *q : g_quarantine) (void)hipFree(q);
    g_quarantine.clear();
}

void segment_cache_flush() { block_flush(); }

}  // namespace gaamd

using namespace gaamd;

extern "C" {

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
    size_t local_bytes = 0, local_map_bytes = 0;
    VmmBlock vblock;
    bool is_vmm = false;
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
                if (q != r.rank) close_peer(s, q);
            local = s.local;
            device = s.device;
            local_map_bytes = s.peer[r.rank].map_bytes;
            if (s.vmm) {
                vblock = s.vmm_local;
                s.vmm_local = VmmBlock();
                is_vmm = true;
            }
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
    if (is_vmm) {
        if (!vblock.va) {
            // this rank owns no bytes of the segment: nothing to keep or give back (a
            // zero-byte entry in the cache would never be taken nor evicted)
        } else if (block_cache_cap()) {   // kept, with its descriptor, for the next comex_malloc
            CachedBlock b;
            b.p = vblock.va;
            b.bytes = local_bytes;
            b.exported = false;
            memset(&b.h, 0, sizeof(b.h));
            b.vmm = true;
            b.vb = vblock;
            block_put(b);
        } else {
            vmm_free(&vblock);   // physical memory back now
        }
    } else if (local && device) {
        if (block_cache_cap()) block_put(local, local_bytes, exported, handle);   // kept for the next comex_malloc
        else block_free_one({local, local_bytes, exported, handle});
    } else if (local) {
        shm_unmap_registered((char *)local, local_map_bytes);
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


unsigned long long gaamd_segment_cache_reuse(void) { return g_block_reuse.load(); }
unsigned long long gaamd_segment_remaps(void) { return g_remapped.load(); }
unsigned long long gaamd_segment_cache_trims(void) { return g_cache_trims.load(); }
int gaamd_segment_kind(const void *p) { return rt().initialized ? segment_kind(p) : 0; }

}  // extern "C"
