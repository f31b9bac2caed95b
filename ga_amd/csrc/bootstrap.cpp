// bootstrap.cpp -- rank discovery, node-local shared memory, allgather and
// barrier for the runtime.
//
// Reference: comex_group_init splits workers from progress ranks with
// MPI_Comm_split by hostname (comex/src-mpi-pr/groups.c:408-588); segment
// registrations and semaphore names travel by MPI_Allgather (comex.c:2461,
// 2874) and comex_barrier ends in MPI_Barrier (comex.c:1217-1234).
//
// Here the whole job lives on one node (one rank per GPU), so the exchange is
// a POSIX shared-memory segment that every rank maps:
//   * with hooks (gaamd_set_bootstrap: torch.distributed, MPI, ...) rank 0
//     names the segment and the name travels through the hook's allgather;
//   * without hooks the name derives from the launcher (parent pid + port),
//     so every local rank of one launch opens the same segment.
// The name is unlinked right after the first barrier, so a crashed job leaves
// nothing behind in /dev/shm.
#include "runtime.hpp"
#include <stdio.h>
#include <stdlib.h>
#include <stdarg.h>
#include <string.h>
#include <unistd.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <sched.h>

#include <string>

namespace gaamd {

static Runtime g_rt;
Runtime &rt() { return g_rt; }

void fatal(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    fprintf(stderr, "[%d] ga_amd fatal: %s\n", g_rt.rank, buf);
    fflush(stderr);
    abort();
}

void trace(int level, const char *fmt, ...) {
    if (g_rt.debug < level) return;
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    fprintf(stderr, "[ga_amd %d] %s\n", g_rt.rank, buf);
    fflush(stderr);
}

size_t node_shm_bytes(int size) {
    return sizeof(NodeShm) + sizeof(Inbox) * (size_t)(size > 1 ? size - 1 : 0) + kBootSlot * (size_t)size +
           sizeof(std::atomic<uint32_t>) * (size_t)kMaxMutexes * (size_t)size;
}
Inbox *inbox_of(NodeShm *s, int rank) { return &s->inbox[rank]; }
char *boot_area(NodeShm *s, int size) {
    return reinterpret_cast<char *>(s) + sizeof(NodeShm) + sizeof(Inbox) * (size_t)(size > 1 ? size - 1 : 0);
}
std::atomic<uint32_t> *mutex_words(NodeShm *s, int size, int rank) {
    char *base = boot_area(s, size) + kBootSlot * (size_t)size;
    return reinterpret_cast<std::atomic<uint32_t> *>(base) + (size_t)kMaxMutexes * (size_t)rank;
}

static int env_int(const char *const *names, int dflt) {
    for (int i = 0; names[i]; ++i) {
        const char *v = getenv(names[i]);
        if (v && *v) return atoi(v);
    }
    return dflt;
}

static double now_s() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static double barrier_timeout() {
    const char *v = getenv("COMEX_AMD_BARRIER_TIMEOUT");
    return v ? atof(v) : 900.0;
}

// sense-reversing barrier on two shm counters
static void shm_barrier(NodeShm *s, int size) {
    const uint64_t gen = s->bar_gen.load(std::memory_order_acquire);
    if (s->bar_count.fetch_add(1, std::memory_order_acq_rel) == (uint64_t)size - 1) {
        s->bar_count.store(0, std::memory_order_relaxed);
        s->bar_gen.fetch_add(1, std::memory_order_release);
        return;
    }
    const double t0 = now_s(), tmo = barrier_timeout();
    for (unsigned spins = 0; s->bar_gen.load(std::memory_order_acquire) == gen; ++spins) {
        if (spins > 1024) {
            sched_yield();
            if ((spins & 0xffff) == 0 && now_s() - t0 > tmo) fatal("node barrier timed out after %.0f s", tmo);
        }
    }
}

static NodeShm *open_shm(const char *name, size_t bytes, bool create) {
    int fd = -1;
    const double t0 = now_s();
    for (;;) {
        fd = shm_open(name, O_RDWR | (create ? O_CREAT : 0), 0600);
        if (fd >= 0) break;
        if (create || now_s() - t0 > barrier_timeout()) fatal("shm_open(%s) failed", name);
        usleep(1000);
    }
    if (create && ftruncate(fd, (off_t)bytes) != 0) fatal("ftruncate(%s) failed", name);
    // a non-creating opener waits until the creator has sized the segment
    for (;;) {
        struct stat st;
        if (fstat(fd, &st) == 0 && (size_t)st.st_size >= bytes) break;
        if (now_s() - t0 > barrier_timeout()) fatal("shm %s never sized", name);
        usleep(1000);
    }
    void *p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) fatal("mmap(%s) failed", name);
    return reinterpret_cast<NodeShm *>(p);
}

void boot_init() {
    Runtime &r = g_rt;
    if (r.boot_ready) return;
    if (!r.hooks) {
        static const char *rank_env[] = {"RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", "PMIX_RANK", nullptr};
        static const char *size_env[] = {"WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", nullptr};
        static const char *lrank_env[] = {"LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", nullptr};
        r.rank = env_int(rank_env, 0);
        r.size = env_int(size_env, 1);
        r.local_rank = env_int(lrank_env, r.rank);
    }
    if (r.size < 1 || r.rank < 0 || r.rank >= r.size) fatal("bad rank %d / size %d", r.rank, r.size);

    r.node_of.assign(r.size, 0);
    r.node_index.assign(r.size, 0);
    r.nnodes = 1;
    r.node = 0;
    r.node_size = r.size;
    if (r.size == 1) {
        const size_t bytes = node_shm_bytes(1);
        r.shm_bytes = bytes;
        void *p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) fatal("mmap(anon) failed");
        r.shm = reinterpret_cast<NodeShm *>(p);
        r.shm->size = 1;
        r.boot_ready = true;
        return;
    }
    // nodes: ranks that share a host (MPI_Comm_split by hostname, groups.c:408-588).
    // COMEX_AMD_NODE overrides the host name (several "nodes" on one host: the
    // cross-node wire path can then be exercised on a single machine).
    const char *node_env = getenv("COMEX_AMD_NODE");
    r.node_of.assign(r.size, 0);
    r.nnodes = 1;
    if (r.hooks) {
        char key[64] = {0};
        if (node_env) snprintf(key, sizeof(key), "env:%s", node_env);
        else if (gethostname(key, sizeof(key) - 1) != 0) fatal("gethostname failed");
        std::vector<char> keys((size_t)r.size * sizeof(key));
        if (r.ag(key, keys.data(), sizeof(key), r.ctx) != 0) fatal("bootstrap allgather hook failed");
        std::vector<std::string> seen;
        for (int q = 0; q < r.size; ++q) {
            std::string k(keys.data() + (size_t)q * sizeof(key), strnlen(keys.data() + (size_t)q * sizeof(key), sizeof(key)));
            int idx = -1;
            for (int i = 0; i < (int)seen.size(); ++i) if (seen[i] == k) idx = i;
            if (idx < 0) { idx = (int)seen.size(); seen.push_back(k); }
            r.node_of[q] = idx;
        }
        r.nnodes = (int)seen.size();
    } else if (node_env) {
        fatal("COMEX_AMD_NODE needs bootstrap hooks (gaamd_set_bootstrap): the node-shm rendezvous is per host");
    }
    r.node = r.node_of[r.rank];
    // the node shm holds one inbox and one done[][] row/column per rank of the
    // node, indexed by the rank's position on its node
    int leader = -1;
    std::vector<int> seen_on(r.nnodes, 0);
    for (int q = 0; q < r.size; ++q) {
        r.node_index[q] = seen_on[r.node_of[q]]++;
        if (r.node_of[q] == r.node && leader < 0) leader = q;
    }
    r.node_size = seen_on[r.node];
    if (r.node_size > kMaxRanks) fatal("%d ranks on one node exceed %d", r.node_size, kMaxRanks);
    const size_t bytes = node_shm_bytes(r.node_size);
    r.shm_bytes = bytes;

    char name[128];
    if (r.hooks) {
        // each node's leader names its segment; the names travel by the hook
        char mine[64] = {0};
        if (r.rank == leader) {
            struct timespec ts;
            clock_gettime(CLOCK_REALTIME, &ts);
            snprintf(mine, sizeof(mine), "/gaamd_%d_%d_%ld", (int)getuid(), (int)getpid(), (long)ts.tv_nsec);
        }
        std::vector<char> all((size_t)r.size * sizeof(mine));
        if (r.ag(mine, all.data(), sizeof(mine), r.ctx) != 0) fatal("bootstrap allgather hook failed");
        memcpy(name, all.data() + (size_t)leader * sizeof(mine), sizeof(mine));
        name[63] = 0;
        if (strncmp(name, "/gaamd_", 7) != 0) fatal("bootstrap allgather hook returned a corrupt segment name");
        r.shm = open_shm(name, bytes, r.rank == leader);
        if (r.bar(r.ctx) != 0) fatal("bootstrap barrier hook failed");
    } else {
        const char *port = getenv("MASTER_PORT");
        const char *job = getenv("COMEX_AMD_JOBID");
        snprintf(name, sizeof(name), "/gaamd_%d_%d_%s_%s", (int)getuid(), (int)getppid(),
                 port ? port : "0", job ? job : "0");
        r.shm = open_shm(name, bytes, true);
    }
    r.boot_ready = true;
    shm_barrier(r.shm, r.node_size);
    if (r.rank == leader) shm_unlink(name);
    r.shm->size = r.size;
    shm_barrier(r.shm, r.node_size);
}

void boot_barrier() {
    Runtime &r = g_rt;
    if (r.size == 1) return;
    if (r.nnodes > 1) {   // across nodes: the launcher's barrier (MPI, torch.distributed)
        if (r.bar(r.ctx) != 0) fatal("bootstrap barrier hook failed");
        return;
    }
    shm_barrier(r.shm, r.size);
}

// allgather through the shm boot area, kBootSlot bytes per rank per round
// (several nodes: the launcher's allgather)
void boot_allgather(const void *send, void *recv, size_t bytes) {
    Runtime &r = g_rt;
    if (r.size == 1) {
        memcpy(recv, send, bytes);
        return;
    }
    if (r.nnodes > 1) {
        if (r.ag(send, recv, bytes, r.ctx) != 0) fatal("bootstrap allgather hook failed");
        return;
    }
    char *area = boot_area(r.shm, r.node_size);   // one node: node_size == size
    for (size_t off = 0; off < bytes || (bytes == 0 && off == 0); off += kBootSlot) {
        const size_t n = bytes - off < kBootSlot ? bytes - off : kBootSlot;
        memcpy(area + (size_t)r.rank * kBootSlot, (const char *)send + off, n);
        shm_barrier(r.shm, r.size);
        for (int q = 0; q < r.size; ++q)
            memcpy((char *)recv + (size_t)q * bytes + off, area + (size_t)q * kBootSlot, n);
        shm_barrier(r.shm, r.size);
        if (bytes == 0) break;
    }
}

void boot_finalize() {
    Runtime &r = g_rt;
    if (!r.boot_ready) return;
    if (r.shm) munmap(r.shm, r.shm_bytes);
    r.shm = nullptr;
    r.boot_ready = false;
}

}  // namespace gaamd

using namespace gaamd;

extern "C" int gaamd_set_bootstrap(int rank, int size, int local_rank, gaamd_allgather_fn allgather,
                                   gaamd_barrier_fn barrier, void *ctx) {
    Runtime &r = rt();
    if (r.initialized || r.boot_ready) return -1;
    if (size < 1 || rank < 0 || rank >= size) return -2;
    if (size > 1 && (!allgather || !barrier)) return -3;
    r.rank = rank;
    r.size = size;
    r.local_rank = local_rank < 0 ? rank : local_rank;
    r.ag = allgather;
    r.bar = barrier;
    r.ctx = ctx;
    r.hooks = true;
    return 0;
}

extern "C" int gaamd_bootstrap_selftest(int rounds) {
    Runtime &r = rt();
    boot_init();
    int bad = 0;
    for (int it = 0; it < rounds; ++it) {
        // a payload larger than one boot slot exercises the chunked path
        const size_t n = kBootSlot / sizeof(int) + 17;
        std::vector<int> mine(n), all(n * (size_t)r.size);
        for (size_t i = 0; i < n; ++i) mine[i] = r.rank * 1000003 + (int)i + it;
        boot_allgather(mine.data(), all.data(), n * sizeof(int));
        for (int q = 0; q < r.size; ++q)
            for (size_t i = 0; i < n; ++i)
                if (all[(size_t)q * n + i] != q * 1000003 + (int)i + it) ++bad;
        boot_barrier();
    }
    return bad ? -1 : 0;
}

extern "C" int gaamd_rank(void) { return rt().rank; }
extern "C" int gaamd_size(void) { return rt().size; }
extern "C" int gaamd_device(void) { return rt().device; }

extern "C" int gaamd_device_topology(int *ranks_on_gpu, int *gpus_on_node, int *peer_loads) {
    Runtime &r = rt();
    if (!r.initialized) return -1;
    int same = 0;
    for (uint8_t d : r.same_dev) same += d ? 1 : 0;
    if (ranks_on_gpu) *ranks_on_gpu = same;
    if (gpus_on_node) *gpus_on_node = r.node_gpus;
    if (peer_loads) *peer_loads = r.peer_loads;
    return 0;
}
