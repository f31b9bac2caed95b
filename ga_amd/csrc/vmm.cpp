// vmm.cpp -- HBM segments through HIP's virtual memory API.
//
// hipMalloc + hipIpcGetMemHandle / hipIpcOpenMemHandle leave two things to the
// runtime that GA's create/destroy cycles stress: the virtual addresses (a freed
// block's range comes straight back from the next hipMalloc) and the IPC handle
// bookkeeping keyed by them.  With eight ranks on one GPU the runtime now and
// then refused to export a fresh block at a recycled address, and after such a
// refusal a peer's mapping of another fresh export reached a THIRD process's
// allocation (profiles/r03/s32, s33).  This allocator takes both
// away from the runtime:
//   * physical HBM from hipMemCreate, exported as a dmabuf file descriptor
//     (hipMemExportToShareableHandle, POSIX fd);
//   * the descriptor reaches each peer process as SCM_RIGHTS ancillary data on a
//     datagram socket of the abstract namespace, one per process, named after its
//     pid (the pid and allocation number travel in the comex_malloc allgather, as
//     reg_entry_t does at comex.c:2461), and is imported there
//     (hipMemImportFromShareableHandle).  pidfd_getfd was the first carrier; it
//     needs ptrace rights over the owner, which the box's Yama policy refuses
//     between sibling ranks (EPERM, gpurun_out r04s03), so it was dropped;
//   * every mapping -- the owner's and each peer's -- goes to a virtual range this
//     library reserved for it and does not reserve again afterwards, and what a peer maps is named by the descriptor it
//     received for (owner rank, allocation number), never by an address: no runtime
//     bookkeeping keyed by recycled addresses is involved.
// COMEX_AMD_SEGMENT_ALLOC=vmm selects it (ipc: hipMalloc + hipIpc*, the round-3 path).
#include "comex_impl.hpp"
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stddef.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <time.h>
#include <unistd.h>
#include <atomic>
#include <map>
#include <mutex>
#include <vector>

namespace gaamd {

namespace {
std::mutex g_vmm_mu;
size_t g_gran = 0;

size_t granularity() {
    if (g_gran) return g_gran;
    hipMemAllocationProp prop;
    memset(&prop, 0, sizeof(prop));
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = rt().device;
    prop.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    size_t g = 0;
    GA_HIP(hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityRecommended));
    // whole 2 MiB units at least (the runtime reports 4 KiB): sizes off 2 MiB made a
    // new block's hipMemSetAccess fail now and then (invalid argument: 0x202000 and
    // 0x208000 bytes in gpurun_out r04s05 / r04s07, never a 2 MiB multiple), and 2 MiB
    // units map with large pages; the cost is < 2 MiB per segment
    g_gran = std::max<size_t>(g, 2u << 20);
    return g_gran;
}

// Each mapping gets a virtual range of its own, taken from a window of the address
// space no runtime allocation uses ([COMEX_AMD_VMM_VA_BASE, COMEX_AMD_VMM_VA_LIMIT),
// default [32 TiB, 96 TiB): below the runtime's own mappings, which sit near the top
// of the 128 TiB user space), asked for by address hint, bump-allocated, never handed
// out twice -- a range the runtime places elsewhere, or a window used up, is an error
// that names the two variables (a range it picks itself may be one handed back
// earlier, which is what read stale), and a range is not
// reserved again after its mapping is gone: it stays reserved (retired) until the
// retired total passes COMEX_AMD_VMM_RETAIN_GB (default 16384 = 16 TiB), oldest first.
// Measured (tools/vmm_probe.hip, profiles/r04/s05): two processes exchanging 2 MiB
// blocks, the importer releasing its range and reserving it again at the same
// address -- the new mapping read zeros where the owner's tags were, every round
// after the first; with ranges never reserved twice every round read right.
struct Retired { char *va; size_t bytes; };
std::vector<Retired> g_retired;
std::atomic<unsigned long long> g_access_retries{0};
size_t g_retired_bytes = 0;
uintptr_t g_window = 0;            // next hint in the private window

size_t retain_cap() {
    return (size_t)16384 << 30;   // 16 TiB (the former COMEX_AMD_VMM_RETAIN_GB knob)
}

uintptr_t g_window_end = 0, g_window_start = 0;

char *va_take(size_t bytes) {
    std::lock_guard<std::mutex> g(g_vmm_mu);
    constexpr uintptr_t kAlign = 2u << 20;
    if (!g_window) {
        const char *e = getenv("COMEX_AMD_VMM_VA_BASE");
        g_window = e ? (uintptr_t)strtoull(e, nullptr, 0) : (uintptr_t)0x200000000000ull;
        g_window = (g_window + kAlign - 1) & ~(kAlign - 1);
        g_window_start = g_window;
        const char *l = getenv("COMEX_AMD_VMM_VA_LIMIT");
        g_window_end = l ? (uintptr_t)strtoull(l, nullptr, 0) : (uintptr_t)0x600000000000ull;
    }
    // one empty 2 MiB guard after every range, so no range starts where another
    // ends (a precaution: tools/vmm_probe.hip r_adjacent found adjacent ranges fine)
    const uintptr_t step = ((bytes + kAlign - 1) & ~(kAlign - 1)) + kAlign;
    if (g_window + step > g_window_end)
        fatal("vmm: the private address window is used up (%zu more bytes at %p, window end %p): every mapping "
              "takes a range never used before, and a long job of many array creations needs a larger window -- "
              "raise COMEX_AMD_VMM_VA_LIMIT (or lower COMEX_AMD_VMM_VA_BASE), or keep freed blocks for reuse "
              "(COMEX_AMD_SEGMENT_CACHE_MB); COMEX_AMD_VMM_RETAIN_GB bounds the retired ranges still reserved",
              bytes, (void *)g_window, (void *)g_window_end);
    void *hint = (void *)g_window;
    void *base = nullptr;
    trace(2, "vmm: hipMemAddressReserve(%zu at %p)", bytes, hint);
    GA_HIP(hipMemAddressReserve(&base, bytes, granularity(), hint, 0));
    g_window += step;
    if (base != hint) {
        (void)hipMemAddressFree(base, bytes);
        fatal("vmm: the runtime placed a range at %p, not at the requested %p: the private window "
              "[COMEX_AMD_VMM_VA_BASE, COMEX_AMD_VMM_VA_LIMIT) meets other mappings, and a range the runtime "
              "chooses may be one handed back earlier (which read stale data); move the window", base, hint);
    }
    return (char *)base;
}

void va_retire(char *va, size_t bytes) {
    std::lock_guard<std::mutex> g(g_vmm_mu);
    g_retired.push_back({va, bytes});
    g_retired_bytes += bytes;
    size_t k = 0;
    while (g_retired_bytes > retain_cap() && k < g_retired.size()) {
        (void)hipMemAddressFree(g_retired[k].va, g_retired[k].bytes);
        g_retired_bytes -= g_retired[k].bytes;
        ++k;
    }
    g_retired.erase(g_retired.begin(), g_retired.begin() + k);
}

// the descriptor exchange: one datagram socket per process, abstract namespace
int g_sock = -1;
std::map<std::pair<int, uint64_t>, int> g_stash;   // (rank, allocation number) -> descriptor received early

struct FdMsg {
    int32_t rank, pad;
    uint64_t gen;
};

socklen_t sock_addr(int pid, sockaddr_un *a) {
    memset(a, 0, sizeof(*a));
    a->sun_family = AF_UNIX;
    const int n = snprintf(a->sun_path + 1, sizeof(a->sun_path) - 1, "gaamd_vmm_%d_%d", (int)getuid(), pid);
    return (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + n);
}

double now_s() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

bool send_fd(int pid, int fd, int rank, uint64_t gen) {
    sockaddr_un a;
    const socklen_t alen = sock_addr(pid, &a);
    FdMsg m{rank, 0, gen};
    iovec io{&m, sizeof(m)};
    alignas(cmsghdr) char ctl[CMSG_SPACE(sizeof(int))];
    memset(ctl, 0, sizeof(ctl));
    msghdr h;
    memset(&h, 0, sizeof(h));
    h.msg_name = &a;
    h.msg_namelen = alen;
    h.msg_iov = &io;
    h.msg_iovlen = 1;
    h.msg_control = ctl;
    h.msg_controllen = sizeof(ctl);
    cmsghdr *c = CMSG_FIRSTHDR(&h);
    c->cmsg_level = SOL_SOCKET;
    c->cmsg_type = SCM_RIGHTS;
    c->cmsg_len = CMSG_LEN(sizeof(int));
    memcpy(CMSG_DATA(c), &fd, sizeof(int));
    if (sendmsg(g_sock, &h, MSG_DONTWAIT) == (ssize_t)sizeof(m)) return true;
    if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) return false;   // the peer's queue is full
    fatal("sending a segment descriptor to process %d failed: %s", pid, strerror(errno));
}

// one received descriptor into the stash; false when none is waiting
bool recv_fd() {
    FdMsg m;
    iovec io{&m, sizeof(m)};
    alignas(cmsghdr) char ctl[CMSG_SPACE(sizeof(int))];
    msghdr h;
    memset(&h, 0, sizeof(h));
    h.msg_iov = &io;
    h.msg_iovlen = 1;
    h.msg_control = ctl;
    h.msg_controllen = sizeof(ctl);
    const ssize_t n = recvmsg(g_sock, &h, MSG_DONTWAIT | MSG_CMSG_CLOEXEC);
    if (n < 0) {
        if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) return false;
        fatal("receiving a segment descriptor failed: %s", strerror(errno));
    }
    int fd = -1;
    for (cmsghdr *c = CMSG_FIRSTHDR(&h); c; c = CMSG_NXTHDR(&h, c))
        if (c->cmsg_level == SOL_SOCKET && c->cmsg_type == SCM_RIGHTS) memcpy(&fd, CMSG_DATA(c), sizeof(int));
    if (n != (ssize_t)sizeof(m) || fd < 0 || (h.msg_flags & MSG_CTRUNC))
        fatal("a malformed segment-descriptor message (%zd bytes, descriptor %d)", n, fd);
    const auto key = std::make_pair((int)m.rank, m.gen);
    if (g_stash.count(key)) fatal("rank %d sent the descriptor of its allocation %llu twice", m.rank,
                                  (unsigned long long)m.gen);
    g_stash[key] = fd;
    return true;
}

// map `h` at a fresh range and give this GPU access, the launch lock held so no other
// thread of this process issues HIP work meanwhile; nullptr (range retired, logged)
// when the runtime refuses the access -- the handle is then broken (below)
char *map_fresh(hipMemGenericAllocationHandle_t h, size_t bytes, int q) {
    Runtime &r = rt();
    hipMemAccessDesc d;
    memset(&d, 0, sizeof(d));
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = r.device;
    d.flags = hipMemAccessFlagsProtReadWrite;
    char *va = va_take(bytes);
    hipError_t e;
    {
        std::lock_guard<std::mutex> g(r.launch_mu);
        trace(2, "vmm: hipMemMap(%p, %zu) of %s", (void *)va, bytes, q < 0 ? "a new block" : "an imported block");
        GA_HIP(hipMemMap(va, bytes, 0, h, 0));
        trace(2, "vmm: hipMemSetAccess");
        e = hipMemSetAccess(va, bytes, &d, 1);
        trace(2, "vmm: hipMemSetAccess -> %d", (int)e);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            (void)hipMemUnmap(va, bytes);   // may be refused as well: the range is retired either way
            (void)hipGetLastError();
        }
    }
    if (e == hipSuccess) return va;
    g_access_retries.fetch_add(1, std::memory_order_relaxed);
    fprintf(stderr, "[ga_amd %d] hipMemSetAccess(%p, %zu bytes) of %s refused: %s\n", r.rank, (void *)va, bytes,
            q < 0 ? "a new block of this rank" : "a block imported from another rank", hipGetErrorString(e));
    addr_history(va, bytes);
    va_retire(va, bytes);
    return nullptr;
}

// handles the runtime broke: never released (the memory behind them may be another
// allocation's, tools/vmm_probe.hip distinctva), kept until comex_finalize
std::vector<hipMemGenericAllocationHandle_t> g_broken;
std::vector<VmmBlock> g_quarantined;
}  // namespace

// the private window's use: bytes taken so far (ranges + guards) and bytes left; a
// mapping of B bytes takes round_up(B, 2 MiB) + 2 MiB, never returned
void vmm_window_usage(unsigned long long *used, unsigned long long *left) {
    std::lock_guard<std::mutex> g(g_vmm_mu);
    *used = g_window ? (unsigned long long)(g_window - g_window_start) : 0;
    *left = g_window ? (unsigned long long)(g_window_end > g_window ? g_window_end - g_window : 0) : 0;
}

bool vmm_enabled() {
    static const bool on = [] {
        const char *e = getenv("COMEX_AMD_SEGMENT_ALLOC");
        return e && !strcmp(e, "vmm");
    }();
    return on;
}

size_t vmm_round(size_t bytes) {
    const size_t g = granularity();
    return (bytes + g - 1) / g * g;
}

// HBM of this GPU mapped at a fresh address; *fd: its dmabuf descriptor (owned by
// the caller's VmmBlock until vmm_free)
void *vmm_alloc(size_t bytes, VmmBlock *b) {
    const size_t n = vmm_round(bytes);
    hipMemAllocationProp prop;
    memset(&prop, 0, sizeof(prop));
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = rt().device;
    prop.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    // A new handle the runtime refuses access to is broken: measured without this
    // library (tools/vmm_probe.hip, three processes on one GPU, profiles/r04/s08),
    // about one new block in 120 is refused hipMemSetAccess / hipMemcpy, and its
    // exported descriptor resolves in the peers to ANOTHER process's new block.  Such
    // a handle is set aside and another created; its descriptor never leaves.
    for (int attempt = 0;; ++attempt) {
        hipMemGenericAllocationHandle_t h;
        trace(2, "vmm: hipMemCreate(%zu)", n);
        hipError_t e = hipMemCreate(&h, n, &prop, 0);
        if (e == hipErrorOutOfMemory) {   // the freed-segment cache first (segments.cpp)
            (void)hipGetLastError();
            segment_cache_flush();
            e = hipMemCreate(&h, n, &prop, 0);
        }
        if (e != hipSuccess) fatal("hipMemCreate of %zu bytes failed: %s", n, hipGetErrorString(e));
        char *va = map_fresh(h, n, -1);
        if (!va) {
            g_broken.push_back(h);
            if (attempt >= 3) fatal("4 new blocks in a row refused access");
            continue;
        }
        int fd = -1;
        trace(2, "vmm: hipMemExportToShareableHandle");
        GA_HIP(hipMemExportToShareableHandle(&fd, h, hipMemHandleTypePosixFileDescriptor, 0));
        trace(2, "vmm: exported as descriptor %d", fd);
        b->va = va;
        b->bytes = n;
        b->handle = h;
        b->fd = fd;
        b->imported = false;
        addr_event('a', va, n, -1);
        return va;
    }
}

// a new block whose peers' mappings did not read its tags: set aside like a handle
// refused access (mapping and handle kept until comex_finalize), its descriptor closed
void vmm_quarantine(VmmBlock *b) {
    if (!b->va) return;
    std::lock_guard<std::mutex> g(g_vmm_mu);
    g_quarantined.push_back(*b);
    if (b->fd >= 0) close(b->fd);
    g_quarantined.back().fd = -1;
    *b = VmmBlock();
}

// this process's descriptor socket; bound before the comex_malloc allgather, so a
// peer that has the allgather's result can send to it
void vmm_listen() {
    std::lock_guard<std::mutex> g(g_vmm_mu);
    if (g_sock >= 0) return;
    g_sock = socket(AF_UNIX, SOCK_DGRAM | SOCK_CLOEXEC, 0);
    if (g_sock < 0) fatal("socket(AF_UNIX) for segment descriptors failed: %s", strerror(errno));
    sockaddr_un a;
    const socklen_t alen = sock_addr((int)getpid(), &a);
    if (bind(g_sock, (sockaddr *)&a, alen) != 0) fatal("binding the segment-descriptor socket failed: %s", strerror(errno));
}

// send `fd` (allocation `gen` of `rank`) to every process in `to_pids` and receive
// the descriptor of each (rank, allocation) in `from`, into fds[k]; both sides
// progress together (non-blocking sends, a full peer queue retried), so no pair of
// ranks waits on each other
void vmm_exchange(int fd, int rank, uint64_t gen, const std::vector<int> &to_pids,
                  const std::vector<std::pair<int, uint64_t>> &from, int *fds) {
    std::lock_guard<std::mutex> g(g_vmm_mu);
    if (g_sock < 0) fatal("vmm_exchange before vmm_listen");
    std::vector<uint8_t> sent(to_pids.size(), 0);
    size_t nsent = 0, ngot = 0;
    for (size_t k = 0; k < from.size(); ++k) fds[k] = -1;
    const double t0 = now_s();
    for (;;) {
        bool moved = false;
        for (size_t k = 0; k < to_pids.size(); ++k)
            if (!sent[k] && send_fd(to_pids[k], fd, rank, gen)) {
                sent[k] = 1;
                ++nsent;
                moved = true;
            }
        while (recv_fd()) moved = true;
        ngot = 0;
        for (size_t k = 0; k < from.size(); ++k) {
            if (fds[k] < 0) {
                auto it = g_stash.find(from[k]);
                if (it != g_stash.end()) {
                    fds[k] = it->second;
                    g_stash.erase(it);
                }
            }
            ngot += fds[k] >= 0;
        }
        if (nsent == to_pids.size() && ngot == from.size()) return;
        if (now_s() - t0 > 120.0) {
            for (size_t k = 0; k < from.size(); ++k)
                if (fds[k] < 0) fprintf(stderr, "[ga_amd %d] no descriptor from rank %d (allocation %llu)\n", rank,
                                        from[k].first, (unsigned long long)from[k].second);
            fatal("segment-descriptor exchange: %zu of %zu sent, %zu of %zu received in 120 s", nsent,
                  to_pids.size(), ngot, from.size());
        }
        if (!moved) usleep(20);
    }
}

// rank q's block: `myfd` (this process's descriptor of it, from vmm_exchange, owned
// by b from here on), `bytes` (granularity-rounded); nullptr when the runtime refuses
// this GPU access to it
void *vmm_import(int myfd, size_t bytes, int q, VmmBlock *b) {
    hipMemGenericAllocationHandle_t h;
    trace(2, "vmm: hipMemImportFromShareableHandle(descriptor %d) of rank %d", myfd, q);
    // the descriptor is passed by value, as the POSIX-fd handle type is documented
    // for the driver API this one mirrors
    GA_HIP(hipMemImportFromShareableHandle(&h, (void *)(uintptr_t)myfd, hipMemHandleTypePosixFileDescriptor));
    char *va = map_fresh(h, bytes, q);
    if (!va) {
        // refused (the runtime defect above, seen from the importer): kept like a broken
        // handle, the descriptor closed; the caller reports the mapping stale so the owner
        // replaces the block and every member repeats the exchange together
        std::lock_guard<std::mutex> g(g_vmm_mu);
        g_broken.push_back(h);
        if (myfd >= 0) close(myfd);
        *b = VmmBlock();
        return nullptr;
    }
    b->va = va;
    b->bytes = bytes;
    b->handle = h;
    b->fd = myfd;
    b->imported = true;
    addr_event('o', va, bytes, q);
    return va;
}

// unmap and release; the virtual range is retired, not reserved again
void vmm_free(VmmBlock *b) {
    if (!b->va) return;
    addr_event(b->imported ? 'c' : 'f', b->va, b->bytes, -1);
    // (no launch lock here: comex_free calls this under seg_mu, and launch_mu is
    // taken before seg_mu elsewhere)
    GA_HIP(hipMemUnmap(b->va, b->bytes));
    GA_HIP(hipMemRelease(b->handle));
    va_retire(b->va, b->bytes);
    if (b->fd >= 0) close(b->fd);
    b->va = nullptr;
    b->fd = -1;
}

// comex_finalize: the retired ranges and the descriptor socket (every mapping is
// gone by then)
void vmm_finalize() {
    std::lock_guard<std::mutex> g(g_vmm_mu);
    for (VmmBlock &q : g_quarantined) {
        (void)hipMemUnmap(q.va, q.bytes);
        (void)hipMemRelease(q.handle);
    }
    g_quarantined.clear();
    for (auto h : g_broken) (void)hipMemRelease(h);
    g_broken.clear();
    (void)hipGetLastError();
    for (const Retired &x : g_retired) (void)hipMemAddressFree(x.va, x.bytes);
    g_retired.clear();
    g_retired_bytes = 0;
    for (auto &kv : g_stash) close(kv.second);
    g_stash.clear();
    if (g_sock >= 0) close(g_sock);
    g_sock = -1;
}

}  // namespace gaamd

extern "C" unsigned long long gaamd_vmm_access_retries() { return gaamd::g_access_retries.load(); }

// CPU self-test of the descriptor exchange (no GPU): every rank of the bootstrap
// makes a memfd per round holding "rank:round", exchanges the descriptors with every
// other rank exactly as comex_malloc does, and reads each received one back; the number
// of wrong or missing descriptors (0 = pass)
extern "C" int gaamd_vmm_exchange_selftest(int rounds) {
    using namespace gaamd;
    Runtime &r = rt();
    boot_init();
    vmm_listen();
    struct Who { int32_t pid, pad; uint64_t gen; };
    int bad = 0;
    for (int it = 1; it <= rounds; ++it) {
        const int fd = (int)memfd_create("gaamd_fdx", MFD_CLOEXEC);
        if (fd < 0) return -1;
        char msg[32];
        const int len = snprintf(msg, sizeof(msg), "%d:%d", r.rank, it);
        if (write(fd, msg, (size_t)len) != len) return -1;
        Who me{(int32_t)getpid(), 0, (uint64_t)(1000 + it)};
        std::vector<Who> all((size_t)r.size);
        boot_allgather(&me, all.data(), sizeof(Who));
        std::vector<int> to;
        std::vector<std::pair<int, uint64_t>> from;
        for (int q = 0; q < r.size; ++q) {
            if (q == r.rank) continue;
            to.push_back(all[(size_t)q].pid);
            from.push_back({q, all[(size_t)q].gen});
        }
        std::vector<int> got(from.size(), -1);
        vmm_exchange(fd, r.rank, me.gen, to, from, got.data());
        for (size_t k = 0; k < from.size(); ++k) {
            char buf[32] = {0};
            const ssize_t n = pread(got[k], buf, sizeof(buf) - 1, 0);
            char want[32];
            snprintf(want, sizeof(want), "%d:%d", from[k].first, it);
            if (n <= 0 || strcmp(buf, want) != 0) ++bad;
            close(got[k]);
        }
        close(fd);
        boot_barrier();
    }
    return bad;
}
