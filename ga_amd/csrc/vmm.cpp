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
//   * the descriptor reaches a peer process through pidfd_getfd (the owner's pid
//     and descriptor number travel in the comex_malloc allgather, as reg_entry_t
//     does at comex.c:2461) and is imported there (hipMemImportFromShareableHandle);
//   * every mapping -- the owner's and each peer's -- goes to virtual addresses this
//     library reserved itself and NEVER hands out twice in the process's life (a bump
//     allocator over reserved chunks), so no export or import ever meets an address
//     the runtime has seen before.
// COMEX_AMD_SEGMENT_ALLOC=vmm selects it (ipc: hipMalloc + hipIpc*, the round-3 path).
#include "comex_impl.hpp"
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <mutex>
#include <vector>

#ifndef SYS_pidfd_open
#define SYS_pidfd_open 434
#endif
#ifndef SYS_pidfd_getfd
#define SYS_pidfd_getfd 438
#endif

namespace gaamd {

namespace {
std::mutex g_vmm_mu;
struct Chunk { char *base; size_t bytes, used; };
std::vector<Chunk> g_chunks;            // reserved virtual ranges, never released before finalize
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
    g_gran = g ? g : (2u << 20);
    return g_gran;
}

// a fresh virtual range of `bytes` (a multiple of the granularity), never used before
char *va_take(size_t bytes) {
    std::lock_guard<std::mutex> g(g_vmm_mu);
    const size_t gr = granularity();
    for (Chunk &c : g_chunks) {
        if (c.bytes - c.used >= bytes) {
            char *p = c.base + c.used;
            c.used += bytes;   // bump only: a range is never handed out again
            return p;
        }
    }
    const size_t chunk = std::max<size_t>((bytes + gr - 1) / gr * gr, 256ull << 30);
    void *base = nullptr;
    GA_HIP(hipMemAddressReserve(&base, chunk, gr, nullptr, 0));
    g_chunks.push_back({(char *)base, chunk, bytes});
    return (char *)base;
}

void set_access(char *va, size_t bytes) {
    hipMemAccessDesc d;
    memset(&d, 0, sizeof(d));
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = rt().device;
    d.flags = hipMemAccessFlagsProtReadWrite;
    GA_HIP(hipMemSetAccess(va, bytes, &d, 1));
}
}  // namespace

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
    hipMemGenericAllocationHandle_t h;
    hipError_t e = hipMemCreate(&h, n, &prop, 0);
    if (e == hipErrorOutOfMemory) {   // the freed-segment cache first (segments.cpp)
        (void)hipGetLastError();
        segment_cache_flush();
        e = hipMemCreate(&h, n, &prop, 0);
    }
    if (e != hipSuccess) fatal("hipMemCreate of %zu bytes failed: %s", n, hipGetErrorString(e));
    char *va = va_take(n);
    GA_HIP(hipMemMap(va, n, 0, h, 0));
    set_access(va, n);
    int fd = -1;
    GA_HIP(hipMemExportToShareableHandle(&fd, h, hipMemHandleTypePosixFileDescriptor, 0));
    b->va = va;
    b->bytes = n;
    b->handle = h;
    b->fd = fd;
    b->imported = false;
    addr_event('a', va, n, -1);
    return va;
}

// rank q's block: descriptor `fd` in process `pid`, `bytes` (granularity-rounded)
void *vmm_import(int pid, int fd, size_t bytes, int q, VmmBlock *b) {
    const int pidfd = (int)syscall(SYS_pidfd_open, pid, 0);
    if (pidfd < 0) fatal("pidfd_open(%d) for rank %d's segment failed: %s", pid, q, strerror(errno));
    const int myfd = (int)syscall(SYS_pidfd_getfd, pidfd, fd, 0);
    close(pidfd);
    if (myfd < 0) fatal("pidfd_getfd(rank %d's descriptor %d) failed: %s", q, fd, strerror(errno));
    hipMemGenericAllocationHandle_t h;
    // the descriptor is passed by value, as the POSIX-fd handle type is documented
    // for the driver API this one mirrors
    GA_HIP(hipMemImportFromShareableHandle(&h, (void *)(uintptr_t)myfd, hipMemHandleTypePosixFileDescriptor));
    char *va = va_take(bytes);
    GA_HIP(hipMemMap(va, bytes, 0, h, 0));
    set_access(va, bytes);
    b->va = va;
    b->bytes = bytes;
    b->handle = h;
    b->fd = myfd;
    b->imported = true;
    addr_event('o', va, bytes, q);
    return va;
}

// unmap and release; the virtual range stays reserved (never reused)
void vmm_free(VmmBlock *b) {
    if (!b->va) return;
    addr_event(b->imported ? 'c' : 'f', b->va, b->bytes, -1);
    GA_HIP(hipMemUnmap(b->va, b->bytes));
    GA_HIP(hipMemRelease(b->handle));
    if (b->fd >= 0) close(b->fd);
    b->va = nullptr;
    b->fd = -1;
}

// comex_finalize: the reserved ranges (every mapping is gone by then)
void vmm_finalize() {
    std::lock_guard<std::mutex> g(g_vmm_mu);
    for (const Chunk &c : g_chunks) (void)hipMemAddressFree(c.base, c.bytes);
    g_chunks.clear();
}

}  // namespace gaamd
