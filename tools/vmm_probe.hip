// vmm_probe.hip -- two processes, HIP's virtual-memory API, segment create/free cycles
// as GA's create/destroy drives them (the comex_malloc / comex_free of the vmm
// allocator, ga_amd/csrc/vmm.cpp), every step's result printed.
//
// The parent allocates (hipMemCreate + reserve + map + access), writes a tag at both
// ends, exports a dmabuf descriptor and passes it to the child over a socketpair
// (SCM_RIGHTS); the child imports, maps, reads both tags, and each side unmaps and
// releases before the next round.  Variants (argv[1]):
//   close   the child closes its received descriptor right after the import
//   keep    the child closes it only when the mapping goes (what vmm.cpp does)
//   dupfar  the child moves the descriptor to a number it never used before
//   retain  as keep, and neither side releases its virtual ranges
//   fdcheck as retain, printing after each step whether the descriptors are still
//           open in this process (who owns an exported / imported descriptor)
//   mix     as retain, each round first doing a hipMalloc + hipFree of the same size
//           on both sides (GA's scratch buffers between create/destroy cycles)
// Single-process modes (the virtual-range cases behind the library's failures):
//   r_malloc  hipMalloc + hipFree a block, then reserve a range AT its address
//             (hint) and map a new allocation there: map, access, copy
//   r_chunk   one 1 GiB reservation; map blocks one after another inside it (bump),
//             unmapping each before mapping the next
//   r_hint    per-mapping reservations at hinted addresses in a private window far
//             from the runtime's allocations, with hipMalloc/hipFree churn between
//   r_adjacent  a 2 MiB mapping kept, then a mapping of n bytes reserved right at its
//             end (hint), then one 2 MiB further (a gap); each gets hipMemSetAccess
//   samevva / distinctva  three processes: 0 and 1 each allocate a block (at the SAME
//             virtual address in their own spaces, or at different ones), write their
//             tags and send the descriptor to the other two; each imports the other
//             two blocks at fresh ranges and reads the tags (GA's collective
//             comex_malloc makes every rank's allocation sequence the same, so the
//             ranks' blocks coincide in address unless told otherwise); with the
//             suffix _keep no block is released before the last round; with _serial
//             the allocation steps (reserve, create, map, access, export) of the three
//             processes take turns under a file lock
// The sockets are made before either process touches the GPU (fork before HIP).
//
// hipcc --offload-arch=gfx950 -O2 -o tools/vmm_probe tools/vmm_probe.hip
#include <hip/hip_runtime.h>
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/file.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>
#include <vector>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            printf("[%s] %s -> %s\n", who, #x, hipGetErrorString(e_));                           \
            fflush(stdout);                                                                      \
            ok = false;                                                                          \
        }                                                                                        \
    } while (0)

static const char *who = "?";
static bool ok = true;

static void send_fd(int s, int fd, int round) {
    char ctl[CMSG_SPACE(sizeof(int))];
    memset(ctl, 0, sizeof(ctl));
    iovec io{&round, sizeof(round)};
    msghdr h{};
    h.msg_iov = &io;
    h.msg_iovlen = 1;
    h.msg_control = ctl;
    h.msg_controllen = sizeof(ctl);
    cmsghdr *c = CMSG_FIRSTHDR(&h);
    c->cmsg_level = SOL_SOCKET;
    c->cmsg_type = SCM_RIGHTS;
    c->cmsg_len = CMSG_LEN(sizeof(int));
    memcpy(CMSG_DATA(c), &fd, sizeof(int));
    if (sendmsg(s, &h, 0) < 0) perror("sendmsg");
}

static int recv_fd(int s, int *round) {
    char ctl[CMSG_SPACE(sizeof(int))];
    iovec io{round, sizeof(*round)};
    msghdr h{};
    h.msg_iov = &io;
    h.msg_iovlen = 1;
    h.msg_control = ctl;
    h.msg_controllen = sizeof(ctl);
    if (recvmsg(s, &h, 0) <= 0) return -1;
    int fd = -1;
    for (cmsghdr *c = CMSG_FIRSTHDR(&h); c; c = CMSG_NXTHDR(&h, c))
        if (c->cmsg_type == SCM_RIGHTS) memcpy(&fd, CMSG_DATA(c), sizeof(int));
    return fd;
}

static hipMemAllocationProp prop_of() {
    hipMemAllocationProp p;
    memset(&p, 0, sizeof(p));
    p.type = hipMemAllocationTypePinned;
    p.location.type = hipMemLocationTypeDevice;
    p.location.id = 0;
    p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    return p;
}

static void access_rw(void *va, size_t n) {
    hipMemAccessDesc d;
    memset(&d, 0, sizeof(d));
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = 0;
    d.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(va, n, &d, 1));
}

static int single(const char *mode, int rounds, size_t n) {
    who = mode;
    CK(hipSetDevice(0));
    hipMemAllocationProp prop = prop_of();
    size_t gran = 0;
    CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
    char *chunk = nullptr;
    const size_t chunk_bytes = 1ull << 30;
    if (!strcmp(mode, "r_chunk")) CK(hipMemAddressReserve((void **)&chunk, chunk_bytes, gran, nullptr, 0));
    uintptr_t window = 0x200000000000ull;   // 32 TiB
    size_t used = 0;
    for (int r = 0; r < rounds; ++r) {
        ok = true;
        void *hint = nullptr;
        void *tmp = nullptr;
        CK(hipMalloc(&tmp, n));
        CK(hipFree(tmp));
        void *va = nullptr;
        bool own_range = true;
        if (!strcmp(mode, "r_malloc")) {
            hint = tmp;
        } else if (!strcmp(mode, "r_hint")) {
            hint = (void *)(window + used);
            used += (n + gran - 1) / gran * gran;
        }
        if (!strcmp(mode, "r_chunk")) {
            va = chunk + used;
            used += (n + gran - 1) / gran * gran;
            own_range = false;
        } else {
            CK(hipMemAddressReserve(&va, n, gran, hint, 0));
        }
        hipMemGenericAllocationHandle_t h;
        CK(hipMemCreate(&h, n, &prop, 0));
        CK(hipMemMap(va, n, 0, h, 0));
        access_rw(va, n);
        const uint64_t t0 = 0x1000 + r, t1 = 0x2000 + r;
        uint64_t b[2] = {0, 0};
        CK(hipMemcpy(va, &t0, 8, hipMemcpyHostToDevice));
        CK(hipMemcpy((char *)va + n - 8, &t1, 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(&b[0], va, 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&b[1], (char *)va + n - 8, 8, hipMemcpyDeviceToHost));
        printf("[%s] round %d: scratch %p, hint %p -> va %p, reads %#llx / %#llx %s\n", mode, r, tmp, hint, va,
               (unsigned long long)b[0], (unsigned long long)b[1], ok && b[0] == t0 && b[1] == t1 ? "ok" : "FAIL");
        fflush(stdout);
        CK(hipMemUnmap(va, n));
        CK(hipMemRelease(h));
        if (own_range && !strcmp(mode, "r_malloc")) CK(hipMemAddressFree(va, n));
    }
    return 0;
}

static int adjacent(size_t n) {
    who = "r_adjacent";
    CK(hipSetDevice(0));
    hipMemAllocationProp prop = prop_of();
    size_t gran = 0;
    CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
    char *base = (char *)0x210000000000ull;
    auto map_at = [&](char *hint, size_t bytes, const char *what) {
        ok = true;
        void *va = nullptr;
        CK(hipMemAddressReserve(&va, bytes, gran, hint, 0));
        hipMemGenericAllocationHandle_t h;
        CK(hipMemCreate(&h, bytes, &prop, 0));
        CK(hipMemMap(va, bytes, 0, h, 0));
        access_rw(va, bytes);
        printf("[r_adjacent] %s: %zu bytes at %p (asked %p): %s\n", what, bytes, va, hint, ok ? "ok" : "FAILED");
        fflush(stdout);
    };
    map_at(base, 2u << 20, "first (2 MiB)");
    map_at(base + (2u << 20), n, "right at its end");
    map_at(base + (8u << 20), n, "2 MiB past the next boundary (gap)");
    map_at(base + (8u << 20) + ((n + (2u << 20) - 1) & ~((size_t)(2u << 20) - 1)), 2u << 20, "2 MiB right at that one's rounded end");
    return 0;
}

// three processes, each with one datagram socketpair end per peer
static int three(bool same, bool keep, bool serial, int rounds) {
    std::vector<std::pair<void *, hipMemGenericAllocationHandle_t>> kept;
    int sp[3][3][2];   // sp[a][b]: a sends to b on sp[a][b][0], b receives on sp[a][b][1]
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b)
            if (a != b && socketpair(AF_UNIX, SOCK_DGRAM, 0, sp[a][b])) return 2;
    int me = 0;
    pid_t kids[2] = {0, 0};
    for (int k = 1; k < 3; ++k) {
        const pid_t p = fork();
        if (p == 0) { me = k; break; }
        kids[k - 1] = p;
    }
    static char name[16];
    snprintf(name, sizeof(name), "proc%d", me);
    who = name;
    CK(hipSetDevice(0));
    hipMemAllocationProp prop = prop_of();
    size_t gran = 0;
    CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
    const size_t n = 2u << 20;
    uintptr_t next = 0x220000000000ull + (same ? 0 : (uintptr_t)me << 40);
    int bad = 0;
    for (int r = 0; r < rounds; ++r) {
        void *va = nullptr;
        const int lk = serial ? open("/tmp/vmm_probe_alloc.lock", O_CREAT | O_RDWR, 0600) : -1;
        if (lk >= 0) flock(lk, LOCK_EX);   // _serial: one process of the GPU allocates at a time
        CK(hipMemAddressReserve(&va, n, gran, (void *)next, 0));
        next += 4u << 20;
        hipMemGenericAllocationHandle_t h;
        CK(hipMemCreate(&h, n, &prop, 0));
        CK(hipMemMap(va, n, 0, h, 0));
        access_rw(va, n);
        const uint64_t tag = 0xabc000 + 0x100 * me + r;
        CK(hipMemcpy(va, &tag, 8, hipMemcpyHostToDevice));
        CK(hipMemcpy((char *)va + n - 8, &tag, 8, hipMemcpyHostToDevice));
        CK(hipDeviceSynchronize());
        int fd = -1;
        CK(hipMemExportToShareableHandle(&fd, h, hipMemHandleTypePosixFileDescriptor, 0));
        if (lk >= 0) {
            flock(lk, LOCK_UN);
            close(lk);
        }
        for (int b = 0; b < 3; ++b)
            if (b != me) send_fd(sp[me][b][0], fd, r);
        for (int a = 0; a < 3; ++a) {
            if (a == me) continue;
            int rr = -1;
            const int f = recv_fd(sp[a][me][1], &rr);
            hipMemGenericAllocationHandle_t ih;
            CK(hipMemImportFromShareableHandle(&ih, (void *)(uintptr_t)f, hipMemHandleTypePosixFileDescriptor));
            void *iva = nullptr;
            CK(hipMemAddressReserve(&iva, n, gran, (void *)next, 0));
            next += 4u << 20;
            CK(hipMemMap(iva, n, 0, ih, 0));
            access_rw(iva, n);
            uint64_t t[2] = {0, 0};
            CK(hipMemcpy(&t[0], iva, 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&t[1], (char *)iva + n - 8, 8, hipMemcpyDeviceToHost));
            const uint64_t want = 0xabc000 + 0x100 * a + r;
            const bool good = t[0] == want && t[1] == want;
            bad += !good;
            printf("[%s] round %d: own block at %p; proc%d's block mapped at %p reads %#llx / %#llx (want %#llx) %s\n",
                   name, r, va, a, iva, (unsigned long long)t[0], (unsigned long long)t[1], (unsigned long long)want,
                   good ? "ok" : "WRONG");
            fflush(stdout);
            CK(hipMemUnmap(iva, n));
            CK(hipMemRelease(ih));
            close(f);
        }
        // everyone done reading before anyone frees (one byte to each peer and back)
        for (int b = 0; b < 3; ++b)
            if (b != me) send(sp[me][b][0], &r, sizeof(r), 0);
        for (int a = 0; a < 3; ++a)
            if (a != me) { int x; recv(sp[a][me][1], &x, sizeof(x), 0); }
        if (keep) {
            kept.push_back({va, h});
        } else {
            CK(hipMemUnmap(va, n));
            CK(hipMemRelease(h));
        }
        close(fd);
    }
    for (auto &k : kept) {
        CK(hipMemUnmap(k.first, n));
        CK(hipMemRelease(k.second));
    }
    if (me) return bad ? 1 : 0;
    int all_ok = !bad;
    for (pid_t k : kids) {
        int st = 0;
        waitpid(k, &st, 0);
        all_ok = all_ok && WIFEXITED(st) && WEXITSTATUS(st) == 0;
    }
    printf("mode %s%s%s: %s\n", same ? "samevva" : "distinctva", keep ? "_keep" : "", serial ? "_serial" : "",
           all_ok ? "PASS" : "FAIL");
    return all_ok ? 0 : 1;
}

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "keep";
    if (!strncmp(mode, "samevva", 7) || !strncmp(mode, "distinctva", 10))
        return three(!strncmp(mode, "samevva", 7), strstr(mode, "_keep") != nullptr, strstr(mode, "_serial") != nullptr,
                     argc > 2 ? atoi(argv[2]) : 3);
    if (!strcmp(mode, "r_adjacent")) return adjacent(argc > 3 ? strtoull(argv[3], nullptr, 0) : 0x202000);
    if (!strncmp(mode, "r_", 2))
        return single(mode, argc > 2 ? atoi(argv[2]) : 4, argc > 3 ? strtoull(argv[3], nullptr, 0) : (2u << 20));
    const int rounds = argc > 2 ? atoi(argv[2]) : 6;
    const size_t n = argc > 3 ? strtoull(argv[3], nullptr, 0) : (2u << 20);
    const bool mix = !strcmp(mode, "mix");
    const bool fdcheck = !strcmp(mode, "fdcheck");
    const bool retain = !strcmp(mode, "retain") || mix || fdcheck;
    auto fd_open = [](int f) { return f >= 0 && fcntl(f, F_GETFD) != -1; };
    int sv[2], ack[2];
    if (socketpair(AF_UNIX, SOCK_DGRAM, 0, sv) || socketpair(AF_UNIX, SOCK_DGRAM, 0, ack)) return 2;
    const pid_t child = fork();
    if (child < 0) return 2;
    who = child ? "owner" : "peer";
    CK(hipSetDevice(0));
    hipMemAllocationProp prop = prop_of();
    size_t gran = 0;
    CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
    if (child) printf("mode %s, %d rounds of %zu bytes, granularity %zu\n", mode, rounds, n, gran);
    int far = 900;
    for (int r = 0; r < rounds; ++r) {
        if (mix) {
            void *tmp = nullptr;
            CK(hipMalloc(&tmp, n));
            printf("[%s] round %d: hipMalloc scratch at %p (freed)\n", who, r, tmp);
            CK(hipFree(tmp));
        }
        if (child) {
            hipMemGenericAllocationHandle_t h;
            CK(hipMemCreate(&h, n, &prop, 0));
            void *va = nullptr;
            CK(hipMemAddressReserve(&va, n, gran, nullptr, 0));
            CK(hipMemMap(va, n, 0, h, 0));
            access_rw(va, n);
            const uint64_t t0 = 0x1000 + r, t1 = 0x2000 + r;
            CK(hipMemcpy(va, &t0, 8, hipMemcpyHostToDevice));
            CK(hipMemcpy((char *)va + n - 8, &t1, 8, hipMemcpyHostToDevice));
            int fd = -1;
            CK(hipMemExportToShareableHandle(&fd, h, hipMemHandleTypePosixFileDescriptor, 0));
            printf("[owner] round %d: va %p, descriptor %d\n", r, va, fd);
            fflush(stdout);
            send_fd(sv[0], fd, r);
            int a = 0;
            if (recv(ack[0], &a, sizeof(a), 0) <= 0) break;
            if (fdcheck) printf("[owner] round %d: export descriptor %d open after send: %d\n", r, fd, fd_open(fd));
            CK(hipMemUnmap(va, n));
            CK(hipMemRelease(h));
            if (fdcheck) printf("[owner] round %d: export descriptor %d open after hipMemRelease: %d\n", r, fd, fd_open(fd));
            if (!retain) CK(hipMemAddressFree(va, n));
            close(fd);
        } else {
            int rr = -1;
            int fd = recv_fd(sv[1], &rr);
            if (fd < 0) break;
            if (!strcmp(mode, "dupfar")) {
                const int f2 = fcntl(fd, F_DUPFD_CLOEXEC, far++);
                close(fd);
                fd = f2;
            }
            hipMemGenericAllocationHandle_t h;
            CK(hipMemImportFromShareableHandle(&h, (void *)(uintptr_t)fd, hipMemHandleTypePosixFileDescriptor));
            if (fdcheck) printf("[peer] round %d: received descriptor %d open after import: %d\n", rr, fd, fd_open(fd));
            if (!strcmp(mode, "close")) {
                close(fd);
                fd = -1;
            }
            void *va = nullptr;
            CK(hipMemAddressReserve(&va, n, gran, nullptr, 0));
            CK(hipMemMap(va, n, 0, h, 0));
            access_rw(va, n);
            uint64_t t[2] = {0, 0};
            CK(hipMemcpy(&t[0], va, 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&t[1], (char *)va + n - 8, 8, hipMemcpyDeviceToHost));
            const bool good = t[0] == 0x1000u + rr && t[1] == 0x2000u + rr;
            printf("[peer] round %d: descriptor %d, va %p reads %#llx / %#llx %s\n", rr, fd, va,
                   (unsigned long long)t[0], (unsigned long long)t[1], good ? "ok" : "WRONG");
            fflush(stdout);
            if (!good) ok = false;
            CK(hipMemUnmap(va, n));
            CK(hipMemRelease(h));
            if (fdcheck) printf("[peer] round %d: received descriptor %d open after hipMemRelease: %d\n", rr, fd, fd_open(fd));
            if (!retain) CK(hipMemAddressFree(va, n));
            if (fd >= 0) close(fd);
            int a = 1;
            send(ack[1], &a, sizeof(a), 0);
        }
    }
    if (!child) return ok ? 0 : 1;
    int st = 0;
    waitpid(child, &st, 0);
    const bool all = ok && WIFEXITED(st) && WEXITSTATUS(st) == 0;
    printf("mode %s: %s\n", mode, all ? "PASS" : "FAIL");
    return all ? 0 : 1;
}
