// wire.cpp -- the host fallback between nodes: the MPI-PR message protocol
// (comex/src-mpi-pr/comex.c) restated over TCP.
//
// Inside a node every rank maps every other rank's HBM (IPC) and remote
// accumulates go through the owner's inbox (comex.cpp).  Ranks on different
// nodes cannot map each other, so -- like the reference, where every remote
// operation is a message to the target's progress rank -- they exchange
// messages: one frame carrying the fields of header_t (comex.c:115-121), the
// scale and stride_t (131-136), followed by the packed payload.
//
//   initiator (client)                         target (server thread)
//   put/acc : pack kernel -> pinned host buf   recv into pinned host buf ->
//             -> send frame + payload          unpack(-acc) kernel reading the
//                                              mapped buffer into its HBM
//             (nb_puts_packed 6342-6533,       (_put_packed_handler 3605-3677,
//              nb_accs_packed 6965-7109)        _acc_packed_handler 4133-4281)
//   get     : send frame; recv payload ->      pack kernel from its HBM into
//             unpack kernel into local dst      pinned buf -> send payload
//             (nb_gets_packed 6617-6804)       (_get_packed_handler 3854-3902)
//   io-vec  : k_iov gathers the n sources;     k_iov scatters / accumulates into
//             payload = data + n addresses      the n addresses (4284-4397)
//   fence   : OP_FENCE, wait for the reply     reply once every earlier kernel of
//             (comex_fence_proc 1074-1234)      this connection has completed
//
// Op codes keep the values of op_t (comex.c:74-112).  Differences from the
// reference, all internal to this transport: one fixed-size frame instead of
// header + scale + stride_t messages; payloads larger than the pinned buffer
// are cut into row ranges (each frame carries its rows [row_begin, row_end)),
// not into backwards max_message_size chunks; a connection per (initiator,
// target) pair gives in-order delivery, which the reference gets from MPI's
// message ordering.  The target applies a frame's kernel on its library
// streams through the dependency scheduler, so accumulates into one target
// stay mutually exclusive (the reference's per-target semaphores).
//
// Exposure: the listener binds ONE interface -- COMEX_AMD_WIRE_ADDR, default
// 127.0.0.1 (a job spanning hosts must name the interface explicitly) -- and a
// connection is served only after it presents the job's 32-byte secret, drawn
// from /dev/urandom by rank 0 and handed to every rank through the bootstrap
// allgather (the launcher's channel).  Every address a frame names must lie
// inside one of the target's comex_malloc segments (reg_cache_find) or the
// target aborts.
#include "runtime.hpp"
#include "gaamd_kernels.h"
#include "../../include/comex.h"
#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>
#include <algorithm>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>

namespace gaamd {

namespace {

// op_t, comex.c:74-112 (the values travel on the wire)
enum : int32_t {
    W_PUT = 0, W_PUT_PACKED = 1, W_PUT_IOV = 3,
    W_GET = 4, W_GET_PACKED = 5, W_GET_IOV = 7,
    W_ACC = 8,          // + COMEX_ACC_x - 37: INT DBL FLT CPL DCP LNG
    W_ACC_PACKED = 14,  // + ...
    W_ACC_IOV = 20,     // + ...
    W_FENCE = 26, W_FETCH_AND_ADD = 27, W_SWAP = 28, W_LOCK = 31, W_UNLOCK = 32, W_QUIT = 33,
    W_PING = 1000,      // bootstrap self-test (not a reference op)
    W_MSG = 1001        // armci_msg_snd payload (MPI_Send in the reference, message.c:354)
};

struct Frame {
    // header_t
    int32_t operation;
    int32_t rank;              // target rank
    uint64_t remote_address;   // target-side address: dst of put/acc, src of get
    uint64_t local_address;    // initiator-side address (informational)
    uint64_t length;           // payload bytes after the frame (get: bytes asked for)
    // stride_t of the target side
    int32_t stride_levels;
    int32_t stride[8];
    int32_t count[9];
    // rows of the patch this frame carries (odometer order, comex.c:1308-1322)
    uint64_t row_begin, row_end;
    uint8_t scale[16];
    // io-vector: n pairs of `iov_bytes`; serial: destinations overlap (in order)
    int32_t iov_n, iov_bytes, iov_serial, src_rank;
};

struct Peer {
    int fd = -1;
    bool dirty = false;   // frames sent since the last fence
};

struct Pinned {   // mapped pinned host buffer + completion of the last kernel using it
    char *host = nullptr;
    char *dev = nullptr;
    size_t bytes = 0;
    hipEvent_t ev = nullptr;
    bool pending = false;
};

struct Endpoint {
    uint32_t addr;   // network order
    uint16_t port;   // network order
    uint16_t pad;
};

std::vector<Endpoint> g_ep;
std::vector<std::unique_ptr<Peer>> g_peer;
int g_listen = -1;
int g_wake[2] = {-1, -1};
std::thread g_server;
bool g_active = false;
Pinned g_cli[2];
Pinned g_srv[2];
int g_srv_next = 0;
size_t g_chunk = 64u << 20;
constexpr size_t kSecret = 32;

// armci_msg point-to-point messages received for this rank, in arrival order
// (per sender in send order: one connection per sender)
struct Msg {
    int from, tag;
    std::vector<char> data;
};
std::mutex g_msg_mu;
std::mutex g_send_mu;   // initiator connections: messages may be sent from any user thread
std::condition_variable g_msg_cv;
std::deque<Msg> g_msgs;

void msg_push(int from, int tag, std::vector<char> &&data) {
    {
        std::lock_guard<std::mutex> g(g_msg_mu);
        g_msgs.push_back({from, tag, std::move(data)});
    }
    g_msg_cv.notify_all();
}
unsigned char g_secret[kSecret];

void wait_pinned(Pinned &b) {
    if (b.pending) GA_HIP(hipEventSynchronize(b.ev));
    b.pending = false;
}

void ensure_pinned(Pinned &b, size_t need) {
    need = std::max<size_t>(need, 4096);
    if (!b.ev) GA_HIP(hipEventCreateWithFlags(&b.ev, hipEventDisableTiming));
    if (b.bytes >= need) return;
    wait_pinned(b);
    if (b.host) GA_HIP(hipHostFree(b.host));
    GA_HIP(hipHostMalloc((void **)&b.host, need, hipHostMallocMapped | hipHostMallocPortable));
    void *d = nullptr;
    GA_HIP(hipHostGetDevicePointer(&d, b.host, 0));
    b.dev = (char *)d;
    b.bytes = need;
}

void free_pinned(Pinned &b) {
    wait_pinned(b);
    if (b.host) (void)hipHostFree(b.host);
    if (b.ev) (void)hipEventDestroy(b.ev);
    b = Pinned();
}

void send_all(int fd, const void *p, size_t n) {
    const char *c = (const char *)p;
    while (n) {
        const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) fatal("wire: send failed (%s)", strerror(errno));
        c += k;
        n -= (size_t)k;
    }
}

// false: the peer closed the connection before the first byte
bool recv_all(int fd, void *p, size_t n, bool eof_ok = false) {
    char *c = (char *)p;
    size_t got = 0;
    while (got < n) {
        const ssize_t k = ::recv(fd, c + got, n - got, 0);
        if (k < 0 && errno == EINTR) continue;
        if (k == 0 && got == 0 && eof_ok) return false;
        if (k <= 0) fatal("wire: recv failed (%s)", k == 0 ? "connection closed" : strerror(errno));
        got += (size_t)k;
    }
    return true;
}

void tune_socket(int fd) {
    int one = 1;
    (void)setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    int buf = 8 << 20;
    (void)setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
    (void)setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
}

Peer &connect_to(int t) {
    Peer &p = *g_peer[t];
    if (p.fd >= 0) return p;
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) fatal("wire: socket failed (%s)", strerror(errno));
    sockaddr_in a;
    memset(&a, 0, sizeof(a));
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = g_ep[t].addr;
    a.sin_port = g_ep[t].port;
    if (::connect(fd, (sockaddr *)&a, sizeof(a)) != 0)
        fatal("wire: connect to rank %d (%s:%d) failed (%s)", t, inet_ntoa(a.sin_addr), ntohs(a.sin_port),
              strerror(errno));
    tune_socket(fd);
    send_all(fd, g_secret, kSecret);   // the job secret opens the connection
    p.fd = fd;
    return p;
}

// a new connection must present the job secret within a few seconds
bool admit(int c) {
    timeval tv;
    tv.tv_sec = 5;
    tv.tv_usec = 0;
    (void)setsockopt(c, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    unsigned char got[kSecret];
    size_t n = 0;
    while (n < kSecret) {
        const ssize_t k = ::recv(c, got + n, kSecret - n, 0);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return false;
        n += (size_t)k;
    }
    unsigned char diff = 0;
    for (size_t i = 0; i < kSecret; ++i) diff |= (unsigned char)(got[i] ^ g_secret[i]);
    tv.tv_sec = 0;
    (void)setsockopt(c, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    return diff == 0;
}

uint64_t fnv1a(const char *p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) { h ^= (uint8_t)p[i]; h *= 1099511628211ull; }
    return h;
}

int acc_index(int op) { return op - COMEX_ACC_INT; }   // 0..5 in op_t order

void packed_strides(const int *count, int levels, int *pstride) {
    int64_t acc = count[0];
    for (int j = 0; j < levels; ++j) { pstride[j] = (int)acc; acc *= count[j + 1]; }
}

uint64_t rows_of(const int *count, int levels) {
    uint64_t rows = 1;
    for (int j = 1; j <= levels; ++j) rows *= (uint64_t)count[j];
    return rows;
}

uint64_t iov_list_off(int n, int bytes) { return (((uint64_t)n * (uint64_t)bytes) + 15) & ~15ull; }

Frame make_frame(int32_t op, int t, uint64_t remote, const int *stride, const int *count, int levels) {
    Frame f;
    memset(&f, 0, sizeof(f));
    f.operation = op;
    f.rank = t;
    f.remote_address = remote;
    f.stride_levels = levels;
    for (int j = 0; j < 8; ++j) f.stride[j] = (stride && j < levels) ? stride[j] : -1;   // unused: -1 (comex.c:7004)
    for (int j = 0; j < 9; ++j) f.count[j] = (count && j <= levels) ? count[j] : -1;
    f.src_rank = rt().rank;
    return f;
}

// ---- target side ------------------------------------------------------------
void check_local(uint64_t p, int64_t lo, int64_t hi, int from) {
    if (!segment_local((const void *)(uintptr_t)p, lo, hi))
        fatal("wire: rank %d addressed %p [%ld,%ld), not inside a local comex_malloc segment", from,
              (void *)(uintptr_t)p, (long)lo, (long)hi);
}

Pinned &next_srv_buf(size_t need) {
    Pinned &b = g_srv[g_srv_next];
    g_srv_next ^= 1;
    wait_pinned(b);   // the kernel that read it last has finished
    ensure_pinned(b, need);
    return b;
}

void serve_put_acc(int fd, const Frame &f, bool iov) {
    Runtime &r = rt();
    const int op = f.operation;
    int cop = kOpCopy;
    if (op >= W_ACC && op < W_ACC + 6) cop = COMEX_ACC_INT + (op - W_ACC);
    if (op >= W_ACC_PACKED && op < W_ACC_PACKED + 6) cop = COMEX_ACC_INT + (op - W_ACC_PACKED);
    if (op >= W_ACC_IOV && op < W_ACC_IOV + 6) cop = COMEX_ACC_INT + (op - W_ACC_IOV);
    Pinned &b = next_srv_buf(f.length);
    recv_all(fd, b.host, f.length);
    if (iov) {
        const int n = f.iov_n, bytes = f.iov_bytes;
        const uint64_t loff = iov_list_off(n, bytes);
        if (f.length != loff + (uint64_t)n * 8) fatal("wire: io-vector frame of %lu bytes for %d pairs", (unsigned long)f.length, n);
        const uint64_t *dst = (const uint64_t *)(b.host + loff);
        uint64_t align_or = 0, dlo = ~0ull, dhi = 0;
        for (int i = 0; i < n; ++i) {
            check_local(dst[i], 0, bytes, f.src_rank);
            align_or |= dst[i];
            dlo = std::min(dlo, dst[i]);
            dhi = std::max(dhi, dst[i] + (uint64_t)bytes);
        }
        IovDesc d;
        memset(&d, 0, sizeof(d));
        d.src_base = b.dev;
        d.dst_list = (const uint64_t *)(b.dev + loff);
        d.bytes = bytes;
        d.n = (uint32_t)n;
        std::lock_guard<std::mutex> g(r.launch_mu);
        Span ss, ds;
        ss.lo = (int64_t)(uintptr_t)b.dev;
        ss.hi = ss.lo + (int64_t)f.length;
        ds.lo = (int64_t)dlo;
        ds.hi = (int64_t)dhi;
        const int si = sched_pick(ss, ds);
        const int rc = launch_iov(cop, f.scale, d, align_or, f.iov_serial != 0, r.streams[si]);
        if (rc) fatal("wire: io-vector launch failed (%d)", rc);
        GA_HIP(hipEventRecord(b.ev, r.streams[si]));
        b.pending = true;
        return;
    }
    const int levels = f.stride_levels;
    int64_t dlo = 0, dhi = 0;
    const int64_t rowb = (cop == kOpCopy) ? f.count[0] : (int64_t)(f.count[0] / elem_size(cop)) * elem_size(cop);
    side_span_host(f.stride, f.count, levels, rowb, &dlo, &dhi);
    check_local(f.remote_address, dlo, dhi, f.src_rank);
    if (f.length != (f.row_end - f.row_begin) * (uint64_t)f.count[0]) fatal("wire: frame length mismatch");
    int pstride[8];
    packed_strides(f.count, levels, pstride);
    std::lock_guard<std::mutex> g(r.launch_mu);
    Span ss, ds;
    ss.lo = (int64_t)(uintptr_t)b.dev;
    ss.hi = ss.lo + (int64_t)f.length;
    ds.lo = (int64_t)f.remote_address + dlo;
    ds.hi = (int64_t)f.remote_address + dhi;
    const int si = sched_pick(ss, ds);
    // packed rows [row_begin, row_end) start at b.dev: rebase the packed side
    const int rc = launch_strided(cop, f.scale, b.dev - (int64_t)f.row_begin * f.count[0], pstride,
                                  (void *)(uintptr_t)f.remote_address, f.stride, f.count, levels, r.streams[si],
                                  nullptr, f.row_begin, f.row_end);
    if (rc) fatal("wire: unpack launch failed (%d)", rc);
    GA_HIP(hipEventRecord(b.ev, r.streams[si]));
    b.pending = true;
}

void serve_get(int fd, const Frame &f, bool iov) {
    Runtime &r = rt();
    if (iov) {
        const int n = f.iov_n, bytes = f.iov_bytes;
        const uint64_t loff = iov_list_off(n, bytes);
        Pinned &b = next_srv_buf(loff + (uint64_t)n * 8);
        recv_all(fd, b.host + loff, (size_t)n * 8);
        const uint64_t *src = (const uint64_t *)(b.host + loff);
        uint64_t align_or = 0, slo = ~0ull, shi = 0;
        for (int i = 0; i < n; ++i) {
            check_local(src[i], 0, bytes, f.src_rank);
            align_or |= src[i];
            slo = std::min(slo, src[i]);
            shi = std::max(shi, src[i] + (uint64_t)bytes);
        }
        IovDesc d;
        memset(&d, 0, sizeof(d));
        d.src_list = (const uint64_t *)(b.dev + loff);
        d.dst_base = b.dev;
        d.bytes = bytes;
        d.n = (uint32_t)n;
        int si;
        {
            std::lock_guard<std::mutex> g(r.launch_mu);
            Span ss, ds;
            ss.lo = (int64_t)slo;
            ss.hi = (int64_t)shi;
            ds.lo = (int64_t)(uintptr_t)b.dev;
            ds.hi = ds.lo + (int64_t)loff;
            si = sched_pick(ss, ds);
            const int rc = launch_iov(kOpCopy, nullptr, d, align_or, false, r.streams[si]);
            if (rc) fatal("wire: io-vector gather failed (%d)", rc);
        }
        GA_HIP(hipStreamSynchronize(r.streams[si]));
        send_all(fd, b.host, (size_t)n * bytes);
        return;
    }
    const int levels = f.stride_levels;
    int64_t slo = 0, shi = 0;
    side_span_host(f.stride, f.count, levels, f.count[0], &slo, &shi);
    check_local(f.remote_address, slo, shi, f.src_rank);
    if (f.length != (f.row_end - f.row_begin) * (uint64_t)f.count[0]) fatal("wire: frame length mismatch");
    Pinned &b = next_srv_buf(f.length);
    int pstride[8];
    packed_strides(f.count, levels, pstride);
    int si;
    {
        std::lock_guard<std::mutex> g(r.launch_mu);
        Span ss, ds;
        ss.lo = (int64_t)f.remote_address + slo;
        ss.hi = (int64_t)f.remote_address + shi;
        ds.lo = (int64_t)(uintptr_t)b.dev;
        ds.hi = ds.lo + (int64_t)f.length;
        si = sched_pick(ss, ds);
        const int rc = launch_strided(kOpCopy, nullptr, (void *)(uintptr_t)f.remote_address, f.stride,
                                      b.dev - (int64_t)f.row_begin * f.count[0], pstride, f.count, levels,
                                      r.streams[si], nullptr, f.row_begin, f.row_end);
        if (rc) fatal("wire: pack launch failed (%d)", rc);
    }
    GA_HIP(hipStreamSynchronize(r.streams[si]));
    send_all(fd, b.host, f.length);
}

// one frame from `fd`; false when the peer has gone (QUIT or close)
bool serve_frame(int fd) {
    Frame f;
    if (!recv_all(fd, &f, sizeof(f), true)) return false;
    const int op = f.operation;
    if (op == W_PING) {
        std::vector<char> buf(f.length);
        if (f.length) recv_all(fd, buf.data(), f.length);
        const uint64_t h = fnv1a(buf.data(), buf.size()) ^ (uint64_t)rt().rank;
        send_all(fd, &h, sizeof(h));
        return true;
    }
    if (op == W_QUIT) return false;
    if (op == W_MSG) {
        std::vector<char> buf(f.length);
        if (f.length) recv_all(fd, buf.data(), f.length);
        msg_push(f.src_rank, (int)(int64_t)f.remote_address, std::move(buf));
        return true;
    }
    if (op == W_LOCK || op == W_UNLOCK) {
        // mutex f.remote_address of this rank (comex_lock/unlock, comex.c OP_LOCK/OP_UNLOCK):
        // a try-lock answered at once; the initiator retries
        char ok = 1;
        if (op == W_LOCK) ok = mutex_try_local(rt().rank, (int)f.remote_address) ? 1 : 0;
        else mutex_release_local(rt().rank, (int)f.remote_address);
        send_all(fd, &ok, 1);
        return true;
    }
    static thread_local bool dev_set = false;
    if (!dev_set) {
        GA_HIP(hipSetDevice(rt().device));
        dev_set = true;
    }
    if (op == W_FENCE) {
        wait_pinned(g_srv[0]);
        wait_pinned(g_srv[1]);
        const char ack = 1;
        send_all(fd, &ack, 1);
        return true;
    }
    if (op == W_FETCH_AND_ADD || op == W_SWAP) {
        // after every earlier frame of this connection: their kernels were scheduled
        // before this one, and the rmw kernel is ordered behind those touching its bytes
        check_local(f.remote_address, 0, (int64_t)f.length, f.src_rank);
        uint64_t val = 0;
        memcpy(&val, f.scale, 8);
        const uint64_t old = rmw_local(op == W_SWAP, (void *)(uintptr_t)f.remote_address, (int)f.length, val);
        send_all(fd, &old, sizeof(old));
        return true;
    }
    if (op == W_PUT || op == W_PUT_PACKED || (op >= W_ACC && op < W_ACC_PACKED + 6)) {
        serve_put_acc(fd, f, false);
        return true;
    }
    if (op == W_PUT_IOV || (op >= W_ACC_IOV && op < W_ACC_IOV + 6)) {
        serve_put_acc(fd, f, true);
        return true;
    }
    if (op == W_GET || op == W_GET_PACKED) {
        serve_get(fd, f, false);
        return true;
    }
    if (op == W_GET_IOV) {
        serve_get(fd, f, true);
        return true;
    }
    fatal("wire: unknown operation %d from rank %d", op, f.src_rank);
}

void server_loop() {
    Runtime &r = rt();
    std::vector<int> conns;
    bool stopping = false;
    for (;;) {
        std::vector<pollfd> pf;
        pf.push_back({g_listen, POLLIN, 0});
        pf.push_back({g_wake[0], POLLIN, 0});
        for (int c : conns) pf.push_back({c, POLLIN, 0});
        const int k = ::poll(pf.data(), pf.size(), stopping ? 0 : 1000);
        if (k < 0 && errno == EINTR) continue;
        if (k < 0) fatal("wire: poll failed (%s)", strerror(errno));
        if (pf[1].revents & POLLIN) {
            // finalize: every initiator has sent its last frame (QUIT) before the
            // barrier that preceded the wake; drain what is still queued
            char w;
            if (::read(g_wake[0], &w, 1) != 1) fatal("wire: wake read failed");
            stopping = true;
        }
        std::vector<int> keep;
        for (size_t i = 2; i < pf.size(); ++i) {
            const int c = pf[i].fd;
            bool alive = true;
            if (pf[i].revents & (POLLIN | POLLHUP | POLLERR)) alive = serve_frame(c);
            if (alive) keep.push_back(c);
            else ::close(c);
        }
        if (pf[0].revents & POLLIN) {
            const int c = ::accept(g_listen, nullptr, nullptr);
            if (c >= 0) {
                if (admit(c)) {
                    tune_socket(c);
                    keep.push_back(c);
                } else {
                    fprintf(stderr, "[%d] wire: refused a connection without the job secret\n", r.rank);
                    ::close(c);
                }
            }
        }
        conns.swap(keep);
        if (stopping && conns.empty() && !(pf[0].revents & POLLIN) && k == 0) break;
    }
    wait_pinned(g_srv[0]);
    wait_pinned(g_srv[1]);
}

// the one interface the listener binds and advertises
uint32_t wire_addr() {
    const char *a = getenv("COMEX_AMD_WIRE_ADDR");
    if (!a) return htonl(INADDR_LOOPBACK);
    in_addr x;
    if (!inet_aton(a, &x)) fatal("COMEX_AMD_WIRE_ADDR=%s is not an IPv4 address", a);
    if (x.s_addr == htonl(INADDR_ANY)) fatal("COMEX_AMD_WIRE_ADDR must name one interface, not 0.0.0.0");
    return x.s_addr;
}

void start_sockets() {
    Runtime &r = rt();
    g_listen = ::socket(AF_INET, SOCK_STREAM, 0);
    if (g_listen < 0) fatal("wire: socket failed (%s)", strerror(errno));
    int one = 1;
    (void)setsockopt(g_listen, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a;
    memset(&a, 0, sizeof(a));
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = wire_addr();
    a.sin_port = 0;
    if (::bind(g_listen, (sockaddr *)&a, sizeof(a)) != 0) fatal("wire: bind failed (%s)", strerror(errno));
    if (::listen(g_listen, 256) != 0) fatal("wire: listen failed (%s)", strerror(errno));
    socklen_t len = sizeof(a);
    if (::getsockname(g_listen, (sockaddr *)&a, &len) != 0) fatal("wire: getsockname failed");
    Endpoint mine;
    memset(&mine, 0, sizeof(mine));
    mine.addr = a.sin_addr.s_addr;
    mine.port = a.sin_port;
    g_ep.assign(r.size, Endpoint());
    boot_allgather(&mine, g_ep.data(), sizeof(Endpoint));
    // the job secret: rank 0's random bytes, through the launcher's allgather
    unsigned char rnd[kSecret] = {0};
    if (r.rank == 0) {
        FILE *f = fopen("/dev/urandom", "rb");
        if (!f || fread(rnd, 1, kSecret, f) != kSecret) fatal("wire: cannot read /dev/urandom");
        fclose(f);
    }
    std::vector<unsigned char> all((size_t)r.size * kSecret);
    boot_allgather(rnd, all.data(), kSecret);
    memcpy(g_secret, all.data(), kSecret);
    g_peer.clear();
    for (int q = 0; q < r.size; ++q) g_peer.emplace_back(new Peer());
    if (::pipe(g_wake) != 0) fatal("wire: pipe failed");
    if (const char *mb = getenv("COMEX_AMD_WIRE_MB")) g_chunk = std::max<size_t>(1, (size_t)atol(mb)) << 20;
    g_active = true;
    g_server = std::thread(server_loop);
}

// ---- initiator side -----------------------------------------------------------
void send_frame(int t, const Frame &f, const void *payload, size_t n) {
    Peer &p = connect_to(t);
    send_all(p.fd, &f, sizeof(f));
    if (n) send_all(p.fd, payload, n);
    p.dirty = true;
}

}  // namespace

bool wire_active() { return g_active; }

void wire_init() {
    Runtime &r = rt();
    // every multi-rank job: the armci_msg messages travel here too, inside a node
    // as between nodes (COMEX_AMD_MSG=0 keeps single-node jobs socket-free; then
    // only the world-group collectives, which use the node shm, are available)
    const char *m = getenv("COMEX_AMD_MSG");
    const bool msg = !(m && atoi(m) == 0);
    if (r.size <= 1 || g_active || (r.nnodes <= 1 && !msg)) return;
    start_sockets();
}

void msg_send(int to, int tag, const void *buf, size_t len) {
    Runtime &r = rt();
    if (to < 0 || to >= r.size) fatal("armci_msg_snd: rank %d out of range", to);
    if (to == r.rank) {
        std::vector<char> d((const char *)buf, (const char *)buf + len);
        msg_push(r.rank, tag, std::move(d));
        return;
    }
    if (!g_active) fatal("armci_msg_snd needs the message transport (COMEX_AMD_MSG=0 disabled it)");
    Frame f = make_frame(W_MSG, to, (uint64_t)(int64_t)tag, nullptr, nullptr, 0);
    f.length = len;
    std::lock_guard<std::mutex> g(g_send_mu);
    send_frame(to, f, buf, len);
}

size_t msg_recv(int from, int tag, void *buf, size_t buflen, int *src) {
    std::unique_lock<std::mutex> g(g_msg_mu);
    for (;;) {
        for (auto it = g_msgs.begin(); it != g_msgs.end(); ++it) {
            if (it->tag != tag || (from >= 0 && it->from != from)) continue;
            if (it->data.size() > buflen)
                fatal("armci_msg_rcv: message of %zu bytes from rank %d, buffer holds %zu", it->data.size(), it->from,
                      buflen);
            const size_t n = it->data.size();
            if (n) memcpy(buf, it->data.data(), n);
            if (src) *src = it->from;
            g_msgs.erase(it);
            return n;
        }
        g_msg_cv.wait(g);
    }
}

uint64_t wire_rmw(int t, int swap, uint64_t addr, int bytes, uint64_t val) {
    Frame f = make_frame(swap ? W_SWAP : W_FETCH_AND_ADD, t, addr, nullptr, nullptr, 0);
    f.length = (uint64_t)bytes;
    memcpy(f.scale, &val, 8);
    std::lock_guard<std::mutex> g(g_send_mu);
    Peer &p = connect_to(t);
    send_all(p.fd, &f, sizeof(f));
    uint64_t old = 0;
    recv_all(p.fd, &old, sizeof(old));
    return old;
}

bool wire_lock(int t, int mutex, bool acquire) {
    Frame f = make_frame(acquire ? W_LOCK : W_UNLOCK, t, (uint64_t)mutex, nullptr, nullptr, 0);
    std::lock_guard<std::mutex> g(g_send_mu);
    Peer &p = connect_to(t);
    send_all(p.fd, &f, sizeof(f));
    char ok = 0;
    recv_all(p.fd, &ok, 1);
    return ok != 0;
}

void wire_finalize() {
    if (!g_active) return;
    Runtime &r = rt();
    for (int t = 0; t < r.size; ++t) {
        Peer &p = *g_peer[t];
        if (p.fd < 0) continue;
        Frame f = make_frame(W_QUIT, t, 0, nullptr, nullptr, 0);
        send_all(p.fd, &f, sizeof(f));
        ::close(p.fd);
        p.fd = -1;
    }
    boot_barrier();   // every initiator has said QUIT; servers may stop
    const char w = 1;
    if (::write(g_wake[1], &w, 1) != 1) fatal("wire: wake failed");
    g_server.join();
    ::close(g_listen);
    ::close(g_wake[0]);
    ::close(g_wake[1]);
    g_listen = g_wake[0] = g_wake[1] = -1;
    for (Pinned &b : g_cli) free_pinned(b);
    for (Pinned &b : g_srv) free_pinned(b);
    g_peer.clear();
    g_ep.clear();
    memset(g_secret, 0, kSecret);
    g_active = false;
}

void wire_detach() {
    if (g_server.joinable()) g_server.detach();
}

void wire_fence(int t) {
    if (!g_active) return;
    Peer &p = *g_peer[t];
    if (p.fd < 0 || !p.dirty) return;
    Frame f = make_frame(W_FENCE, t, 0, nullptr, nullptr, 0);
    send_all(p.fd, &f, sizeof(f));
    char ack = 0;
    recv_all(p.fd, &ack, 1);
    p.dirty = false;
}

void wire_send_strided(int op, const void *scale, const char *src_dev, const int *ss, uint64_t dst,
                       const int *ds, const int *count, int levels, int t) {
    Runtime &r = rt();
    const uint64_t rows = rows_of(count, levels);
    if (!rows) return;
    const uint64_t rowb = (uint64_t)count[0];
    const uint64_t per = std::max<uint64_t>(1, g_chunk / rowb);
    int pstride[8];
    packed_strides(count, levels, pstride);
    const int32_t wop = (op == kOpCopy) ? (levels ? W_PUT_PACKED : W_PUT)
                                        : (levels ? W_ACC_PACKED : W_ACC) + acc_index(op);
    // pack row range k into buffer k % 2 while range k-1 is on the wire
    auto pack = [&](uint64_t rb, uint64_t re, Pinned &b) {
        wait_pinned(b);
        ensure_pinned(b, (re - rb) * rowb);
        std::lock_guard<std::mutex> g(r.launch_mu);
        sched_join();   // after every earlier operation of this rank
        const int rc = launch_strided(kOpCopy, nullptr, src_dev, ss, b.dev - (int64_t)rb * (int64_t)rowb, pstride,
                                      count, levels, r.streams[0], nullptr, rb, re);
        if (rc) fatal("wire: pack launch failed (%d)", rc);
        GA_HIP(hipEventRecord(b.ev, r.streams[0]));
        b.pending = true;
    };
    int cur = 0;
    pack(0, std::min(rows, per), g_cli[0]);
    for (uint64_t rb = 0; rb < rows; rb += per) {
        const uint64_t re = std::min(rows, rb + per);
        if (re < rows) pack(re, std::min(rows, re + per), g_cli[cur ^ 1]);
        Pinned &b = g_cli[cur];
        wait_pinned(b);
        Frame f = make_frame(wop, t, dst, ds, count, levels);
        f.local_address = (uint64_t)(uintptr_t)src_dev;
        f.length = (re - rb) * rowb;
        f.row_begin = rb;
        f.row_end = re;
        if (op != kOpCopy) memcpy(f.scale, scale, (size_t)elem_size(op));
        send_frame(t, f, b.host, f.length);
        cur ^= 1;
    }
}

void wire_get_strided(uint64_t src, const int *ss, char *dst_dev, const int *ds, const int *count, int levels,
                      int t) {
    Runtime &r = rt();
    const uint64_t rows = rows_of(count, levels);
    if (!rows) return;
    const uint64_t rowb = (uint64_t)count[0];
    const uint64_t per = std::max<uint64_t>(1, g_chunk / rowb);
    int pstride[8];
    packed_strides(count, levels, pstride);
    Peer &p = connect_to(t);
    int cur = 0;
    for (uint64_t rb = 0; rb < rows; rb += per) {
        const uint64_t re = std::min(rows, rb + per);
        Frame f = make_frame(levels ? W_GET_PACKED : W_GET, t, src, ss, count, levels);
        f.local_address = (uint64_t)(uintptr_t)dst_dev;
        f.length = (re - rb) * rowb;
        f.row_begin = rb;
        f.row_end = re;
        send_all(p.fd, &f, sizeof(f));
        Pinned &b = g_cli[cur];
        wait_pinned(b);   // its previous unpack has finished
        ensure_pinned(b, f.length);
        recv_all(p.fd, b.host, f.length);
        {
            std::lock_guard<std::mutex> g(r.launch_mu);
            int64_t dlo = 0, dhi = 0;
            side_span_host(ds, count, levels, (int64_t)rowb, &dlo, &dhi);
            Span dsp;
            dsp.lo = (int64_t)(uintptr_t)dst_dev + dlo;
            dsp.hi = (int64_t)(uintptr_t)dst_dev + dhi;
            sched_join_write(dsp);   // dst may be one of our segments
            const int rc = launch_strided(kOpCopy, nullptr, b.dev - (int64_t)rb * (int64_t)rowb, pstride, dst_dev, ds,
                                          count, levels, r.streams[0], nullptr, rb, re);
            if (rc) fatal("wire: unpack launch failed (%d)", rc);
            GA_HIP(hipEventRecord(b.ev, r.streams[0]));
            b.pending = true;
        }
        cur ^= 1;
    }
    wait_pinned(g_cli[0]);
    wait_pinned(g_cli[1]);
}

void wire_send_iov(int op, const void *scale, const uint64_t *src_dev, const uint64_t *dst, int n, int bytes,
                   bool serial, int t) {
    Runtime &r = rt();
    const int per = (int)std::max<uint64_t>(1, g_chunk / ((uint64_t)bytes + 8));
    const int32_t wop = (op == kOpCopy) ? W_PUT_IOV : W_ACC_IOV + acc_index(op);
    for (int i0 = 0; i0 < n; i0 += per) {
        const int m = std::min(per, n - i0);
        const uint64_t loff = iov_list_off(m, bytes);
        const uint64_t len = loff + (uint64_t)m * 8;
        Pinned &b = g_cli[0];
        wait_pinned(b);
        ensure_pinned(b, len);
        // gather the m sources into the data area (the list area holds their addresses first)
        memcpy(b.host + loff, src_dev + i0, (size_t)m * 8);
        uint64_t salign = 0;
        for (int i = 0; i < m; ++i) salign |= src_dev[i0 + i];
        IovDesc d;
        memset(&d, 0, sizeof(d));
        d.src_list = (const uint64_t *)(b.dev + loff);
        d.dst_base = b.dev;
        d.bytes = bytes;
        d.n = (uint32_t)m;
        {
            std::lock_guard<std::mutex> g(r.launch_mu);
            sched_join();
            const int rc = launch_iov(kOpCopy, nullptr, d, salign, false, r.streams[0]);
            if (rc) fatal("wire: io-vector pack failed (%d)", rc);
        }
        GA_HIP(hipStreamSynchronize(r.streams[0]));
        memcpy(b.host + loff, dst + i0, (size_t)m * 8);   // then the target addresses
        Frame f = make_frame(wop, t, 0, nullptr, nullptr, 0);
        f.length = len;
        f.iov_n = m;
        f.iov_bytes = bytes;
        f.iov_serial = serial ? 1 : 0;
        if (op != kOpCopy) memcpy(f.scale, scale, (size_t)elem_size(op));
        send_frame(t, f, b.host, len);
    }
}

void wire_get_iov(const uint64_t *src, const uint64_t *dst_dev, int n, int bytes, int t) {
    Runtime &r = rt();
    const int per = (int)std::max<uint64_t>(1, g_chunk / ((uint64_t)bytes + 8));
    Peer &p = connect_to(t);
    for (int i0 = 0; i0 < n; i0 += per) {
        const int m = std::min(per, n - i0);
        const uint64_t loff = iov_list_off(m, bytes);
        Frame f = make_frame(W_GET_IOV, t, 0, nullptr, nullptr, 0);
        f.length = (uint64_t)m * 8;
        f.iov_n = m;
        f.iov_bytes = bytes;
        send_all(p.fd, &f, sizeof(f));
        send_all(p.fd, src + i0, (size_t)m * 8);
        Pinned &b = g_cli[0];
        wait_pinned(b);
        ensure_pinned(b, loff + (uint64_t)m * 8);
        recv_all(p.fd, b.host, (size_t)m * bytes);
        memcpy(b.host + loff, dst_dev + i0, (size_t)m * 8);
        uint64_t dalign = 0;
        for (int i = 0; i < m; ++i) dalign |= dst_dev[i0 + i];
        IovDesc d;
        memset(&d, 0, sizeof(d));
        d.src_base = b.dev;
        d.dst_list = (const uint64_t *)(b.dev + loff);
        d.bytes = bytes;
        d.n = (uint32_t)m;
        {
            std::lock_guard<std::mutex> g(r.launch_mu);
            Span dsp;   // the listed destinations may lie in our segments
            dsp.lo = INT64_MAX;
            dsp.hi = 0;
            for (int i = 0; i < m; ++i) {
                dsp.lo = std::min(dsp.lo, (int64_t)dst_dev[i0 + i]);
                dsp.hi = std::max(dsp.hi, (int64_t)dst_dev[i0 + i] + bytes);
            }
            sched_join_write(dsp);
            const int rc = launch_iov(kOpCopy, nullptr, d, dalign, false, r.streams[0]);
            if (rc) fatal("wire: io-vector scatter failed (%d)", rc);
        }
        GA_HIP(hipStreamSynchronize(r.streams[0]));
    }
}

}  // namespace gaamd

using namespace gaamd;

// bootstrap + transport self-test without a GPU: every rank sends PING frames
// of several sizes to every other rank and checks the echoed digests.
extern "C" int gaamd_wire_selftest(int rounds) {
    Runtime &r = rt();
    boot_init();
    const bool own = !g_active;
    if (own) start_sockets();
    int bad = 0;
    const size_t sizes[] = {0, 1, 4097, (size_t)1 << 20};
    for (int it = 0; it < rounds; ++it) {
        for (int dq = 1; dq < r.size; ++dq) {
            const int t = (r.rank + dq) % r.size;
            for (size_t n : sizes) {
                std::vector<char> buf(n);
                for (size_t i = 0; i < n; ++i) buf[i] = (char)(i * 131 + r.rank * 7 + it);
                Frame f = make_frame(W_PING, t, 0, nullptr, nullptr, 0);
                f.length = n;
                Peer &p = connect_to(t);
                send_all(p.fd, &f, sizeof(f));
                if (n) send_all(p.fd, buf.data(), n);
                uint64_t h = 0;
                recv_all(p.fd, &h, sizeof(h));
                if (h != (fnv1a(buf.data(), n) ^ (uint64_t)t)) ++bad;
            }
        }
        boot_barrier();
    }
    // a connection without the job secret is closed unanswered
    if (r.size > 1) {
        const int t = (r.rank + 1) % r.size;
        const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
        sockaddr_in a;
        memset(&a, 0, sizeof(a));
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = g_ep[t].addr;
        a.sin_port = g_ep[t].port;
        timeval tv;
        tv.tv_sec = 20;
        tv.tv_usec = 0;
        (void)setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
        if (fd < 0 || ::connect(fd, (sockaddr *)&a, sizeof(a)) != 0) {
            ++bad;
        } else {
            unsigned char wrong[kSecret];
            for (size_t i = 0; i < kSecret; ++i) wrong[i] = (unsigned char)(g_secret[i] ^ 0x5a);
            Frame f = make_frame(W_PING, t, 0, nullptr, nullptr, 0);
            (void)::send(fd, wrong, kSecret, MSG_NOSIGNAL);
            (void)::send(fd, &f, sizeof(f), MSG_NOSIGNAL);
            uint64_t h = 0;
            const ssize_t k = ::recv(fd, &h, sizeof(h), 0);
            // closed (EOF, or a reset because the refused frame was never read) -- not
            // answered, not left hanging until the timeout
            if (k > 0 || (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK))) ++bad;
        }
        if (fd >= 0) ::close(fd);
        boot_barrier();
    }
    if (own) wire_finalize();
    return bad ? -1 : 0;
}

extern "C" int gaamd_node_info(int *node, int *nnodes, int *node_size) {
    Runtime &r = rt();
    if (!r.boot_ready) return -1;
    if (node) *node = r.node;
    if (nnodes) *nnodes = r.nnodes;
    if (node_size) *node_size = r.node_size;
    return 0;
}
