// iov.cpp -- io-vector transfers: comex_accv / putv / getv (include/comex.h).
//
// Reference: comex/src-mpi-pr/comex.c:7327-7400 (nb_accv / nb_putv / nb_getv:
// per-pair nb_acc, or the iov message to the progress rank) and
// _acc_iov_handler 4284-4397.  Here one kernel applies all n pairs of a
// descriptor (k_iov); pairs whose destinations repeat (GA scatter-acc) are
// ordered on the GPU (hashed or radix-sorted runs) or, failing the conditions
// for that, applied one by one in order.  A remote descriptor is packed with its
// owner addresses into staging and applied by the owner's progress thread.
#include "comex_impl.hpp"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

namespace gaamd {

// Reference: comex.c:7327-7400 (nb_accv: per-pair nb_acc, or the iov message to
// the progress rank), _acc_iov_handler 4284-4397.  Here one kernel applies all
// n pairs of a descriptor (k_iov); pairs whose destinations overlap (GA
// scatter-acc duplicates) run one by one in order.
static char *g_iov_scratch = nullptr;
static size_t g_iov_scratch_bytes = 0;
// gaamd_iov_path_counts: local io-vector launches with repeated-destination
// ordering, by path: hashed, hashed + radix fallback (conflicts overflowed), radix
std::atomic<unsigned long long> g_iov_path[4];

static char *g_iov_host = nullptr;
// the partitioned path's overflow flag (mapped pinned; deferred partitions, launch_mu held)
static uint32_t *g_part_flag_host = nullptr, *g_part_flag_dev = nullptr;
static size_t g_iov_host_bytes = 0;

// COMEX_AMD_DEBUG >= 3: the host phases of each io-vector call on stderr (time since
// the previous phase mark; "start" resets)
static void phase(const char *what) {
    if (rt().debug < 3) return;
    static thread_local double last = 0;
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    if (strcmp(what, "start")) trace(3, "iov %-12s %8.1f us", what, (t - last) * 1e6);
    last = t;
}

static char *g_iov_host_dev = nullptr;   // its device view (looked up once per allocation)
static char *iov_host_scratch(size_t bytes) {   // pinned upload staging; caller holds launch_mu
    if (bytes <= g_iov_host_bytes) return g_iov_host;
    if (g_iov_host) GA_HIP(hipHostFree(g_iov_host));
    g_iov_host_bytes = std::max<size_t>(bytes, 1 << 20);
    GA_HIP(hipHostMalloc((void **)&g_iov_host, g_iov_host_bytes, hipHostMallocMapped));
    GA_HIP(hipHostGetDevicePointer((void **)&g_iov_host_dev, g_iov_host, 0));
    return g_iov_host;
}
// the device view of a pinned pointer: inside the upload staging without a runtime call
static char *pinned_dev(const char *p) {
    if (g_iov_host && p >= g_iov_host && p < g_iov_host + g_iov_host_bytes) return g_iov_host_dev + (p - g_iov_host);
    void *dev = nullptr;
    GA_HIP(hipHostGetDevicePointer(&dev, (void *)p, 0));
    return (char *)dev;
}

static char *g_riov_pin = nullptr;   // remote io-vector request upload (pinned)
static size_t g_riov_pin_bytes = 0;
static char *remote_iov_pinned(size_t bytes) {   // caller holds launch_mu; no upload from it in flight
    if (bytes <= g_riov_pin_bytes) return g_riov_pin;
    if (g_riov_pin) GA_HIP(hipHostFree(g_riov_pin));
    g_riov_pin_bytes = std::max<size_t>(bytes, 1 << 20);
    GA_HIP(hipHostMalloc((void **)&g_riov_pin, g_riov_pin_bytes, hipHostMallocMapped));
    return g_riov_pin;
}

// copy `bytes` of the pinned (device-mapped) upload buffer into staging with the
// copy kernel on `st` (one launch, no runtime staging of the host bytes)
static void upload_pinned(char *stage, const char *pin, size_t bytes, hipStream_t st) {
    const char *dev = pinned_dev(pin);
    int count[1] = {(int)bytes};
    const int rc = launch_strided(kOpCopy, nullptr, (const char *)dev, nullptr, stage, nullptr, count, 0, st, nullptr);
    if (rc) fatal("io-vector upload failed (%d)", rc);
}

static char *iov_scratch(size_t bytes) {   // caller holds launch_mu
    if (bytes <= g_iov_scratch_bytes) return g_iov_scratch;
    sched_sync_all();
    if (g_iov_scratch) GA_HIP(hipFree(g_iov_scratch));
    g_iov_scratch_bytes = std::max<size_t>(bytes, 1 << 20);
    GA_HIP(hipMalloc((void **)&g_iov_scratch, g_iov_scratch_bytes));
    return g_iov_scratch;
}

static bool ranges_overlap(std::vector<std::pair<uint64_t, uint64_t>> v) {
    std::sort(v.begin(), v.end());
    for (size_t i = 1; i < v.size(); ++i)
        if (v[i].first < v[i - 1].second) return true;
    return false;
}

// Does any destination repeat?  The destinations are congruent (whole pairs from dlo)
// and fewer than kIovRunsMin: an open-addressing set of their unit indices in a
// thread-local table, a few ns per pair where sorting the pairs took 20-100 us at
// 1-2 Ki pairs.
static bool has_repeat(const uint64_t *dst, int n, uint64_t dlo, int bytes) {
    static thread_local std::vector<uint64_t> tab;
    uint32_t P = 64;
    while (P < 2u * (uint32_t)n) P <<= 1;
    tab.assign(P, 0u);   // 0: empty; unit index + 1 stored
    const bool pow2 = (bytes & (bytes - 1)) == 0;
    const int shift = pow2 ? __builtin_ctz((unsigned)bytes) : 0;
    for (int i = 0; i < n; ++i) {
        const uint64_t off = dst[i] - dlo;
        const uint64_t key = (pow2 ? off >> shift : off / (uint64_t)bytes) + 1u;
        uint32_t h = ((uint32_t)key * 0x9E3779B1u) & (P - 1);
        while (tab[h] != 0) {
            if (tab[h] == key) return true;
            h = (h + 1) & (P - 1);
        }
        tab[h] = key;
    }
    return false;
}

static bool any_cross_overlap(std::vector<std::pair<uint64_t, uint64_t>> a, std::vector<std::pair<uint64_t, uint64_t>> b) {
    std::sort(a.begin(), a.end());
    std::sort(b.begin(), b.end());
    size_t i = 0, j = 0;
    while (i < a.size() && j < b.size()) {
        if (a[i].first < b[j].second && b[j].first < a[i].second) return true;
        if (a[i].second <= b[j].second) ++i; else ++j;
    }
    return false;
}

// Device views of the listed addresses, resolved through a small cache of the
// allocations already seen (one hipPointerGetAttributes per allocation instead of
// per pair: a GA scatter-acc lists up to millions of addresses in a few buffers).
struct ViewCache {
    struct Range { uint64_t lo = 0, hi = 0; int64_t delta = 0; };
    Range r[4];
    uint64_t neg[4] = {~0ull, ~0ull, ~0ull, ~0ull};   // pages known not to be device-accessible
    int next = 0, next_neg = 0;
    bool view(void *p, int bytes, uint64_t *out) {
        const uint64_t a = (uint64_t)(uintptr_t)p;
        for (const Range &x : r)
            if (a >= x.lo && a + (uint64_t)bytes <= x.hi) { *out = (uint64_t)((int64_t)a + x.delta); return true; }
        const uint64_t pg = a & ~(uint64_t)(kPage - 1);
        for (uint64_t q : neg)
            if (q == pg && a + (uint64_t)bytes <= pg + kPage) return false;
        char *d = nullptr;
        if (!direct_view(p, &d)) {
            neg[next_neg] = pg;
            next_neg = (next_neg + 1) % 4;
            return false;
        }
        *out = (uint64_t)(uintptr_t)d;
        hipDeviceptr_t base = nullptr;
        size_t size = 0;
        if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)d) == hipSuccess && size) {
            Range &x = r[next];
            next = (next + 1) % 4;
            x.delta = (int64_t)(uintptr_t)d - (int64_t)a;
            x.lo = (uint64_t)((int64_t)(uintptr_t)base - x.delta);
            x.hi = x.lo + size;
        } else {
            (void)hipGetLastError();
        }
        return true;
    }
    // the allocation holding address a: its range [lo, hi) and device-view offset
    bool range_of(uint64_t a, uint64_t *lo, uint64_t *hi, int64_t *delta) {
        uint64_t d = 0;
        if (!view((void *)(uintptr_t)a, 1, &d)) return false;
        for (const Range &x : r)
            if (a >= x.lo && a < x.hi) { *lo = x.lo; *hi = x.hi; *delta = x.delta; return true; }
        return false;
    }
    // one allocation holding every byte of [lo, hi): its (uniform) device-view offset
    bool span(uint64_t lo, uint64_t hi, int64_t *delta) {
        uint64_t d = 0;
        if (!view((void *)(uintptr_t)lo, 1, &d)) return false;
        for (const Range &x : r)
            if (lo >= x.lo && hi <= x.hi) { *delta = x.delta; return true; }
        return false;
    }
};

// Host passes over io-vector lists (tens of MiB at GA scatter sizes) split into
// contiguous ranges over a few threads: fn(t, i0, i1) for t < T, T = one thread
// per 64 Ki pairs, at most 8 (one per 256 Ki before the pool: interleaved A/B, whole
// calls 256 Ki 0.148 -> 0.110 ms, 1 Mi 0.332 -> 0.30, from host memory 256 Ki 0.418 ->
// 0.284, profiles/r06/host_pool/).  Each range's results are combined by the caller
// in range order, so the outcome does not depend on T.
static int par_threads(long n) {   // one per 64 Ki pairs, at most 8 (the former COMEX_AMD_HOST_THREADS)
    return (int)std::max(1L, std::min(8L, n >> 16));
}
// The ranges run on a few persistent workers (started on first use, blocked on a
// condition variable between calls) and the caller: creating T - 1 threads per pass
// cost more than the pass itself at 256 Ki-1 Mi pairs.  One job at a time (run_mu);
// the workers are never joined (they stay blocked at process exit).
class HostPool {
  public:
    static HostPool &get() {
        static HostPool *p = new HostPool();   // never destroyed: no join at exit
        return *p;
    }
    void run(int T, const std::function<void(int)> &fn) {   // fn(t) for t < T; t = 0 here
        std::lock_guard<std::mutex> one(run_mu_);
        {
            std::lock_guard<std::mutex> g(mu_);
            while ((int)workers_.size() < T - 1) {
                const int id = (int)workers_.size() + 1;
                workers_.emplace_back([this, id] { loop(id); });
            }
            job_ = &fn;
            njobs_ = T;
            pending_ = T - 1;
            ++gen_;
        }
        cv_.notify_all();
        fn(0);
        std::unique_lock<std::mutex> g(mu_);
        done_.wait(g, [this] { return pending_ == 0; });
        job_ = nullptr;
    }

  private:
    void loop(int id) {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> g(mu_);
        for (;;) {
            cv_.wait(g, [&] { return gen_ != seen; });
            seen = gen_;
            if (id >= njobs_) continue;
            const std::function<void(int)> *f = job_;
            g.unlock();
            (*f)(id);
            g.lock();
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> workers_;
    const std::function<void(int)> *job_ = nullptr;
    int njobs_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
};

}  // namespace gaamd

// the pool for callers above the C ABI (the GA layer's gatscat passes)
extern "C" int gaamd_host_parallel(int T, void (*fn)(int t, void *ctx), void *ctx) {
    if (T < 1 || T > 16 || !fn) return -1;
    if (T == 1) {
        fn(0, ctx);
        return 0;
    }
    const std::function<void(int)> job = [&](int t) { fn(t, ctx); };
    gaamd::HostPool::get().run(T, job);
    return 0;
}

namespace gaamd {

template <class F> static void par_for(long n, int T, F fn) {
    if (T <= 1) { fn(0, 0L, n); return; }
    const std::function<void(int)> job = [&](int t) { fn(t, n * t / T, n * (t + 1) / T); };
    HostPool::get().run(T, job);
}

// Is every byte of [lo, hi) ordinary CPU memory of this process (readable, and if
// `write` writable, mappings that are not device files)?  One pass over
// /proc/self/maps replaces a device-view query per page when a whole io-vector
// side lies in pageable host memory (GA's MA buffer `v` of a scatter/gather):
// device allocations are either PROT_NONE reservations or /dev/dri mappings, so
// a side that passes is safe to gather/scatter on the host.  The range may run
// over several adjacent mappings: one buffer is often split into a few VMAs with
// different flags (numpy advises transparent huge pages on the 2 MiB-aligned part
// of an array from 4 MiB up), and a 1 Mi-element scatter whose `v` failed this test
// fell back to the per-page query, 10 ms instead of 1.5 (profiles/r05/scatter).
// Any gap, any address not covered (or a line that does not parse) answers false
// and the per-pair classification decides as before.
std::atomic<unsigned long long> g_iov_host_sides{0};

static bool host_cpu_range(uint64_t lo, uint64_t hi, bool write) {
    if (hi <= lo) return false;
    FILE *f = fopen("/proc/self/maps", "r");
    if (!f) return false;
    char line[512];
    bool ok = false;
    uint64_t need = lo;   // the first byte not yet covered
    while (fgets(line, sizeof(line), f)) {
        const bool whole = strchr(line, '\n') != nullptr;
        unsigned long long a = 0, b = 0;
        char perms[8] = {0};
        int path_at = 0;
        if (sscanf(line, "%llx-%llx %7s %*s %*s %*s %n", &a, &b, perms, &path_at) < 3) break;
        if (need >= a && need < b) {
            const char *path = path_at > 0 ? line + path_at : "";
            if (perms[0] != 'r' || (write && perms[1] != 'w') || strncmp(path, "/dev/", 5) == 0) break;
            if (hi <= b) {
                ok = true;
                break;
            }
            need = b;   // the rest must start exactly where this mapping ends
        } else if (a > need) {
            break;      // a hole: lo not mapped, or a gap after the first part
        }
        while (!whole && fgets(line, sizeof(line), f) && !strchr(line, '\n')) {}   // rest of a long line
    }
    fclose(f);
    if (ok) g_iov_host_sides.fetch_add(1, std::memory_order_relaxed);
    return ok;
}

// gaamd_diag("host_range"): the test hook of host_cpu_range
bool host_cpu_range_probe(uint64_t lo, uint64_t hi, bool write) { return host_cpu_range(lo, hi, write); }

// host-side packing of pageable io-vector runs, in pair order (fixed-size copies
// for the element sizes GA scatters, so the compiler emits plain loads/stores)
template <int B> static void gather_fixed(char *out, void *const *p, int n) {
    for (int i = 0; i < n; ++i) memcpy(out + (size_t)i * B, p[i], B);
}
template <int B> static void scatter_fixed(void *const *p, const char *in, int n) {
    for (int i = 0; i < n; ++i) memcpy(p[i], in + (size_t)i * B, B);
}
static void gather_runs(char *out, void *const *p, int n, int bytes) {
    switch (bytes) {
    case 4: return gather_fixed<4>(out, p, n);
    case 8: return gather_fixed<8>(out, p, n);
    case 16: return gather_fixed<16>(out, p, n);
    }
    for (int i = 0; i < n; ++i) memcpy(out + (size_t)i * bytes, p[i], (size_t)bytes);
}
static void scatter_runs(void *const *p, const char *in, int n, int bytes) {
    switch (bytes) {
    case 4: return scatter_fixed<4>(p, in, n);
    case 8: return scatter_fixed<8>(p, in, n);
    case 16: return scatter_fixed<16>(p, in, n);
    }
    for (int i = 0; i < n; ++i) memcpy(p[i], in + (size_t)i * bytes, (size_t)bytes);
}

// One pass of an io-vector address list: the device-view address of every entry
// into the upload staging, and their OR, OR of XOR with the first, min and max.
// Host-bound at GA scatter sizes (64 Ki pairs: ~85 us per list on one core with
// baseline x86-64 code), so it is built for AVX-512 and AVX2 as well and the
// loader picks the best the host has (GCC function multiversioning).
// Also whether the range continues the progression a0 + i * step from global index
// i0 (*seq_out, 0 or 1): a side that is one contiguous vector of runs in pair order
// (GA's `v` of a scatter from one owner) needs no uploaded list at all.
__attribute__((optimize("O3"), target_clones("avx512f", "avx2", "default")))
static void translate_range(const uint64_t *in, int64_t delta, uint64_t *u, long n, uint64_t a0, long i0,
                            uint64_t step, uint64_t *or_out, uint64_t *xor_out, uint64_t *lo_out, uint64_t *hi_out,
                            uint64_t *seq_out) {
    uint64_t ot = 0, lt = ~0ull, ht = 0, xt = 0, off = 0;
    const uint64_t e0 = a0 + (uint64_t)i0 * step;
    for (long i = 0; i < n; ++i) {
        const uint64_t a = in[i] + (uint64_t)delta;
        u[i] = a;
        ot |= a;
        xt |= a ^ a0;
        off |= a ^ (e0 + (uint64_t)i * step);
        lt = a < lt ? a : lt;
        ht = a > ht ? a : ht;
    }
    *or_out = ot;
    *xor_out = xt;
    *lo_out = lt;
    *hi_out = ht;
    *seq_out = off == 0;
}

// io-vector pairs from this many up have repeated destinations ordered on the GPU (the
// hashed path, or launch_iov_runs) instead of a host-side overlap check (a sort of the
// pairs): whole calls of 4095 pairs took 0.107 ms through the host check against 0.031
// for 4096 on the GPU path, 2048 pairs 0.032 (profiles/r05/iovmid/)
constexpr int kIovRunsMin = 2048;
// io-vectors with at most this many bytes of lists and packed sources skip the upload
constexpr size_t kIovZeroCopyMax = 64 << 10;
// io-vectors from this many pairs try the whole-side host test (host_cpu_range)
constexpr int kIovMapsMin = 65536;

// One descriptor on this GPU.  `src` lists device addresses, or is empty when
// `host_src` holds the n source runs packed on the host (gathered from pageable
// memory by the caller); `dst` lists device addresses, or is empty when the
// results go to the pageable addresses `host_dst` (getv into host memory: copied down
// packed into the pinned staging, then scattered from there on the host).  Reference: nb_accv / nb_putv / nb_getv to a self/SMP target,
// comex.c:7327-7400 (one _acc / memcpy per pair, in order).
// `bounds` (the fast path of xfer_vec): {src lo, src hi, dst lo, dst hi} of the
// allocations the first pair's addresses lie in, with sdelta / ddelta their device-view
// offsets; when some listed address falls outside them the call returns false before
// anything is uploaded or launched (the caller classifies per address instead).
// `src_peer`: the listed sources lie in another GPU's memory (getv): system-scope loads.
static bool iov_local(int cop, const void *scale, const uint64_t *src, const uint64_t *dst, int bytes, int n,
                      const char *host_src = nullptr, void *const *host_dst = nullptr, int64_t sdelta = 0,
                      int64_t ddelta = 0, void *const *gather_src = nullptr, const uint64_t *bounds = nullptr,
                      bool src_peer = false) {
    Runtime &r = rt();
    const bool src_listed = src != nullptr, dst_listed = dst != nullptr;
    // device scratch: [dst list | src list or packed sources | packed results | run-sort work],
    // uploaded from pinned staging; the lists are copied there in the same pass that
    // takes their spans
    const size_t nb = (size_t)n * 8, pk = ((size_t)n * (size_t)bytes + 15) & ~(size_t)15;
    const size_t o_dst = 0, o_src = dst_listed ? nb : 0;
    const size_t o_res = o_src + (src_listed ? nb : pk);
    std::unique_lock<std::mutex> g(r.launch_mu);
    sched_sync_all();   // the previous io-vector kernel and its upload are done with both scratches
    const size_t o_down = (o_res + 255) & ~(size_t)255;   // packed results coming down (host_dst)
    char *up = iov_host_scratch(dst_listed ? o_res : o_down + pk);
    phase("drain");
    uint64_t align_or = 0, slo = ~0ull, shi = 0, dlo = ~0ull, dhi = 0, dxor = 0;
    // translate a list into the staging, taking its OR / min / max and the OR of every
    // address XOR the first one (per range, then combined)
    auto translate = [&](const uint64_t *in, int64_t delta, uint64_t *u, uint64_t *lo_out, uint64_t *hi_out,
                         uint64_t *xor_out, bool *seq) {
        const int T = par_threads(n);
        uint64_t o[8] = {0}, lo[8], hi[8] = {0}, xo[8] = {0}, sq[8] = {0};
        for (int t = 0; t < 8; ++t) lo[t] = ~0ull;
        const uint64_t a0 = in[0] + (uint64_t)delta;
        par_for(n, T, [&](int t, long i0, long i1) {
            translate_range(in + i0, delta, u + i0, i1 - i0, a0, i0, (uint64_t)bytes, &o[t], &xo[t], &lo[t], &hi[t],
                            &sq[t]);
        });
        *seq = true;
        for (int t = 0; t < T; ++t) {
            align_or |= o[t];
            *xor_out |= xo[t];
            *lo_out = std::min(*lo_out, lo[t]);
            *hi_out = std::max(*hi_out, hi[t]);
            *seq = *seq && sq[t];
        }
    };
    uint64_t sxor = 0;
    bool src_seq = false, dst_seq = false;   // a side that is one contiguous vector in pair order
    if (src_listed) {
        translate(src, sdelta, (uint64_t *)(up + o_src), &slo, &shi, &sxor, &src_seq);
        shi += (uint64_t)bytes;
    } else if (gather_src) {
        // pageable sources gathered straight into the pinned staging, in pair order, on
        // the pool (one thread: host-sourced 1 Mi pairs 0.87-0.94 ms against 0.59-0.71,
        // interleaved A/B, profiles/r06/host_pool/; round 1 had measured threads created
        // per call no faster)
        par_for(n, par_threads(n), [&](int, long i0, long i1) {
            gather_runs(up + o_src + i0 * (long)bytes, gather_src + i0, (int)(i1 - i0), bytes);
        });
    } else {
        memcpy(up + o_src, host_src, (size_t)n * (size_t)bytes);
    }
    phase("src side");
    if (dst_listed) {
        translate(dst, ddelta, (uint64_t *)(up + o_dst), &dlo, &dhi, &dxor, &dst_seq);
        dhi += (uint64_t)bytes;
    }
    phase("dst side");
    if (bounds && src_listed && dst_listed &&
        (slo - (uint64_t)sdelta < bounds[0] || shi - (uint64_t)sdelta > bounds[1] ||
         dlo - (uint64_t)ddelta < bounds[2] || dhi - (uint64_t)ddelta > bounds[3]))
        return false;   // an address outside the first pair's allocations: nothing enqueued yet
    // from here on the lists are the translated (device-view) copies in the staging
    if (src_listed) src = (const uint64_t *)(up + o_src);
    if (dst_listed) dst = (const uint64_t *)(up + o_dst);
    bool serial = false, runs = false;
    if (dst_listed) {
        // a source inside a destination: the reference order matters across pairs
        bool cross = false;
        if (src_listed && slo < dhi && dlo < shi) {
            std::vector<std::pair<uint64_t, uint64_t>> sr((size_t)n), dr((size_t)n);
            for (int i = 0; i < n; ++i) {
                sr[i] = {src[i], src[i] + (uint64_t)bytes};
                dr[i] = {dst[i], dst[i] + (uint64_t)bytes};
            }
            cross = any_cross_overlap(sr, dr);
        }
        // every destination a whole number of pairs from dlo (no partial overlaps)
        bool congruent = true;
        if ((bytes & (bytes - 1)) == 0) {
            // all dst[i] == dst[0] (mod bytes), dlo being one of them: from the translate pass
            congruent = (dxor & (uint64_t)(bytes - 1)) == 0;
        } else {
            const FastDiv fd = make_fastdiv((uint32_t)bytes);   // no 64-bit divide per pair
            for (int i = 0; i < n && congruent; ++i) {
                const uint64_t off = dst[i] - dlo;
                congruent = off < (1ull << 32) ? (uint64_t)fd.div((uint32_t)off) * (uint64_t)bytes == off
                                               : off % (uint64_t)bytes == 0;
            }
        }
        const uint64_t units = (dhi - dlo) / (uint64_t)bytes + 1;
        if (cross) {
            serial = true;
        } else if (dst_seq) {
            // one contiguous vector of destinations in pair order: none repeats or overlaps
        } else if (congruent && bytes <= kIovRunsMaxBytes && units <= (1ull << 32)) {
            // destinations on a grid of whole pairs overlap only by repeating: from
            // kIovRunsMin pairs, or when a host hash check finds a repeat among fewer, the
            // GPU orders them (before, a small scatter with one repeated destination went
            // to the one-lane serial kernel)
            runs = n >= kIovRunsMin || has_repeat(dst, n, dlo, bytes);
        } else {
            std::vector<std::pair<uint64_t, uint64_t>> dr((size_t)n);
            for (int i = 0; i < n; ++i) dr[i] = {dst[i], dst[i] + (uint64_t)bytes};
            serial = ranges_overlap(dr);
        }
    }
    phase("classify");
    const size_t o_work = (o_res + (dst_listed ? 0 : pk) + 255) & ~(size_t)255;   // sort work: 256-aligned
    const size_t work = !runs ? 0
                      : std::max(iov_runs_work_bytes((uint32_t)n),
                                 n <= (int)kIovPartMax ? iov_lds_scratch_bytes((uint32_t)n) : (size_t)0);
    char *dev = iov_scratch(o_work + work);
    IovDesc d;
    memset(&d, 0, sizeof(d));
    // sources in one contiguous vector, pair i at src[0] + i * bytes: the kernels read
    // them as a packed side at that device address and the list is not uploaded (half the
    // upload of a scatter-accumulate of GA's `v` into one owner)
    if (src_listed && src_seq) d.src_base = (const char *)(uintptr_t)src[0];
    else if (src_listed) d.src_list = (const uint64_t *)(dev + o_src);
    else d.src_base = dev + o_src;
    if (dst_listed && dst_seq) d.dst_base = (char *)(uintptr_t)dst[0];   // likewise, no list uploaded
    else if (dst_listed) d.dst_list = (const uint64_t *)(dev + o_dst);
    else d.dst_base = dev + o_res;
    d.bytes = bytes;
    d.n = (uint32_t)n;
    Span ss, ds;
    ss.lo = src_listed ? (int64_t)slo : (int64_t)(uintptr_t)(dev + o_src);
    ss.hi = src_listed ? (int64_t)shi : ss.lo + (int64_t)pk;
    ds.lo = dst_listed ? (int64_t)dlo : (int64_t)(uintptr_t)(dev + o_res);
    ds.hi = dst_listed ? (int64_t)dhi : ds.lo + (int64_t)pk;
    const int si = sched_pick(ss, ds);
    // the upload: the copy kernel reading the mapped pinned buffer -- no DMA engine
    // round trip before the first io-vector kernel (64 Ki pairs 0.111-0.120 ms against
    // 0.122-0.130 with the runtime's copy, profiles/r03/s08)
    // the upload: [dst list | src list | packed sources], less a list not needed; on the
    // GPU-ordered path the hashed insert copies the lists itself (one launch less), so only
    // packed sources go up here -- and everything, should that path decline (rc 1 below)
    const size_t up_lo = (dst_listed && dst_seq) ? o_src : 0, up_hi = (src_listed && src_seq) ? o_src : o_res;
    // a small io-vector (at most 64 KiB of lists and packed sources, pairs of at most two
    // 16-byte vectors, no one-lane serial order) is read by its kernel straight from the
    // pinned staging through its device mapping: one launch instead of upload + apply
    const bool zero_copy = !runs && !serial && up_hi - up_lo <= kIovZeroCopyMax && bytes <= 32;
    if (zero_copy) {
        char *up_dev = nullptr;
        up_dev = pinned_dev(up);
        if (d.src_list) d.src_list = (const uint64_t *)(up_dev + o_src);
        else if (!src_listed) d.src_base = up_dev + o_src;
        if (d.dst_list) d.dst_list = (const uint64_t *)(up_dev + o_dst);
    } else if (runs) {
        // (packed sources go up below unless the one-workgroup kernel reads them in place)
    } else if (up_hi > up_lo) {
        upload_pinned(dev + up_lo, up + up_lo, up_hi - up_lo, r.streams[si]);
    }
    const uint64_t units = runs ? (dhi - dlo) / (uint64_t)bytes + 1 : 0;
    int rc;
    if (runs) {
        // repeated destinations: the hashed path (sorts only the pairs that share a
        // destination), or the radix path above 2^19 pairs
        static IovHash *g_hash = nullptr;
        rc = 1;
        char *up_dev = nullptr;   // the device view of the pinned upload buffer
        up_dev = pinned_dev(up);
        if (n <= (int)kIovPartMax && !src_peer && tuning().iov_lds) {
            // up to 4 Mi pairs: ordered in LDS, the destination list read in place from
            // the pinned staging -- below 1 Ki pairs one launch of one workgroup (which
            // reads the sources there too), from 1 Ki the keys and then one workgroup per
            // hash partition
            IovDesc z = d;
            z.dst_list = (const uint64_t *)(up_dev + o_dst);
            // the partitioned path reads sources in destination-hash order, not pair order:
            // a source list or gathered sources go up to HBM first (the copy kernel reads
            // the pinned staging in order) -- read across PCIe in that order, 1 Mi pairs
            // from pageable host memory took 4.2 ms against 1.5 ms uploaded.  (Uploading the
            // destination list too, so that a deferral's radix pass would not bring it across
            // PCIe again, cost random calls more than it saved heavy repeats: 1 Mi pairs
            // 0.37-0.40 ms against 0.32-0.33, profiles/r06/iov_part/to_4mi/)
            const bool src_in_staging = o_res > o_src && !(src_listed && src_seq);
            if (src_in_staging && n >= (int)kIovLdsRoute) {
                upload_pinned(dev + o_src, up + o_src, o_res - o_src, r.streams[si]);
            } else {
                if (d.src_list) z.src_list = (const uint64_t *)(up_dev + o_src);
                else if (!src_listed) z.src_base = up_dev + o_src;
            }
            if (work < iov_lds_scratch_bytes((uint32_t)n)) fatal("io-vector scratch too small for the LDS path");
            // above kIovPartWindowMax pairs, partitions with more pairs than their bucket
            // (heavy repeats) are deferred to the radix path, masked, once the stream is done
            IovPartState ps;
            const bool defer = n > (int)kIovPartWindowMax;
            if (defer) {
                if (!g_part_flag_host) {
                    GA_HIP(hipHostMalloc((void **)&g_part_flag_host, 64, hipHostMallocMapped));
                    GA_HIP(hipHostGetDevicePointer((void **)&g_part_flag_dev, g_part_flag_host, 0));
                }
                *(volatile uint32_t *)g_part_flag_host = 0;
                ps.flag_dev = g_part_flag_dev;
            }
            rc = launch_iov_lds(cop, scale, z, align_or, dlo, units, r.streams[si], false, dev + o_work,
                                defer ? &ps : nullptr);
            if (rc == 0) g_iov_path[3].fetch_add(1, std::memory_order_relaxed);
            if (rc == 0 && defer) {
                GA_HIP(hipStreamSynchronize(r.streams[si]));
                if (*(volatile uint32_t *)g_part_flag_host) {
                    // counted as "lds" and "radix" both
                    if (up_hi > up_lo) upload_pinned(dev + up_lo, up + up_lo, up_hi - up_lo, r.streams[si]);
                    g_iov_path[2].fetch_add(1, std::memory_order_relaxed);
                    rc = launch_iov_runs(cop, scale, d, align_or, dlo, units, dev + o_work, work, r.streams[si],
                                         false, nullptr, &ps);
                }
            }
        }
        if (rc == 1 && !src_listed && o_res > o_src)
            upload_pinned(dev + o_src, up + o_src, o_res - o_src, r.streams[si]);
        if (rc == 1) {
            if (!g_hash) g_hash = iov_hash_create();
            rc = launch_iov_hashed(g_hash, cop, scale, d, align_or, dlo, units, r.streams[si], src_peer,
                                   (const uint64_t *)(up_dev + o_dst),
                                   d.src_list ? (const uint64_t *)(up_dev + o_src) : nullptr);
            if (rc == 0) {
                // more repeated destinations than the hashed launch orders in LDS: after
                // it completed, the radix path applies the pairs it left (the rest masked)
                GA_HIP(hipStreamSynchronize(r.streams[si]));
                const bool over = iov_hash_overflowed(g_hash);
                g_iov_path[over ? 1 : 0].fetch_add(1, std::memory_order_relaxed);
                if (over)
                    rc = launch_iov_runs(cop, scale, d, align_or, dlo, units, dev + o_work, work, r.streams[si],
                                         src_peer, g_hash);
            }
        }
        if (rc == 1) {
            if (up_hi > up_lo) upload_pinned(dev + up_lo, up + up_lo, up_hi - up_lo, r.streams[si]);
            g_iov_path[2].fetch_add(1, std::memory_order_relaxed);
            rc = launch_iov_runs(cop, scale, d, align_or, dlo, units, dev + o_work, work, r.streams[si], src_peer);
        }
    } else {
        rc = launch_iov(cop, scale, d, align_or, serial, r.streams[si], src_peer);
    }
    if (rc) fatal("io-vector launch failed (%d): misaligned elements?", rc);
    phase("launch");
    if (!dst_listed) {
        GA_HIP(hipStreamSynchronize(r.streams[si]));
        phase("kernels");
        GA_HIP(hipMemcpy(up + o_down, dev + o_res, (size_t)n * (size_t)bytes, hipMemcpyDeviceToHost));
        phase("results down");
        par_for(n, par_threads(n), [&](int, long i0, long i1) {
            scatter_runs(host_dst + i0, up + o_down + i0 * (long)bytes, (int)(i1 - i0), bytes);
        });
        phase("host scatter");
    }
    // completion (blocking call) or the handle (non-blocking) is taken by xfer_vec
    return true;
}

int xfer_vec(Xfer kind, int op, void *scale, comex_giov_t *darr, int len, int proc, int group,
             comex_request_t *hdl) {
    ensure_init();
    phase("start");
    Runtime &r = rt();
    const int world = translate_world(group, proc);
    const int cop = (kind == X_ACC) ? op : kOpCopy;
    if (kind == X_ACC && (!elem_size(op) || op == kOpCopy || !scale)) fatal("bad accumulate op/scale");
    for (int k = 0; k < len; ++k) {
        const int n = darr[k].count, bytes = darr[k].bytes;
        if (n <= 0) continue;
        if (bytes <= 0) fatal("io-vector of %d bytes", bytes);
        if (!(kind == X_ACC ? r.acc_iov : (kind == X_PUT ? r.put_iov : r.get_iov)) && !self_smp_route(kind, world)) {
            // COMEX_ENABLE_*_IOV=0: pair by pair as contiguous operations (nb_accv's
            // loop, comex.c:7342-7351)
            ContigWindow w;
            for (int i = 0; i < n; ++i) w.issue(kind, op, scale, darr[k].src[i], darr[k].dst[i], bytes, proc, group);
            w.flush();
            g_toggle[1].fetch_add(1, std::memory_order_relaxed);
            continue;
        }
        const bool remote_side_is_dst = (kind != X_GET);
        // the owner applies it (staging + inbox request): every remote accumulate, and
        // a put into another GPU's memory (no rank writes another GPU's HBM)
        const bool remote_apply = world != r.rank && (kind == X_ACC || (kind == X_PUT && r.peer_src(world)));
        // a getv from another GPU's memory reads it with system-scope loads
        const bool getv_peer = kind == X_GET && world != r.rank && r.peer_src(world);
        // address lists in buffers kept across calls: fresh ones cost a page fault per
        // 512 entries, more than the classification itself at scatter-acc sizes
        static std::vector<uint64_t> g_sv, g_dv;
        if (g_sv.size() < (size_t)n) {
            g_sv.resize((size_t)n);
            g_dv.resize((size_t)n);
        }
        uint64_t *sv = g_sv.data(), *dv = g_dv.data();
        bool host_bounce = false;
        if (world == r.rank) fence_self_if_pending();
        if (world != r.rank && !r.same_node(world)) {
            // another node: one io-vector message per descriptor chunk (wire.cpp)
            for (int i = 0; i < n && !host_bounce; ++i) {
                void *sp = darr[k].src[i], *dp = darr[k].dst[i];
                char *d = nullptr;
                if (remote_side_is_dst) {
                    check_remote(world, dp, 0, bytes);
                    dv[i] = (uint64_t)(uintptr_t)dp;
                    if (direct_view(sp, &d)) sv[i] = (uint64_t)(uintptr_t)d;
                    else host_bounce = true;
                } else {
                    check_remote(world, sp, 0, bytes);
                    sv[i] = (uint64_t)(uintptr_t)sp;
                    if (direct_view(dp, &d)) dv[i] = (uint64_t)(uintptr_t)d;
                    else host_bounce = true;
                }
            }
            if (host_bounce) {
                for (int i = 0; i < n; ++i)
                    xfer_contig(kind, op, scale, darr[k].src[i], darr[k].dst[i], bytes, proc, group, nullptr);
            } else if (kind == X_GET) {
                wire_get_iov(sv, dv, n, bytes, world);
            } else {
                std::vector<std::pair<uint64_t, uint64_t>> dr((size_t)n);
                for (int i = 0; i < n; ++i) dr[i] = {dv[i], dv[i] + (uint64_t)bytes};
                wire_send_iov(cop, scale, sv, dv, n, bytes, ranges_overlap(dr), world);
            }
            continue;
        }
        ViewCache vc;
        if (world == r.rank && n >= 1024) {
            // fast path: each side's addresses all inside one device-accessible allocation
            // (GA's `v` buffer and array block): one range lookup per side, the lists go to
            // the staging translated in the same pass that takes their spans
            const uint64_t *rs = (const uint64_t *)darr[k].src, *rd = (const uint64_t *)darr[k].dst;
            {
                // the allocations of the first pair, checked against every address in the
                // translate pass (no separate min/max pass over both lists)
                uint64_t b[4];
                int64_t sd0 = 0, dd0 = 0;
                if (vc.range_of(rs[0], &b[0], &b[1], &sd0) && vc.range_of(rd[0], &b[2], &b[3], &dd0) &&
                    iov_local(cop, scale, rs, rd, bytes, n, nullptr, nullptr, sd0, dd0, nullptr, b))
                    continue;
            }
            uint64_t smin = ~0ull, smax = 0, dmin = ~0ull, dmax = 0;
            {
                const int T = par_threads(n);
                uint64_t mm[8][4];
                par_for(n, T, [&](int t, long i0, long i1) {
                    uint64_t a0 = ~0ull, a1 = 0, b0 = ~0ull, b1 = 0;
                    for (long i = i0; i < i1; ++i) {
                        a0 = rs[i] < a0 ? rs[i] : a0;
                        a1 = rs[i] > a1 ? rs[i] : a1;
                        b0 = rd[i] < b0 ? rd[i] : b0;
                        b1 = rd[i] > b1 ? rd[i] : b1;
                    }
                    mm[t][0] = a0; mm[t][1] = a1; mm[t][2] = b0; mm[t][3] = b1;
                });
                for (int t = 0; t < T; ++t) {
                    smin = std::min(smin, mm[t][0]);
                    smax = std::max(smax, mm[t][1]);
                    dmin = std::min(dmin, mm[t][2]);
                    dmax = std::max(dmax, mm[t][3]);
                }
            }
            int64_t sdel = 0, ddel = 0;
            const bool sdev = vc.span(smin, smax + (uint64_t)bytes, &sdel);
            const bool ddev = vc.span(dmin, dmax + (uint64_t)bytes, &ddel);
            phase("spans");
            if (sdev && ddev) {
                iov_local(cop, scale, rs, rd, bytes, n, nullptr, nullptr, sdel, ddel);
                continue;
            }
            // one side wholly in pageable host memory (GA's `v`): packed on the host in
            // pair order, as the per-pair classification below would, without it
            if (n >= kIovMapsMin && ddev && !sdev && host_cpu_range(smin, smax + (uint64_t)bytes, false)) {
                phase("host side");
                iov_local(cop, scale, nullptr, rd, bytes, n, nullptr, nullptr, 0, ddel, darr[k].src);
                continue;
            }
            if (n >= kIovMapsMin && sdev && !ddev && cop == kOpCopy &&
                host_cpu_range(dmin, dmax + (uint64_t)bytes, true)) {
                phase("host side");
                iov_local(cop, scale, rs, nullptr, bytes, n, nullptr, darr[k].dst, sdel, 0);
                continue;
            }
        }
        bool src_host = false, dst_host = false;   // a whole side in pageable host memory
        bool classified = false;
        if (remote_apply && n >= kIovMapsMin) {
            // remote accumulate from GA's `v`: a source side in one ordinary host mapping is
            // recognised with one lookup (host_cpu_range) instead of a query per page
            const uint64_t *rs = (const uint64_t *)darr[k].src;
            uint64_t smin = ~0ull, smax = 0;
            for (int i = 0; i < n; ++i) {
                smin = rs[i] < smin ? rs[i] : smin;
                smax = rs[i] > smax ? rs[i] : smax;
            }
            if (host_cpu_range(smin, smax + (uint64_t)bytes, false)) {
                phase("host side");
                src_host = classified = true;
                memcpy(dv, darr[k].dst, (size_t)n * 8);   // owner addresses, checked per chunk below
            }
        }
        phase("fast paths");
        for (int i = 0; i < n && !host_bounce && !classified; ++i) {
            void *sp = darr[k].src[i], *dp = darr[k].dst[i];
            uint64_t v = 0;
            if (world != r.rank && !remote_side_is_dst) {
                sv[i] = (uint64_t)(uintptr_t)remote_view(world, sp, 0, bytes);
            } else if (vc.view(sp, bytes, &v)) {
                if (src_host) host_bounce = true;   // mixed host and device sources
                sv[i] = v;
            } else if (i == 0 || src_host) {
                src_host = true;
            } else {
                host_bounce = true;
            }
            if (world != r.rank && remote_side_is_dst) {
                if (remote_apply) dv[i] = (uint64_t)(uintptr_t)dp;   // owner's address, checked below
                else dv[i] = (uint64_t)(uintptr_t)remote_view(world, dp, 0, bytes);
            } else if (vc.view(dp, bytes, &v)) {
                if (dst_host) host_bounce = true;
                dv[i] = v;
            } else if (i == 0 || dst_host) {
                dst_host = true;
            } else {
                host_bounce = true;
            }
        }
        phase("per pair");
        // packed host side: sources of an accumulate/put (local or same-node put), or the
        // results of a copy (get/put into host memory); an accumulate into host memory
        // needs the old values and stays per pair
        if (src_host && dst_host) host_bounce = true;
        if (dst_host && cop != kOpCopy) host_bounce = true;
        if (!host_bounce && (src_host || dst_host) && !remote_apply) {
            // pageable host runs on one side (GA's MA buffer `v` of a scatter/gather): the
            // sources are gathered on the host and uploaded packed, or the results come
            // back packed and are scattered on the host, in pair order
            if (world != r.rank) fence_target(world);
            if (src_host) {   // gathered straight into the pinned upload staging
                iov_local(cop, scale, nullptr, dv, bytes, n, nullptr, nullptr, 0, 0, darr[k].src);
            } else {
                iov_local(cop, scale, sv, nullptr, bytes, n, nullptr, darr[k].dst, 0, 0, nullptr, nullptr,
                          getv_peer);
            }
            continue;
        }
        if (dst_host) host_bounce = true;   // (a remote accumulate from host sources is gathered below)
        if (host_bounce) {
            // pageable host pairs: per-pair transfers (each maps its pages)
            for (int i = 0; i < n; ++i)
                xfer_contig(kind, op, scale, darr[k].src[i], darr[k].dst[i], bytes, proc, group, nullptr);
            continue;
        }
        if (!remote_apply) {
            if (world != r.rank) fence_target(world);
            iov_local(cop, scale, sv, dv, bytes, n, nullptr, nullptr, 0, 0, nullptr, nullptr, getv_peer);
            continue;
        }
        // remote io-vector accumulate (or put into another GPU): pack the sources + the
        // owner addresses into staging, the owner's progress thread applies them (k_iov)
        drain_target(world);   // its staging ring is allocated and posted in order
        const uint64_t sub = sub_ring_bytes();
        const uint64_t per_pair = (uint64_t)bytes + 8;
        const int pairs_per_req = (int)std::max<uint64_t>(1, (sub - 32) / per_pair);
        for (int i0 = 0; i0 < n; i0 += pairs_per_req) {
            const int m = std::min(pairs_per_req, n - i0);
            uint64_t align_or = 0, dlo = ~0ull, dhi = 0;
            for (int i = 0; i < m; ++i) {
                const uint64_t a = dv[(size_t)i0 + i];
                align_or |= a;
                dlo = std::min(dlo, a);
                dhi = std::max(dhi, a + (uint64_t)bytes);
            }
            // reg_cache_find: one lookup when the chunk's destinations lie in one segment
            // of the owner (a GA block), else one per pair (aborting on a stray address)
            if (segment_of_rank(world, dlo, 0, (int64_t)(dhi - dlo))) {
                (void)remote_view(world, (void *)(uintptr_t)dlo, 0, (int64_t)(dhi - dlo));
            } else {
                for (int i = 0; i < m; ++i)
                    (void)remote_view(world, (void *)(uintptr_t)dv[(size_t)i0 + i], 0, bytes);
            }
            // repeated destinations: the owner orders them on its GPU when every destination
            // is a whole number of pairs from dlo, else a host check picks the serial kernel
            int mode = 0;
            bool congruent = bytes <= kIovRunsMaxBytes && (dhi - dlo) / (uint64_t)bytes < (1ull << 32);
            for (int i = 0; i < m && congruent; ++i) congruent = (dv[(size_t)i0 + i] - dlo) % (uint64_t)bytes == 0;
            if (congruent) {
                // the owner orders repeats on its GPU; fewer pairs with none go plain
                mode = (m >= kIovRunsMin || has_repeat(dv + i0, m, dlo, bytes)) ? 2 : 0;
            } else {
                std::vector<std::pair<uint64_t, uint64_t>> dr((size_t)m);
                for (int i = 0; i < m; ++i) dr[i] = {dv[(size_t)i0 + i], dv[(size_t)i0 + i] + (uint64_t)bytes};
                mode = ranges_overlap(dr) ? 1 : 0;
            }
            const uint64_t loff = iov_list_off(m, bytes);
            const uint64_t len_b = loff + (uint64_t)m * 8;
            const uint64_t off = stage_alloc(world, ring_len(len_b));
            char *stage = r.staging + (size_t)world * sub + off;
            {
                std::lock_guard<std::mutex> g(r.launch_mu);
                // the request's bytes (packed host sources, owner addresses) go up from
                // pinned memory; the previous request's upload from this buffer
                // completed before its post
                char *pin = remote_iov_pinned((size_t)len_b);
                memcpy(pin + loff, dv + i0, (size_t)m * 8);
                if (src_host) {
                    // pageable sources (GA's MA buffer): gathered on the host (on the pool),
                    // one upload
                    void *const *sp = darr[k].src + i0;
                    par_for(m, par_threads(m), [&](int, long j0, long j1) {
                        gather_runs(pin + j0 * (long)bytes, sp + j0, (int)(j1 - j0), bytes);
                    });
                    sched_join();
                    upload_pinned(stage, pin, (size_t)len_b, r.streams[0]);
                } else {
                    char *dev = iov_scratch((size_t)m * 8);
                    sched_sync_all();
                    GA_HIP(hipMemcpy(dev, sv + i0, (size_t)m * 8, hipMemcpyHostToDevice));
                    uint64_t salign = 0;
                    for (int i = 0; i < m; ++i) salign |= sv[(size_t)i0 + i];
                    IovDesc d;
                    memset(&d, 0, sizeof(d));
                    d.src_list = (const uint64_t *)dev;
                    d.dst_base = stage;
                    d.bytes = bytes;
                    d.n = (uint32_t)m;
                    sched_join();
                    const int rc = launch_iov(kOpCopy, nullptr, d, salign, false, r.streams[0]);
                    if (rc) fatal("io-vector pack failed (%d)", rc);
                }
                if (!src_host) upload_pinned(stage + loff, pin + loff, (size_t)m * 8, r.streams[0]);
                GA_HIP(hipStreamSynchronize(r.streams[0]));
            }
            const uint64_t seq = ++r.posted[world];
            g_pend[world].push_back({seq, off, ring_len(len_b)});
            r.stage_head[world] = off + ring_len(len_b);
            post_request_iov(world, op, scale, bytes, m, (uint64_t)world * sub + off, len_b, dlo, dhi, align_or,
                             mode);
        }
    }
    // io-vector kernels may sit on any library stream (sched_pick per descriptor):
    // a handle is recorded after a join, so it covers all of them; a blocking call
    // completes locally before returning
    // (a blocking call completes by synchronising the streams: the completion flag the
    // strided calls wait on measured 7-18 us SLOWER here, interleaved A/B,
    // profiles/r06/iov_flag_ab/ -- the io-vector kernels read the lists across PCIe from
    // pinned memory while the host polls a pinned flag)
    const bool blocking = !hdl && r.blocking_sync;
    {
        std::lock_guard<std::mutex> g(r.launch_mu);
        if (hdl) sched_join();
        else if (blocking) sched_sync_all();
    }
    phase("complete");
    if (world != r.rank && r.same_node(world) && kind != X_ACC && !blocking && !r.direct_pending.empty())
        r.direct_pending[world] = 1;
    if (hdl) nb_complete_now(hdl, 0, true);
    return COMEX_SUCCESS;
}


void iov_finalize() {
    if (g_iov_scratch) (void)hipFree(g_iov_scratch);
    g_iov_scratch = nullptr;
    g_iov_scratch_bytes = 0;
    if (g_iov_host) (void)hipHostFree(g_iov_host);
    g_iov_host = g_iov_host_dev = nullptr;
    g_iov_host_bytes = 0;
    if (g_riov_pin) (void)hipHostFree(g_riov_pin);
    g_riov_pin = nullptr;
    g_riov_pin_bytes = 0;
    if (g_part_flag_host) (void)hipHostFree(g_part_flag_host);
    g_part_flag_host = g_part_flag_dev = nullptr;
    iov_part_release();
}

}  // namespace gaamd
