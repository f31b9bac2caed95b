// gaamd_iov.hip -- gfx950 io-vector kernels (comex_accv / putv / getv,
// comex/src-mpi-pr/comex.c:7327-7400; the owner side _acc_iov_handler 4284-4397)
// and their ordering machinery for repeated destinations: the hashed LDS path
// and the library's own stable LSD radix sort.
#include "gaamd_device.hpp"
#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

namespace gaamd {

// ---------------------------------------------------------------------------
// I/O-vector kernels: n (src[i], dst[i]) pairs of `bytes` each -- comex_accv /
// putv / getv (comex/src-mpi-pr/comex.c:7327-7400; the server side
// _acc_iov_handler 4284-4397).  A side is either a device array of n 64-bit
// addresses or one packed buffer (address = base + i*bytes).  Vectors of all
// pairs are flattened so short pairs (GA scatter-acc: one element each) still
// fill every lane.
// SYS: the sources lie in a peer GPU's memory (getv from another device):
// system-scope source loads, as the strided kernels' vload_sys
template <int W, bool SYS>
__device__ __forceinline__ typename Vec<W>::T src_load(const char *p) {
    if constexpr (SYS) return vload_sys<W>(p);
    else return vload<W, false>(p);
}

// Applies `cnt` pairs that share ONE destination dp, pair idx(0) first: the destination
// is read once, the pairs are applied in a register in that order and the result stored
// once.  The same operations on the same values in the same order as one read-modify-
// write per pair (the reference's, comex.c:7342-7351), so bit-exact, but a run of r pairs
// costs r independent source loads (16 in flight) and one round trip to the destination
// instead of r dependent round trips (round 6: a heavy-repeat scatter -- 200 slots for
// 64 Ki pairs -- spent its time in exactly that chain).  Sources never overlap the
// destinations on the ordered paths (the host sends such calls to the serial kernel).
template <class OP, int W, bool SYS, class IDX>
__device__ __forceinline__ void iov_apply_chain(const IovDesc &d, const OP &op, char *dp, uint32_t cnt, IDX idx) {
    typedef typename Vec<W>::T V;
    auto src = [&](uint32_t j) -> const char * {
        const uint32_t i = idx(j);
        return d.src_list ? (const char *)d.src_list[i] : d.src_base + (size_t)i * d.bytes;
    };
    for (uint32_t v = 0; v < d.nvec; ++v) {
        V y{};
        if constexpr (OP::kReadsDst) y = vload<W, false>(dp + (size_t)v * W);
        uint32_t j = 0;
        constexpr uint32_t B = 16, b = 4;
        if (cnt >= B) {
            // software-pipelined: the next batch's source addresses (the index loads) are
            // in flight with this batch's source loads
            const char *sp[B];
#pragma unroll
            for (uint32_t k = 0; k < B; ++k) sp[k] = src(k);
            for (; j + B <= cnt; j += B) {
                V x[B];
#pragma unroll
                for (uint32_t k = 0; k < B; ++k) x[k] = src_load<W, SYS>(sp[k] + (size_t)v * W);
                if (j + 2 * B <= cnt) {
#pragma unroll
                    for (uint32_t k = 0; k < B; ++k) sp[k] = src(j + B + k);
                }
#pragma unroll
                for (uint32_t k = 0; k < B; ++k) y = op.template apply<W>(y, x[k]);
            }
        }
        for (; j + b <= cnt; j += b) {
            V x[b];
#pragma unroll
            for (uint32_t k = 0; k < b; ++k) x[k] = src_load<W, SYS>(src(j + k) + (size_t)v * W);
#pragma unroll
            for (uint32_t k = 0; k < b; ++k) y = op.template apply<W>(y, x[k]);
        }
        for (; j < cnt; ++j) y = op.template apply<W>(y, src_load<W, SYS>(src(j) + (size_t)v * W));
        vstore<W, false>(dp + (size_t)v * W, y);
    }
}

template <class OP, int W, int U, bool SYS = false>
__global__ __launch_bounds__(256) void k_iov(const IovDesc d, const OP op) {
    typedef typename Vec<W>::T V;
    const uint32_t span = 256u * U;
    for (uint32_t base = blockIdx.x * span; base < d.items; base += gridDim.x * span) {
        V a[U], b[U];
        char *dps[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const uint32_t g = base + threadIdx.x + (uint32_t)(k * 256);
            dps[k] = nullptr;
            if (g < d.items) {
                const uint32_t i = d.nvec_div.div(g);
                const uint32_t v = g - i * d.nvec;
                const char *sp = d.src_list ? (const char *)d.src_list[i] : d.src_base + (size_t)i * d.bytes;
                char *dp = d.dst_list ? (char *)d.dst_list[i] : d.dst_base + (size_t)i * d.bytes;
                dps[k] = dp + (size_t)v * W;
                a[k] = src_load<W, SYS>(sp + (size_t)v * W);
                if constexpr (OP::kReadsDst) b[k] = vload<W, false>(dps[k]);
            }
        }
#pragma unroll
        for (int k = 0; k < U; ++k)
            if (dps[k]) vstore<W, false>(dps[k], op.template apply<W>(b[k], a[k]));
    }
}

// pairs in reference order when destinations overlap (duplicates in a scatter-acc)
template <class OP, int W, bool SYS = false>
__global__ __launch_bounds__(64) void k_iov_serial(const IovDesc d, const OP op) {
    if (threadIdx.x != 0) return;
    for (uint32_t i = 0; i < d.n; ++i) {
        const char *sp = d.src_list ? (const char *)d.src_list[i] : d.src_base + (size_t)i * d.bytes;
        char *dp = d.dst_list ? (char *)d.dst_list[i] : d.dst_base + (size_t)i * d.bytes;
        for (uint32_t v = 0; v < d.nvec; ++v) {
            typename Vec<W>::T x = src_load<W, SYS>(sp + (size_t)v * W), y = x;
            if constexpr (OP::kReadsDst) y = vload<W, false>(dp + (size_t)v * W);
            vstore<W, false>(dp + (size_t)v * W, op.template apply<W>(y, x));
        }
    }
}

constexpr uint32_t kIovRunSkip = 0xffffffffu;   // k_iov_runs: a run of this key was applied already

// the hashed path's state for one launch (see k_iovh_insert below)
struct IovHashArgs {
    bool lds;              // k_iov_lds (one workgroup) instead of the hashed apply + conflicts
    uint32_t part_lg;      // > 0 with part_keys: k_iov_keyof + k_iov_part on 2^part_lg partitions
    uint32_t *part_keys;   // their scratch: keys (4 bytes a pair) and buckets; counters in `count`
    uint64_t dlo;
    uint32_t shift;
    bool pow2;
    uint32_t epoch;
    const uint32_t *dup;
    const uint32_t *slot;
    uint64_t *conf;
    uint32_t *count, *overflow;   // partitioned path: its counters, and (deferring) the overflow flag
};

// launch_iov_runs: sort keys = destination index relative to dlo, values = pair index
__global__ __launch_bounds__(256) void k_iov_keys(const uint64_t *dst_list, uint64_t dlo, uint32_t bytes, uint32_t n,
                                                  uint32_t *keys, uint32_t *vals) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    keys[i] = (uint32_t)((dst_list[i] - dlo) / bytes);
    vals[i] = i;
}

// one lane per distinct destination (the first sorted position of its run)
// applies the run's pairs in input order
template <class OP, int W, bool SYS = false>
__global__ __launch_bounds__(256) void k_iov_runs(const IovDesc d, const OP op) {
    const uint32_t j0 = blockIdx.x * 256u + threadIdx.x;
    if (j0 >= d.n) return;
    const uint32_t key = d.run_key[j0];
    if (key == kIovRunSkip || (j0 > 0 && d.run_key[j0 - 1] == key)) return;
    // the run's end: galloping, then a binary search (keys are sorted) -- a long run
    // (thousands of pairs on one destination) no longer walks its keys one by one
    uint32_t lo = j0 + 1, hi = j0 + 1, step = 1;   // run_key[lo - 1] == key
    while (hi < d.n && d.run_key[hi] == key) {
        lo = hi + 1;
        hi = (d.n - hi > step) ? hi + step : d.n;
        step <<= 1;
    }
    while (lo < hi) {                                // first position past the run in [lo, hi]
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if (d.run_key[mid] == key) lo = mid + 1;
        else hi = mid;
    }
    const uint32_t cnt = lo - j0;
    const uint32_t *perm = d.run_perm + j0;
    iov_apply_chain<OP, W, SYS>(d, op, (char *)d.dst_list[perm[0]], cnt, [&](uint32_t j) { return perm[j]; });
}

// ---------------------------------------------------------------------------
// Hashed io-vector path (the radix sort is 8 launches,
// ~40 us at 64 Ki pairs).  Only repeated destinations need ordering, and in a
// scatter they are rare, so:
//   k_iovh_insert : every pair's unit key = (dst - dlo) / bytes goes into an
//                   open-addressing table (tag = epoch:key, no clearing between
//                   calls); the lane whose compare-and-swap claims a slot is its
//                   key's first pair, any other lane that finds the key there marks
//                   the slot repeated (dup[slot] = epoch) -- one load and one CAS for
//                   a destination that does not repeat (round 5; an atomicMin and an
//                   atomicMax of epoch-tagged pair indices on every pair before: the
//                   insert of 16 Ki pairs took 13.7 us, profiles/r05/ivt)
//   k_iovh_apply  : a pair whose slot is not marked repeated is its destination's
//                   only pair: applied at once; the others are appended to a
//                   conflict list as key:index
//   k_iovh_conf   : one workgroup sorts the conflict list in LDS (bitonic, by
//                   key then index) and one lane per distinct key applies its
//                   pairs in index order -- the reference's order
// More conflicts than the LDS holds (heavy repeats, a histogram-like scatter):
// k_iovh_conf applies nothing and raises a flag; the caller, after the stream
// completed, runs launch_iov_runs with the table as a mask (pairs already
// applied get the sentinel key and are skipped).
constexpr uint32_t kIovhCap = 8192;          // conflict entries sorted in LDS (64 KiB)
constexpr uint32_t kIovhBS = 64;             // insert / apply block: one wave, spread over more CUs
constexpr uint32_t kIovhMaxPairs = 1u << 19;  // above: the radix path (1 Mi random pairs overflow the LDS list)

struct IovHash {
    char *mem = nullptr;          // keys (8 B x P) | dup (4 B x P) | slot (n) | conflicts (cap) | count
    size_t bytes = 0;
    uint32_t P = 0;               // table slots (power of two >= 2n)
    uint32_t npairs = 0;          // capacity of the slot array
    uint32_t epoch = 0;
    uint32_t *flag_host = nullptr, *flag_dev = nullptr;   // overflow flag (mapped pinned)
    uint64_t dlo = 0;
    uint32_t n = 0, shift = 0;    // the last hashed launch (for the masked fallback)
    bool pow2 = false;
};

IovHash *iov_hash_create() { return new IovHash(); }

// where the slot array starts in IovHash::mem (after the keys and the dup marks)
static size_t iovh_off_slot(uint32_t P) { return ((size_t)P * 12 + 255) & ~(size_t)255; }

static __device__ __forceinline__ uint32_t iovh_slot0(uint32_t key, uint32_t mask) {
    return (key * 0x9E3779B1u) & mask;
}

// dst_in / src_in (optional): the address lists still in the caller's mapped pinned
// buffer -- read here over PCIe and written to dst_list / src_out in HBM for the kernels
// after this one, which saves the separate upload launch (7-16 us, profiles/r05/ivt)
__global__ __launch_bounds__(kIovhBS) void k_iovh_insert(uint64_t *dst_list, uint64_t dlo, uint32_t bytes,
                                                     uint32_t shift, bool pow2, uint32_t n, uint64_t *keys,
                                                     uint32_t *dup, uint32_t mask, uint32_t epoch, uint32_t *slot,
                                                     uint32_t *count, const uint64_t *dst_in, const uint64_t *src_in,
                                                     uint64_t *src_out) {
    const uint32_t i = blockIdx.x * kIovhBS + threadIdx.x;
    if (i == 0) *count = 0;   // the conflict list of this call (k_iovh_apply runs after this kernel)
    if (i >= n) return;
    if (src_in) src_out[i] = src_in[i];
    uint64_t a;
    if (dst_in) {
        a = dst_in[i];
        dst_list[i] = a;
    } else {
        a = dst_list[i];
    }
    const uint64_t off = a - dlo;
    const uint32_t key = (uint32_t)(pow2 ? (off >> shift) : off / bytes);
    const uint64_t tag = ((uint64_t)epoch << 32) | key;
    uint32_t h = iovh_slot0(key, mask);
    bool repeated = false;
    for (;;) {
        const uint64_t cur = __hip_atomic_load(keys + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == tag) {                        // another pair of this call holds the key
            repeated = true;
            break;
        }
        if ((uint32_t)(cur >> 32) != epoch) {   // empty this call (an earlier call's tag): claim it
            const uint64_t old = atomicCAS((unsigned long long *)(keys + h), cur, tag);
            if (old == cur) break;               // claimed: the first pair of this key
            if (old == tag) {                    // claimed by another pair of the same key meanwhile
                repeated = true;
                break;
            }
            if ((uint32_t)(old >> 32) != epoch) continue;   // another stale value: try again here
        }
        h = (h + 1) & mask;                      // a different key of this call: probe on
    }
    slot[i] = h;
    if (repeated) __hip_atomic_store(dup + h, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <class OP, int W, bool SYS>
__device__ __forceinline__ void iov_apply_pair(const IovDesc &d, const OP &op, uint32_t i) {
    const char *sp = d.src_list ? (const char *)d.src_list[i] : d.src_base + (size_t)i * d.bytes;
    char *dp = (char *)d.dst_list[i];
    for (uint32_t v = 0; v < d.nvec; ++v) {
        typename Vec<W>::T x = src_load<W, SYS>(sp + (size_t)v * W), y = x;
        if constexpr (OP::kReadsDst) y = vload<W, false>(dp + (size_t)v * W);
        vstore<W, false>(dp + (size_t)v * W, op.template apply<W>(y, x));
    }
}

template <class OP, int W, bool SYS>
__global__ __launch_bounds__(kIovhBS) void k_iovh_apply(const IovDesc d, const OP op, uint64_t dlo, uint32_t shift,
                                                    bool pow2, uint32_t epoch, const uint32_t *dup,
                                                    const uint32_t *slot, uint64_t *conf, uint32_t *count) {
    const uint32_t i = blockIdx.x * kIovhBS + threadIdx.x;
    if (i >= d.n) return;
    const uint32_t h = slot[i];
    if (dup[h] != epoch) {
        iov_apply_pair<OP, W, SYS>(d, op, i);
        return;
    }
    const uint64_t off = d.dst_list[i] - dlo;
    const uint32_t key = (uint32_t)(pow2 ? (off >> shift) : off / (uint64_t)d.bytes);
    const uint32_t pos = atomicAdd(count, 1u);
    if (pos < kIovhCap) conf[pos] = ((uint64_t)key << 32) | i;
}

template <class OP, int W, bool SYS>
__global__ __launch_bounds__(1024) void k_iovh_conf(const IovDesc d, const OP op, const uint64_t *conf,
                                                    const uint32_t *count, uint32_t *overflow) {
    __shared__ uint64_t s[kIovhCap];
    const uint32_t m = *count;
    if (m == 0) return;
    if (m > kIovhCap) {
        if (threadIdx.x == 0) *overflow = 1;
        return;
    }
    uint32_t P = 1;
    while (P < m) P <<= 1;
    for (uint32_t t = threadIdx.x; t < P; t += 1024) s[t] = t < m ? conf[t] : ~0ull;
    __syncthreads();
    for (uint32_t k = 2; k <= P; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = threadIdx.x; t < P; t += 1024) {
                const uint32_t l = t ^ j;
                if (l > t) {
                    const uint64_t a = s[t], b = s[l];
                    const bool up = (t & k) == 0;
                    if ((a > b) == up) {
                        s[t] = b;
                        s[l] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t t = threadIdx.x; t < m; t += 1024) {
        const uint32_t key = (uint32_t)(s[t] >> 32);
        if (t > 0 && (uint32_t)(s[t - 1] >> 32) == key) continue;
        uint32_t cnt = 1;
        while (t + cnt < m && (uint32_t)(s[t + cnt] >> 32) == key) ++cnt;
        iov_apply_chain<OP, W, SYS>(d, op, (char *)d.dst_list[(uint32_t)s[t]], cnt,
                                    [&](uint32_t j) { return (uint32_t)s[t + j]; });
    }
}

// ---------------------------------------------------------------------------
// One-workgroup io-vector path: up to kIovLdsMax pairs whose
// destinations may repeat are ordered AND applied by one launch of one 1024-thread
// workgroup, everything it orders held in LDS, instead of the hashed path's three
// launches (insert, apply, conflicts: 17.6 + 5.1 + 4.1 us at 16 Ki pairs,
// profiles/r05/iov3) with their device-scope atomics on an HBM table.
//   keys  : each pair's destination unit (dst - dlo) / bytes, read once from the
//           list (through the mapped pinned staging: no upload launch)
//   table : open addressing, 2^15 16-bit slots (pair index; top bit: the slot's key
//           has more than one pair), claimed with an LDS compare-and-swap
//   apply : a pair alone on its destination is applied at once, its vectors spread
//           over all lanes; the pairs of repeated destinations are listed (over the
//           table, no longer needed), sorted by (key, index) with an LDS bitonic sort,
//           and each destination's pairs applied in index order by one lane -- the
//           reference's order (comex.c:7342-7351: one _acc per pair, in order).
// A destination is rebuilt from its key (dlo + key * bytes: the caller guarantees
// every destination a whole number of pairs from dlo), so the list is read once.
// Where it pays (round 6, tools/iov_lds_probe.cpp, profiles/r06/iov_lds/): small
// io-vectors.  Kernel time, random single-f64 destinations in 1 GiB, back-to-back
// launches: 1 Ki pairs 5.9 us against 11.5 for the hashed path's three launches, 2 Ki 8.4
// against 13.0, 4 Ki 13.4 against 13.8 -- and then 26 against 19 at 8 Ki, 76 against 18
// at 16 Ki: one CU cannot keep enough random destinations in flight.  From 1 Ki pairs the
// partitioned path below is used instead (about the same at 1 Ki, faster above, and far
// faster on heavy repeats: 200 destinations, 2 Ki pairs 23 us against 62 here).
constexpr uint32_t kIovLdsLog = 15;                       // table slots: 2^15 = 2 x pairs
constexpr uint32_t kIovLdsEmpty = 0xffffu;

__device__ __forceinline__ const char *iov_lds_src(const IovDesc &d, uint32_t i) {
    return d.src_list ? (const char *)__builtin_nontemporal_load(d.src_list + i) : d.src_base + (size_t)i * d.bytes;
}

template <class OP, int W, bool SYS>
__device__ __forceinline__ void iov_lds_pair(const IovDesc &d, const OP &op, uint32_t i, char *dp) {
    const char *sp = iov_lds_src(d, i);
    for (uint32_t v = 0; v < d.nvec; ++v) {
        typename Vec<W>::T x = src_load<W, SYS>(sp + (size_t)v * W), y = x;
        if constexpr (OP::kReadsDst) y = vload<W, false>(dp + (size_t)v * W);
        vstore<W, false>(dp + (size_t)v * W, op.template apply<W>(y, x));
    }
}

// Double hashing: a key's probe step is odd (so it visits every slot of the power-of-two
// table) and depends on the key.  Linear probing (step 1) let clusters grow at the
// table's load of one half: with random destinations every 64-lane wave waited for its
// longest probe, and marking 16 Ki keys took 37 us against 8 for keys that never collide
// (tools/lds_mark_probe.hip, profiles/r06/iov_lds/lds_mark_*.jsonl).
__device__ __forceinline__ uint32_t iov_lds_step(uint32_t key) {
    return ((key * 0x85EBCA6Bu) >> (32 - kIovLdsLog)) | 1u;
}

// the LDS table of k_iov_lds: keys[0..n) in LDS -> rep (bit i: pair i's
// destination has more than one pair).  Insert: the lane whose compare-and-swap claims
// an empty slot is its key's first pair; a lane that finds its key in a slot marks that
// slot repeated.  Then every pair looks its key up again and copies the mark.  (Every
// lane with a given key walks the same probe sequence, so they meet at its first empty
// slot; no slot is emptied again, so the lookup finds the key before any empty slot.)
__device__ __forceinline__ void iov_lds_mark(const uint32_t *keys, uint32_t *tab, uint32_t *rep, uint32_t n) {
    const uint32_t t = threadIdx.x;
    constexpr uint32_t mask = (1u << kIovLdsLog) - 1u;
    for (uint32_t i = t; i < n; i += 1024) {
        const uint32_t key = keys[i];
        uint32_t h = (key * 0x9E3779B1u) >> (32 - kIovLdsLog);
        const uint32_t step = iov_lds_step(key);
        for (;;) {
            uint32_t *wp = &tab[h >> 1];
            const uint32_t sh = (h & 1u) * 16u;
            const uint32_t cur = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint32_t e = (cur >> sh) & 0xffffu;
            if (e == kIovLdsEmpty) {
                if (atomicCAS(wp, cur, (cur & ~(0xffffu << sh)) | (i << sh)) == cur) break;
                continue;                                   // the word changed under us: look again
            }
            if (keys[e & 0x7fffu] == key) {
                atomicOr(wp, 0x8000u << sh);
                break;
            }
            h = (h + step) & mask;
        }
    }
    __syncthreads();
    for (uint32_t i = t; i < n; i += 1024) {
        const uint32_t key = keys[i];
        uint32_t h = (key * 0x9E3779B1u) >> (32 - kIovLdsLog), e;
        const uint32_t step = iov_lds_step(key);
        for (;; h = (h + step) & mask) {
            e = (tab[h >> 1] >> ((h & 1u) * 16u)) & 0xffffu;
            if (keys[e & 0x7fffu] == key) break;            // the key's slot (it was inserted)
        }
        if (e & 0x8000u) atomicOr(&rep[i >> 5], 1u << (i & 31u));
    }
    __syncthreads();
}

// the listed pairs of repeated destinations conf[0..m), sorted by (key, pair index) with
// an LDS bitonic sort, then one lane per destination applies its pairs in index order
template <class OP, int W, bool SYS>
__device__ __forceinline__ void iov_lds_runs(const IovDesc &d, const OP &op, uint64_t dlo, const uint32_t *keys,
                                             uint32_t *conf, uint32_t m) {
    const uint32_t t = threadIdx.x;
    if (m == 0) return;
    uint32_t P = 1;
    while (P < m) P <<= 1;
    for (uint32_t u = m + t; u < P; u += 1024) conf[u] = 0xffffffffu;   // sorts last
    __syncthreads();
    for (uint32_t k = 2; k <= P; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t u = t; u < P; u += 1024) {
                const uint32_t l = u ^ j;
                if (l <= u) continue;
                const uint32_t x = conf[u], y = conf[l];
                const bool gt = x == 0xffffffffu ? y != 0xffffffffu
                              : y == 0xffffffffu ? false
                              : (keys[x] != keys[y] ? keys[x] > keys[y] : x > y);
                if (gt == ((u & k) == 0)) {
                    conf[u] = y;
                    conf[l] = x;
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t u = t; u < m; u += 1024) {
        const uint32_t key = keys[conf[u]];
        if (u > 0 && keys[conf[u - 1]] == key) continue;
        char *dp = (char *)(dlo + (uint64_t)key * (uint64_t)d.bytes);
        uint32_t cnt = 1;
        while (u + cnt < m && keys[conf[u + cnt]] == key) ++cnt;
        iov_apply_chain<OP, W, SYS>(d, op, dp, cnt, [&](uint32_t j) { return conf[u + j]; });
    }
}

template <class OP, int W, bool SYS>
__global__ __launch_bounds__(1024) void k_iov_lds(const IovDesc d, const OP op, uint64_t dlo, uint32_t shift,
                                                  bool pow2) {
    __shared__ uint32_t keys[kIovLdsMax];
    __shared__ uint32_t tab[(1u << kIovLdsLog) / 2];      // two 16-bit slots per word; later the conflict list
    __shared__ uint32_t rep[kIovLdsMax / 32];             // pair i's destination repeats
    __shared__ uint32_t nconf;
    const uint32_t t = threadIdx.x, n = d.n;
    for (uint32_t w = t; w < (1u << kIovLdsLog) / 2; w += 1024) tab[w] = 0xffffffffu;
    for (uint32_t w = t; w < kIovLdsMax / 32; w += 1024) rep[w] = 0;
    if (t == 0) nconf = 0;
    {
        // every list load of this lane in flight at once
        constexpr int K = kIovLdsMax / 1024;
        uint32_t kk[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t i = t + (uint32_t)k * 1024u;
            const uint64_t off = i < n ? __builtin_nontemporal_load(d.dst_list + i) - dlo : 0;
            kk[k] = (uint32_t)(pow2 ? (off >> shift) : off / (uint64_t)d.bytes);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t i = t + (uint32_t)k * 1024u;
            if (i < n) keys[i] = kk[k];
        }
    }
    __syncthreads();
    iov_lds_mark(keys, tab, rep, n);
    uint32_t *conf = tab;                                   // the table is done with
    // pairs alone on their destination: every vector of them at once, U per lane in flight
    // (source addresses first -- a listed source is one more round trip -- then the data)
    constexpr int U = W == 16 ? 8 : 16;
    for (uint32_t base = 0; base < d.items; base += 1024u * U) {
        typename Vec<W>::T a[U], b[U];
        const char *sps[U];
        char *dps[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const uint32_t g = base + (uint32_t)k * 1024u + t;
            dps[k] = nullptr;
            if (g >= d.items) continue;
            const uint32_t i = d.nvec_div.div(g), v = g - i * d.nvec;
            if ((rep[i >> 5] >> (i & 31u)) & 1u) {
                if (v == 0) conf[atomicAdd(&nconf, 1u)] = i;
                continue;
            }
            sps[k] = iov_lds_src(d, i) + (size_t)v * W;
            dps[k] = (char *)(dlo + (uint64_t)keys[i] * (uint64_t)d.bytes) + (size_t)v * W;
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (!dps[k]) continue;
            a[k] = src_load<W, SYS>(sps[k]);
            if constexpr (OP::kReadsDst) b[k] = vload<W, false>(dps[k]);
        }
#pragma unroll
        for (int k = 0; k < U; ++k)
            if (dps[k]) vstore<W, false>(dps[k], op.template apply<W>(b[k], a[k]));
    }
    __syncthreads();
    iov_lds_runs<OP, W, SYS>(d, op, dlo, keys, conf, nconf);
}

// ---------------------------------------------------------------------------
// Partitioned io-vector path (round 6) for kIovLdsRoute .. kIovPartMax pairs whose
// destinations may repeat.  Repeats can only meet on one key, so the keys are split by a
// hash into G partitions of about kIovPartMean pairs, and each workgroup orders and
// applies ONE partition on its own: no table, no cross-workgroup hand-off, and the
// random destinations spread over G CUs.
//   k_iov_keyof : key = (dst_list[i] - dlo) / bytes, the list read once (chip-wide; it
//                 may sit across PCIe in the mapped pinned staging); keys[i] = key, and
//                 (key, i) appended to its partition's bucket (an atomic on its counter:
//                 an array per calling thread and device, zero at rest -- k_iov_part
//                 zeroes its own after use, so no clearing launch)
//   k_iov_part  : workgroup w reads its bucket into LDS and applies it (iov_part_apply:
//                 keys alone in the bucket at once, repeated keys sorted by (key, index)
//                 and applied in index order, the reference's, comex.c:7342-7351).  A
//                 bucket that overflowed (a skewed scatter: thousands of pairs on a few
//                 destinations) is done in windows of the input instead -- the window's
//                 pairs of the partition gathered and applied, window after window, so
//                 input order per key is kept -- or, above kIovPartWindowMax pairs, left
//                 to the caller's radix fallback (IovPartState).
// A first version without buckets (each workgroup scanned every key for its own) grew
// with n x G: 53 us at 64 Ki random pairs against 26 for the hashed path; one with a
// memset clearing the counters before each call: 25 us at 4 Ki pairs, 39 at 64 Ki.
constexpr uint32_t kIovPartMean = 128;      // pairs per partition on average
constexpr uint32_t kIovPartCap = 1024;      // bucket entries (LDS: the entries and the repeated ones, 16 KiB)
constexpr uint32_t kIovPartBS = 128;        // k_iov_part threads
constexpr uint32_t kIovPartGMax = 8192;     // partitions at most (kIovPartMax / kIovPartMean)

// The counters: zero at rest, so one array serves one caller at a time -- each calling
// thread gets its own per device (the local io-vector path under launch_mu and the
// progress thread's owner-side applies may run together), taken from a pool and returned
// to it, still zero, when the thread ends (no device free at thread exit).  A caller
// orders its own calls: the local path synchronises the streams first, the progress
// thread waits for its previous apply (prog_work_ev).
struct IovPartCounts {
    uint32_t *dev[64] = {};
    ~IovPartCounts();
};
static std::mutex g_part_mu;
static std::vector<uint32_t *> g_part_pool[64];
IovPartCounts::~IovPartCounts() {
    std::lock_guard<std::mutex> g(g_part_mu);
    for (int i = 0; i < 64; ++i)
        if (dev[i]) g_part_pool[i].push_back(dev[i]);
}
static thread_local IovPartCounts t_part_counts;
static uint32_t *iov_part_counts() {
    IovPartCounts &mine = t_part_counts;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    if (mine.dev[dev]) return mine.dev[dev];
    std::lock_guard<std::mutex> g(g_part_mu);
    if (!g_part_pool[dev].empty()) {
        mine.dev[dev] = g_part_pool[dev].back();
        g_part_pool[dev].pop_back();
        return mine.dev[dev];
    }
    uint32_t *p = nullptr;
    if (hipMalloc((void **)&p, kIovPartGMax * 4) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, kIovPartGMax * 4) != hipSuccess) return nullptr;
    mine.dev[dev] = p;
    return p;
}

// comex_finalize (streams idle): the pool's arrays and the calling thread's are freed;
// arrays of other threads still running go back to the pool when those end
void iov_part_release() {
    std::lock_guard<std::mutex> g(g_part_mu);
    for (int i = 0; i < 64; ++i) {
        for (uint32_t *p : g_part_pool[i]) (void)hipFree(p);
        g_part_pool[i].clear();
        if (t_part_counts.dev[i]) (void)hipFree(t_part_counts.dev[i]);
        t_part_counts.dev[i] = nullptr;
    }
}

// log2 of the partitions for n pairs: about kIovPartMean pairs each, at most kIovPartGMax
// partitions (above 1 Mi pairs the partitions grow instead: 512 pairs each at 4 Mi)
static uint32_t iov_part_lg(uint32_t n) {
    uint32_t lg = 0;
    while ((n >> lg) > kIovPartMean && (1u << lg) < kIovPartGMax) ++lg;
    return lg;
}

__device__ __forceinline__ uint32_t iov_part_of(uint32_t key, uint32_t lg) {
    return lg ? (key * 0x9E3779B1u) >> (32 - lg) : 0u;
}

// 1024 threads x kKeyofPer pairs a workgroup: the ranks within a partition from an LDS
// histogram, then ONE device atomic per (workgroup, partition) reserves the bucket
// range (one returning atomic per pair instead -- 128 on each counter -- took ~10 us at
// 4 Ki pairs, this 5)
constexpr uint32_t kKeyofPer = 4;
__global__ __launch_bounds__(1024) void k_iov_keyof(const uint64_t *dst_list, uint64_t dlo, uint32_t shift, bool pow2,
                                                    uint32_t bytes, uint32_t n, uint32_t lg, uint32_t *counts,
                                                    uint32_t *keys, uint64_t *bucket, uint32_t *overflow) {
    __shared__ uint32_t hist[kIovPartGMax];
    const uint32_t t = threadIdx.x, G = 1u << lg;
    for (uint32_t p = t; p < G; p += 1024) hist[p] = 0;
    uint64_t a[kKeyofPer];
    const uint32_t i0 = blockIdx.x * 1024u * kKeyofPer + t;
#pragma unroll
    for (uint32_t k = 0; k < kKeyofPer; ++k) {
        const uint32_t i = i0 + k * 1024u;
        a[k] = i < n ? __builtin_nontemporal_load(dst_list + i) : 0;
    }
    __syncthreads();
    uint32_t key[kKeyofPer], part[kKeyofPer], rank[kKeyofPer];
#pragma unroll
    for (uint32_t k = 0; k < kKeyofPer; ++k) {
        const uint32_t i = i0 + k * 1024u;
        if (i >= n) continue;
        const uint64_t off = a[k] - dlo;
        key[k] = (uint32_t)(pow2 ? (off >> shift) : off / bytes);
        keys[i] = key[k];
        part[k] = iov_part_of(key[k], lg);
        rank[k] = atomicAdd(&hist[part[k]], 1u);
    }
    __syncthreads();
    for (uint32_t p = t; p < G; p += 1024)
        if (hist[p]) {
            const uint32_t h = hist[p];
            hist[p] = atomicAdd(counts + p, h);   // now the range's start
            if (overflow && hist[p] + h > kIovPartCap) *overflow = 1u;   // (mapped pinned: the host reads it)
        }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kKeyofPer; ++k) {
        const uint32_t i = i0 + k * 1024u;
        if (i >= n) continue;
        const uint32_t s = hist[part[k]] + rank[k];
        if (s < kIovPartCap) bucket[(size_t)part[k] * kIovPartCap + s] = ((uint64_t)key[k] << 32) | i;
    }
}

// ent[0..m) (key:index) of one partition: an LDS hash table (16-bit slots: entry index,
// top bit = the key has more than one entry; double hashing as iov_lds_mark) finds the
// entries whose key repeats; every other entry is its destination's only pair and is
// applied at once, the repeated ones are sorted by (key, index) in `aux`, their
// source-side products computed by all lanes, and one lane per distinct key adds them to
// its destination in index order (a run of hundreds of pairs on one destination: one
// lane's chain of source loads took ~90 us at 32 Ki pairs on 200 destinations).
// (Sorting every entry instead -- a bitonic sort of about kIovPartMean -- cost ~13 us a
// partition at 128 threads and ~21 at 64: latency of the barrier stages, where a random
// scatter has no repeats to order.)  Every thread of the workgroup calls it (barriers
// inside).
constexpr uint32_t kIovPartTabLog = 11;     // 2048 slots for at most kIovPartCap entries
template <class OP, int W, bool SYS>
__device__ __forceinline__ void iov_part_apply(const IovDesc &d, const OP &op, uint64_t dlo, const uint64_t *ent,
                                               uint32_t m, uint32_t *tab, uint64_t *aux, uint32_t *naux,
                                               typename Vec<W>::T *pv) {
    const uint32_t t = threadIdx.x;
    constexpr uint32_t mask = (1u << kIovPartTabLog) - 1u;
    for (uint32_t w = t; w < (1u << kIovPartTabLog) / 2; w += kIovPartBS) tab[w] = 0xffffffffu;
    if (t == 0) *naux = 0;
    __syncthreads();
    for (uint32_t u = t; u < m; u += kIovPartBS) {
        const uint32_t key = (uint32_t)(ent[u] >> 32);
        uint32_t h = (key * 0x85EBCA6Bu) >> (32 - kIovPartTabLog);
        const uint32_t step = ((key * 0xC2B2AE35u) >> (32 - kIovPartTabLog)) | 1u;
        for (;;) {
            uint32_t *wp = &tab[h >> 1];
            const uint32_t sh = (h & 1u) * 16u;
            const uint32_t cur = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint32_t e = (cur >> sh) & 0xffffu;
            if (e == kIovLdsEmpty) {
                if (atomicCAS(wp, cur, (cur & ~(0xffffu << sh)) | (u << sh)) == cur) break;
                continue;                                   // the word changed under us: look again
            }
            if ((uint32_t)(ent[e & 0x7fffu] >> 32) == key) {
                atomicOr(wp, 0x8000u << sh);
                break;
            }
            h = (h + step) & mask;
        }
    }
    __syncthreads();
    for (uint32_t u = t; u < m; u += kIovPartBS) {
        const uint64_t en = ent[u];
        const uint32_t key = (uint32_t)(en >> 32);
        uint32_t h = (key * 0x85EBCA6Bu) >> (32 - kIovPartTabLog), e;
        const uint32_t step = ((key * 0xC2B2AE35u) >> (32 - kIovPartTabLog)) | 1u;
        for (;; h = (h + step) & mask) {
            e = (tab[h >> 1] >> ((h & 1u) * 16u)) & 0xffffu;
            if ((uint32_t)(ent[e & 0x7fffu] >> 32) == key) break;   // the key's slot
        }
        if (e & 0x8000u) aux[atomicAdd(naux, 1u)] = en;
        else iov_lds_pair<OP, W, SYS>(d, op, (uint32_t)en, (char *)(dlo + (uint64_t)key * (uint64_t)d.bytes));
    }
    __syncthreads();
    const uint32_t mr = *naux;
    if (mr) {
        uint32_t P = 1;
        while (P < mr) P <<= 1;
        for (uint32_t u = mr + t; u < P; u += kIovPartBS) aux[u] = ~0ull;   // sorts last
        __syncthreads();
        for (uint32_t k = 2; k <= P; k <<= 1) {
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t u = t; u < P; u += kIovPartBS) {
                    const uint32_t l = u ^ j;
                    if (l <= u) continue;
                    const uint64_t x = aux[u], y = aux[l];
                    if ((x > y) == ((u & k) == 0)) {
                        aux[u] = y;
                        aux[l] = x;
                    }
                }
                __syncthreads();
            }
        }
        // vector v of every repeated pair: the source-only part of the operation (the
        // products) by all lanes into LDS, then one lane per destination adds them in index
        // order -- op.pre / op.add, the same operations as op.apply (gaamd_device.hpp)
        for (uint32_t v = 0; v < d.nvec; ++v) {
            for (uint32_t u = t; u < mr; u += kIovPartBS)
                pv[u] = op.template pre<W>(src_load<W, SYS>(iov_lds_src(d, (uint32_t)aux[u]) + (size_t)v * W));
            __syncthreads();
            for (uint32_t u = t; u < mr; u += kIovPartBS) {
                const uint32_t key = (uint32_t)(aux[u] >> 32);
                if (u > 0 && (uint32_t)(aux[u - 1] >> 32) == key) continue;
                char *dp = (char *)(dlo + (uint64_t)key * (uint64_t)d.bytes) + (size_t)v * W;
                typename Vec<W>::T y{};
                if constexpr (OP::kReadsDst) y = vload<W, false>(dp);
                uint32_t lo = u + 1, hi = mr;                 // the run's end (aux is sorted)
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if ((uint32_t)(aux[mid] >> 32) == key) lo = mid + 1;
                    else hi = mid;
                }
#pragma unroll 8
                for (uint32_t j = u; j < lo; ++j) y = op.template add<W>(y, pv[j]);
                vstore<W, false>(dp, y);
            }
            __syncthreads();
        }
    }
    __syncthreads();
}

template <class OP, int W, bool SYS>
__global__ __launch_bounds__(kIovPartBS) void k_iov_part(const IovDesc d, const OP op, uint64_t dlo, uint32_t lg,
                                                         uint32_t *counts, const uint32_t *keys,
                                                         const uint64_t *bucket, bool defer) {
    __shared__ uint64_t ent[kIovPartCap], aux[kIovPartCap];
    __shared__ uint32_t tab[(1u << kIovPartTabLog) / 2];
    __shared__ uint32_t cnt, naux;
    __shared__ typename Vec<W>::T pv[kIovPartCap];
    const uint32_t t = threadIdx.x, w = blockIdx.x;
    // the bucket's first kIovPartBS entries loaded with the count, not after it
    const uint64_t *bk = bucket + (size_t)w * kIovPartCap;
    const uint64_t e0 = bk[t];
    const uint32_t m = counts[w];
    if (m == 0) return;
    // an overflowed partition of a large call is left, count and all, to the caller's
    // radix fallback (launch_iov_runs with this call's IovPartState as the mask)
    if (defer && m > kIovPartCap) return;
    __syncthreads();
    if (t == 0) counts[w] = 0;   // zero at rest for the next call (stream-ordered after this one)
    if (m <= kIovPartCap) {
        if (t < m) ent[t] = e0;
        for (uint32_t u = t + kIovPartBS; u < m; u += kIovPartBS) ent[u] = bk[u];
        iov_part_apply<OP, W, SYS>(d, op, dlo, ent, m, tab, aux, &naux, pv);
        return;
    }
    // overflowed: windows of kIovPartCap input pairs (at most kIovPartCap of them match);
    // n / kIovPartCap windows for this one workgroup, so only for calls of up to
    // kIovPartWindowMax pairs -- larger ones defer (above)
    for (uint32_t base = 0; base < d.n; base += kIovPartCap) {
        if (t == 0) cnt = 0;
        __syncthreads();
        for (uint32_t i = base + t; i < base + kIovPartCap && i < d.n; i += kIovPartBS) {
            const uint32_t key = keys[i];
            if (iov_part_of(key, lg) == w) ent[atomicAdd(&cnt, 1u)] = ((uint64_t)key << 32) | i;
        }
        __syncthreads();
        const uint32_t mw = cnt;
        if (mw) iov_part_apply<OP, W, SYS>(d, op, dlo, ent, mw, tab, aux, &naux, pv);   // mw is uniform
    }
}

// the fallback's keys: pairs k_iovh_apply already applied (their slot not marked
// repeated) get the sentinel key, sorted last and skipped by k_iov_runs
__global__ __launch_bounds__(256) void k_iov_keys_masked(const uint64_t *dst_list, uint64_t dlo, uint32_t bytes,
                                                         uint32_t n, uint32_t epoch, const uint32_t *dup,
                                                         const uint32_t *slot, uint32_t *keys, uint32_t *vals) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const uint32_t h = slot[i];
    keys[i] = (dup[h] != epoch) ? kIovRunSkip : (uint32_t)((dst_list[i] - dlo) / bytes);
    vals[i] = i;
}

// the partition fallback's keys: pairs of partitions that did not overflow were applied
// by k_iov_part and get the sentinel key
__global__ __launch_bounds__(256) void k_iov_keys_partmask(const uint64_t *dst_list, uint64_t dlo, uint32_t bytes,
                                                           uint32_t n, const uint32_t *counts, uint32_t lg,
                                                           uint32_t *keys, uint32_t *vals) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const uint32_t key = (uint32_t)((dst_list[i] - dlo) / bytes);
    keys[i] = counts[iov_part_of(key, lg)] > kIovPartCap ? key : kIovRunSkip;
    vals[i] = i;
}

template <class OP, int W, bool SYS>
static hipError_t iov_ws(const IovDesc &d, const OP &op, bool serial, hipStream_t st, const IovHashArgs *ha) {
    if (ha && ha->part_keys) {
        // scratch: keys (4 B a pair) | buckets (G x kIovPartCap x 8 B)
        char *sc = (char *)ha->part_keys;
        const uint32_t G = 1u << ha->part_lg;
        uint32_t *counts = ha->count, *keys = (uint32_t *)sc;
        uint64_t *bucket = (uint64_t *)(sc + (((size_t)d.n * 4 + 255) & ~(size_t)255));
        hipLaunchKernelGGL(k_iov_keyof, dim3((d.n + 1024u * kKeyofPer - 1) / (1024u * kKeyofPer)), dim3(1024), 0, st,
                           d.dst_list, ha->dlo, ha->shift,
                           ha->pow2, (uint32_t)d.bytes, d.n, ha->part_lg, counts, keys, bucket, ha->overflow);
        hipLaunchKernelGGL((k_iov_part<OP, W, SYS>), dim3(G), dim3(kIovPartBS), 0, st, d, op, ha->dlo, ha->part_lg,
                           counts, keys, bucket, ha->overflow != nullptr);
    } else if (ha && ha->lds) {
        hipLaunchKernelGGL((k_iov_lds<OP, W, SYS>), dim3(1), dim3(1024), 0, st, d, op, ha->dlo, ha->shift, ha->pow2);
    } else if (ha) {
        hipLaunchKernelGGL((k_iovh_apply<OP, W, SYS>), dim3((d.n + kIovhBS - 1) / kIovhBS), dim3(kIovhBS), 0, st, d, op,
                           ha->dlo,
                           ha->shift, ha->pow2, ha->epoch, ha->dup, ha->slot, ha->conf, ha->count);
        hipLaunchKernelGGL((k_iovh_conf<OP, W, SYS>), dim3(1), dim3(1024), 0, st, d, op, ha->conf, ha->count,
                           ha->overflow);
    } else if (d.run_key) {
        hipLaunchKernelGGL((k_iov_runs<OP, W, SYS>), dim3((d.n + 255u) / 256u), dim3(256), 0, st, d, op);
    } else if (serial) {
        hipLaunchKernelGGL((k_iov_serial<OP, W, SYS>), dim3(1), dim3(64), 0, st, d, op);
    } else {
        constexpr int U = 2;
        uint64_t blocks = ((uint64_t)d.items + 256u * U - 1) / (256u * U);
        if (blocks > 65536) blocks = 65536;
        hipLaunchKernelGGL((k_iov<OP, W, U, SYS>), dim3((uint32_t)blocks), dim3(256), 0, st, d, op);
    }
    return hipGetLastError();
}

// sys: sources in a peer GPU's memory -- built for the byte copy only (getv from
// another device; every other cross-device io-vector is applied by the owner)
template <class OP, int W>
static hipError_t iov_w(const IovDesc &d, const OP &op, bool serial, bool sys, hipStream_t st,
                        const IovHashArgs *ha) {
    if constexpr (W < OP::kElem) {
        return hipErrorInvalidValue;
    } else {
        if (sys) {
            if constexpr (std::is_same<OP, CopyOp>::value) return iov_ws<OP, W, true>(d, op, serial, st, ha);
            else return hipErrorInvalidValue;
        }
        return iov_ws<OP, W, false>(d, op, serial, st, ha);
    }
}

template <class OP>
static hipError_t iov_op(int W, const IovDesc &d, const OP &op, bool serial, bool sys, hipStream_t st,
                         const IovHashArgs *ha) {
    switch (W) {
    case 16: return iov_w<OP, 16>(d, op, serial, sys, st, ha);
    case 8: return iov_w<OP, 8>(d, op, serial, sys, st, ha);
    case 4: return iov_w<OP, 4>(d, op, serial, sys, st, ha);
    case 2: return iov_w<OP, 2>(d, op, serial, sys, st, ha);
    case 1: return iov_w<OP, 1>(d, op, serial, sys, st, ha);
    }
    return hipErrorInvalidValue;
}

static int iov_dispatch(int op, const void *scale, int W, const IovDesc &d, bool serial, bool sys,
                        hipStream_t stream, const IovHashArgs *ha = nullptr);

int launch_iov(int op, const void *scale, IovDesc d, uint64_t align_or, bool serial, hipStream_t stream,
               bool src_peer) {
    const int esz = elem_size(op);
    if (!esz || d.bytes <= 0) return -4;
    if (op != kOpCopy && !scale) return -5;
    const int64_t row = (op == kOpCopy) ? d.bytes : (int64_t)(d.bytes / esz) * esz;   // acc.h:122
    if (d.n == 0 || row == 0) return 0;
    uint64_t a = align_or | (uint64_t)row | 16;
    if (!d.src_list) a |= (uint64_t)(uintptr_t)d.src_base | (uint64_t)d.bytes;
    if (!d.dst_list) a |= (uint64_t)(uintptr_t)d.dst_base | (uint64_t)d.bytes;
    int W = (int)lowbit(a);
    if (W > 16) W = 16;
    if (W < esz) {   // sub-natural element alignment: see launch_strided
        if (W < 4) return -8;
        W = esz;
    }
    if (serial) W = esz;
    d.nvec = (uint32_t)(row / W);
    d.nvec_div = make_fastdiv(d.nvec);
    if ((uint64_t)d.n * d.nvec >= (1ull << 31)) return -7;
    d.items = d.n * d.nvec;
    return iov_dispatch(op, scale, W, d, serial, src_peer, stream);
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// ---------------------------------------------------------------------------
// stable LSD radix sort of (key, value) u32 pairs for the io-vector run path,
// 8-bit digits over bits [0, end_bit).  Per pass three launches:
//   k_rs_hist    one workgroup per tile of 4096 keys: digit counts in LDS,
//                stored digit-major (counts[digit * ntiles + tile])
//   k_rs_scan    one workgroup per digit: exclusive prefix of its row of tile
//                counts, the digit's total to totals[digit]
//   k_rs_scatter one workgroup per tile: the 256 digit bases (exclusive scan of
//                the totals) + the tile's offsets; the tile's keys in 16 rounds
//                of 256 (input order), each key's rank among equal digits of
//                its round from wave ballots (8 of them: the lanes whose digit
//                matches) and per-wave counts in LDS -- equal keys keep their
//                input order, which the run kernel's order relies on.
// A hand-written sort rather than a library one: one instantiation, three
// kernels, no per-architecture dispatch code in the shipped object.
constexpr int kRsThreads = 256, kRsRounds = 16, kRsTile = kRsThreads * kRsRounds;

__global__ __launch_bounds__(256) void k_rs_hist(const uint32_t *keys, uint32_t n, uint32_t shift, uint32_t ntiles,
                                                 uint32_t *counts) {
    __shared__ uint32_t h[256];
    const uint32_t t = threadIdx.x, tile = blockIdx.x;
    h[t] = 0;
    __syncthreads();
    const uint32_t base = tile * (uint32_t)kRsTile;
#pragma unroll 4
    for (int j = 0; j < kRsRounds; ++j) {
        const uint32_t i = base + (uint32_t)j * kRsThreads + t;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    counts[(size_t)t * ntiles + tile] = h[t];
}

// exclusive scan of one digit's tile counts (in place); its total to totals[digit]
__global__ __launch_bounds__(256) void k_rs_scan(uint32_t *counts, uint32_t ntiles, uint32_t *totals) {
    __shared__ uint32_t part[256];
    const uint32_t t = threadIdx.x;
    uint32_t *row = counts + (size_t)blockIdx.x * ntiles;
    const uint32_t per = (ntiles + 255u) / 256u, lo = min(ntiles, t * per), hi = min(ntiles, lo + per);
    uint32_t sum = 0;
    for (uint32_t k = lo; k < hi; ++k) sum += row[k];
    part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 256; off <<= 1) {   // inclusive Hillis-Steele scan of the partial sums
        const uint32_t v = t >= off ? part[t - off] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = part[t] - sum;
    for (uint32_t k = lo; k < hi; ++k) {
        const uint32_t c = row[k];
        row[k] = run;
        run += c;
    }
    if (t == 255) totals[blockIdx.x] = part[255];
}

__global__ __launch_bounds__(256) void k_rs_scatter(const uint32_t *kin, const uint32_t *vin, uint32_t *kout,
                                                    uint32_t *vout, uint32_t n, uint32_t shift, uint32_t ntiles,
                                                    const uint32_t *counts, const uint32_t *totals) {
    __shared__ uint32_t base[256];
    __shared__ uint32_t wcnt[4][256];
    const uint32_t t = threadIdx.x, tile = blockIdx.x, lane = t & 63u, w = t >> 6;
    const uint32_t tot = totals[t];
    base[t] = tot;
    __syncthreads();
    for (uint32_t off = 1; off < 256; off <<= 1) {
        const uint32_t v = t >= off ? base[t - off] : 0u;
        __syncthreads();
        base[t] += v;
        __syncthreads();
    }
    const uint32_t mine = base[t] - tot + counts[(size_t)t * ntiles + tile];   // exclusive + the tile's offset
    __syncthreads();
    base[t] = mine;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int j = 0; j < kRsRounds; ++j) {
        wcnt[0][t] = wcnt[1][t] = wcnt[2][t] = wcnt[3][t] = 0;
        __syncthreads();
        const uint32_t i = tile * (uint32_t)kRsTile + (uint32_t)j * kRsThreads + t;
        const bool valid = i < n;
        const uint32_t key = valid ? kin[i] : 0u;
        const uint32_t dg = (key >> shift) & 255u;
        uint64_t m = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (dg >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            m &= bit ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(m & lt);
        if (valid && rank == 0) wcnt[w][dg] = (uint32_t)__popcll(m);
        __syncthreads();
        if (valid) {
            uint32_t pos = base[dg] + rank;
            for (uint32_t q = 0; q < w; ++q) pos += wcnt[q][dg];
            kout[pos] = key;
            vout[pos] = vin[i];
        }
        __syncthreads();
        base[t] += wcnt[0][t] + wcnt[1][t] + wcnt[2][t] + wcnt[3][t];
    }
}

static size_t iov_sort_temp_bytes(uint32_t n) {
    const size_t ntiles = ((size_t)n + kRsTile - 1) / kRsTile;
    return (256 * ntiles + 256) * 4;
}

// sorts (k[0], v[0]), (k[1], v[1]) the other half of the ping-pong; returns the index
// of the pair of buffers that holds the result
static int radix_sort_pairs(uint32_t *const k[2], uint32_t *const v[2], uint32_t n, int end_bit, void *temp,
                            hipStream_t stream) {
    const uint32_t ntiles = (n + kRsTile - 1) / kRsTile;
    uint32_t *counts = (uint32_t *)temp, *totals = counts + (size_t)256 * ntiles;
    int cur = 0;
    for (int shift = 0; shift < end_bit; shift += 8, cur ^= 1) {
        hipLaunchKernelGGL(k_rs_hist, dim3(ntiles), dim3(256), 0, stream, k[cur], n, (uint32_t)shift, ntiles, counts);
        hipLaunchKernelGGL(k_rs_scan, dim3(256), dim3(256), 0, stream, counts, ntiles, totals);
        hipLaunchKernelGGL(k_rs_scatter, dim3(ntiles), dim3(256), 0, stream, k[cur], v[cur], k[cur ^ 1], v[cur ^ 1], n,
                           (uint32_t)shift, ntiles, counts, totals);
    }
    return cur;
}

size_t iov_lds_scratch_bytes(uint32_t n) {
    const uint32_t lg = iov_part_lg(n);
    return (((size_t)n * 4 + 255) & ~(size_t)255) + ((size_t)kIovPartCap * 8 << lg);
}

size_t iov_runs_work_bytes(uint32_t n) { return 4 * align256((size_t)n * 4) + align256(iov_sort_temp_bytes(n)); }

int launch_iov_runs(int op, const void *scale, IovDesc d, uint64_t align_or, uint64_t dlo, uint64_t units,
                    void *work, size_t work_bytes, hipStream_t stream, bool src_peer, const IovHash *mask,
                    const IovPartState *pmask) {
    const int esz = elem_size(op);
    if (!esz || d.bytes <= 0 || d.bytes > kIovRunsMaxBytes || !d.dst_list) return -4;
    if (op != kOpCopy && !scale) return -5;
    if (units > (1ull << 32)) return -7;
    const int64_t row = (op == kOpCopy) ? d.bytes : (int64_t)(d.bytes / esz) * esz;   // acc.h:122
    if (d.n == 0 || row == 0) return 0;
    if (work_bytes < iov_runs_work_bytes(d.n)) return -6;
    uint64_t a = align_or | (uint64_t)row | 16;
    if (!d.src_list) a |= (uint64_t)(uintptr_t)d.src_base | (uint64_t)d.bytes;
    int W = (int)lowbit(a);
    if (W > 16) W = 16;
    if (W < esz) {
        if (W < 4) return -8;
        W = esz;
    }
    d.nvec = (uint32_t)(row / W);
    d.nvec_div = make_fastdiv(d.nvec);
    d.items = d.n * d.nvec;
    char *w = (char *)work;
    const size_t q = align256((size_t)d.n * 4);
    uint32_t *kin = (uint32_t *)w, *kout = (uint32_t *)(w + q), *vin = (uint32_t *)(w + 2 * q),
             *vout = (uint32_t *)(w + 3 * q);
    void *temp = w + 4 * q;
    int end_bit = 1;
    while (end_bit < 32 && (1ull << end_bit) < units) ++end_bit;
    if (mask) {
        // the pairs the hashed launch applied already sort last (sentinel key)
        if (mask->n != d.n || mask->dlo != dlo || units >= (uint64_t)kIovRunSkip) return -9;
        const uint64_t P = mask->P;
        const uint32_t *dup = (const uint32_t *)(mask->mem + P * 8);
        const uint32_t *slot = (const uint32_t *)(mask->mem + iovh_off_slot((uint32_t)P));
        hipLaunchKernelGGL(k_iov_keys_masked, dim3((d.n + 255u) / 256u), dim3(256), 0, stream, d.dst_list, dlo,
                           (uint32_t)d.bytes, d.n, mask->epoch, dup, slot, kin, vin);
        end_bit = 32;
    } else if (pmask) {
        // the pairs of partitions k_iov_part applied sort last (sentinel key); then the
        // deferred partitions' counters back to zero
        if (!pmask->counts || units >= (uint64_t)kIovRunSkip) return -9;
        hipLaunchKernelGGL(k_iov_keys_partmask, dim3((d.n + 255u) / 256u), dim3(256), 0, stream, d.dst_list, dlo,
                           (uint32_t)d.bytes, d.n, pmask->counts, pmask->lg, kin, vin);
        hipError_t e0 = hipGetLastError();
        if (e0 != hipSuccess) return -100 - (int)e0;
        e0 = hipMemsetAsync(pmask->counts, 0, (size_t)4 << pmask->lg, stream);
        if (e0 != hipSuccess) return -100 - (int)e0;
        end_bit = 32;
    } else {
        hipLaunchKernelGGL(k_iov_keys, dim3((d.n + 255u) / 256u), dim3(256), 0, stream, d.dst_list, dlo,
                           (uint32_t)d.bytes, d.n, kin, vin);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return -100 - (int)e;
    uint32_t *const kb[2] = {kin, kout}, *const vb[2] = {vin, vout};
    const int r = radix_sort_pairs(kb, vb, d.n, end_bit, temp, stream);
    e = hipGetLastError();
    if (e != hipSuccess) return -100 - (int)e;
    d.run_key = kb[r];
    d.run_perm = vb[r];
    return iov_dispatch(op, scale, W, d, false, src_peer, stream);
}

int launch_iov_hashed(IovHash *h, int op, const void *scale, IovDesc d, uint64_t align_or, uint64_t dlo,
                      uint64_t units, hipStream_t stream, bool src_peer, const uint64_t *dst_in,
                      const uint64_t *src_in) {
    const int esz = elem_size(op);
    if (!esz || d.bytes <= 0 || d.bytes > kIovRunsMaxBytes || !d.dst_list) return -4;
    if (op != kOpCopy && !scale) return -5;
    if (d.n > kIovhMaxPairs || units >= (uint64_t)kIovRunSkip) return 1;   // the radix path
    const int64_t row = (op == kOpCopy) ? d.bytes : (int64_t)(d.bytes / esz) * esz;   // acc.h:122
    if (d.n == 0 || row == 0) return 0;
    uint64_t a = align_or | (uint64_t)row | 16;
    if (!d.src_list) a |= (uint64_t)(uintptr_t)d.src_base | (uint64_t)d.bytes;
    int W = (int)lowbit(a);
    if (W > 16) W = 16;
    if (W < esz) {
        if (W < 4) return -8;
        W = esz;
    }
    d.nvec = (uint32_t)(row / W);
    d.nvec_div = make_fastdiv(d.nvec);
    d.items = d.n * d.nvec;
    // table of P >= 2n slots, kept across calls (epoch tags: no clearing); grown
    // (and re-initialised) when a larger n arrives -- the caller has drained every
    // earlier launch that used it
    uint32_t P = 1024;
    while (P < 2 * d.n) P <<= 1;
    auto off_conf = [&](uint32_t P_, uint32_t np) { return align256(iovh_off_slot(P_) + (size_t)np * 4); };
    if (P > h->P || d.n > h->npairs) {
        const uint32_t nP = std::max(P, h->P), np = std::max(d.n, h->npairs);
        if (h->mem) {
            hipError_t e = hipFree(h->mem);
            if (e != hipSuccess) return -100 - (int)e;
        }
        h->bytes = off_conf(nP, np) + (size_t)kIovhCap * 8 + 256;
        hipError_t e = hipMalloc((void **)&h->mem, h->bytes);
        if (e != hipSuccess) return -100 - (int)e;
        e = hipMemsetAsync(h->mem, 0, (size_t)nP * 12, stream);   // keys and dup marks: epoch 0
        if (e != hipSuccess) return -100 - (int)e;
        h->P = nP;
        h->npairs = np;
        h->epoch = 0;
    }
    if (!h->flag_host) {
        hipError_t e = hipHostMalloc((void **)&h->flag_host, 64, hipHostMallocMapped);
        if (e == hipSuccess) e = hipHostGetDevicePointer((void **)&h->flag_dev, h->flag_host, 0);
        if (e != hipSuccess) return -100 - (int)e;
    }
    if (++h->epoch == 0) {   // 2^32 calls: start the tags over
        hipError_t e = hipMemsetAsync(h->mem, 0, (size_t)h->P * 12, stream);
        if (e != hipSuccess) return -100 - (int)e;
        h->epoch = 1;
    }
    *(volatile uint32_t *)h->flag_host = 0;
    const bool pow2 = (d.bytes & (d.bytes - 1)) == 0;
    const uint32_t shift = pow2 ? (uint32_t)__builtin_ctz((unsigned)d.bytes) : 0;
    uint64_t *keys = (uint64_t *)h->mem;
    uint32_t *dup = (uint32_t *)(keys + h->P);
    uint32_t *slot = (uint32_t *)(h->mem + iovh_off_slot(h->P));
    uint64_t *conf = (uint64_t *)(h->mem + off_conf(h->P, h->npairs));
    uint32_t *count = (uint32_t *)(conf + kIovhCap);
    if (src_in && !d.src_list) return -4;
    hipLaunchKernelGGL(k_iovh_insert, dim3((d.n + kIovhBS - 1) / kIovhBS), dim3(kIovhBS), 0, stream,
                       (uint64_t *)d.dst_list, dlo,
                       (uint32_t)d.bytes, shift, pow2, d.n, keys, dup, h->P - 1, h->epoch, slot, count, dst_in, src_in,
                       (uint64_t *)d.src_list);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return -100 - (int)e;
    IovHashArgs ha{false, 0, nullptr, dlo, shift, pow2, h->epoch, dup, slot, conf, count, h->flag_dev};
    h->dlo = dlo;
    h->n = d.n;
    h->shift = shift;
    h->pow2 = pow2;
    return iov_dispatch(op, scale, W, d, false, src_peer, stream, &ha);
}

int launch_iov_lds(int op, const void *scale, IovDesc d, uint64_t align_or, uint64_t dlo, uint64_t units,
                   hipStream_t stream, bool src_peer, void *scratch, IovPartState *defer) {
    const int esz = elem_size(op);
    if (!esz || d.bytes <= 0 || d.bytes > kIovRunsMaxBytes || !d.dst_list) return -4;
    if (op != kOpCopy && !scale) return -5;
    if (units > (1ull << 32)) return 1;   // another path
    const int64_t row = (op == kOpCopy) ? d.bytes : (int64_t)(d.bytes / esz) * esz;   // acc.h:122
    if (d.n == 0 || row == 0) return 0;
    uint64_t a = align_or | (uint64_t)row | 16;
    if (!d.src_list) a |= (uint64_t)(uintptr_t)d.src_base | (uint64_t)d.bytes;
    int W = (int)lowbit(a);
    if (W > 16) W = 16;
    if (W < esz) {
        if (W < 4) return -8;
        W = esz;
    }
    d.nvec = (uint32_t)(row / W);
    d.nvec_div = make_fastdiv(d.nvec);
    d.items = d.n * d.nvec;
    const bool pow2 = (d.bytes & (d.bytes - 1)) == 0;
    const uint32_t shift = pow2 ? (uint32_t)__builtin_ctz((unsigned)d.bytes) : 0;
    // from kIovLdsRoute pairs (with scratch, iov_lds_scratch_bytes): the partitioned path,
    // about kIovPartMean pairs a partition
    uint32_t lg = 0;
    uint32_t *keys = nullptr, *counts = nullptr;
    if (scratch && d.n >= kIovLdsRoute) {
        if (d.n > kIovPartMax) return 1;
        lg = iov_part_lg(d.n);
        counts = iov_part_counts();
        if (!counts) return -7;
        keys = (uint32_t *)scratch;
        if (d.n > kIovPartWindowMax && !(defer && defer->flag_dev)) return -10;   // must defer
        if (defer) {
            defer->counts = counts;
            defer->lg = lg;
        }
    } else if (d.n > kIovLdsMax) {
        return 1;
    }
    IovHashArgs ha{true, lg, keys, dlo, shift, pow2, 0, nullptr, nullptr, nullptr, counts,
                   (keys && defer) ? defer->flag_dev : nullptr};
    return iov_dispatch(op, scale, W, d, false, src_peer, stream, &ha);
}

bool iov_hash_overflowed(const IovHash *h) { return h->flag_host && *(volatile uint32_t *)h->flag_host != 0; }

static int iov_dispatch(int op, const void *scale, int W, const IovDesc &d, bool serial, bool sys,
                        hipStream_t stream, const IovHashArgs *ha) {
    hipError_t e;
    switch (op) {
    case kOpCopy: e = iov_op(W, d, CopyOp{}, serial, sys, stream, ha); break;
    case 37: { AccInt o; int32_t s; memcpy(&s, scale, 4); o.s = (uint32_t)s; e = iov_op(W, d, o, serial, sys, stream, ha); break; }
    case 42: { AccLng o; int64_t s; memcpy(&s, scale, 8); o.s = (uint64_t)s; e = iov_op(W, d, o, serial, sys, stream, ha); break; }
    case 39: { AccFlt o; memcpy(&o.s, scale, 4); e = iov_op(W, d, o, serial, sys, stream, ha); break; }
    case 38: { AccDbl o; memcpy(&o.s, scale, 8); e = iov_op(W, d, o, serial, sys, stream, ha); break; }
    case 40: { AccCpl o; float s[2]; memcpy(s, scale, 8); o.sr = s[0]; o.si = s[1]; e = iov_op(W, d, o, serial, sys, stream, ha); break; }
    case 41: { AccDcp o; double s[2]; memcpy(s, scale, 16); o.sr = s[0]; o.si = s[1]; e = iov_op(W, d, o, serial, sys, stream, ha); break; }
    default: return -4;
    }
    return e == hipSuccess ? 0 : -100 - (int)e;
}

}  // namespace gaamd
