// gaamd_kernels.h -- internal interface between the host runtime and the
// gfx950 strided pack/unpack/accumulate kernels (gaamd_kernels.hip).
//
// One descriptor covers every operation on the hot path:
//   * fused strided accumulate   dst[row_d(r)] += scale * src[row_s(r)]
//       (comex_accs self/SMP path, comex.c:6890-6962 -> _acc acc.h:106-154)
//   * pack / unpack / put / get  strided byte copy with either side possibly
//       packed-contiguous (comex.c:1267-1384, 6342-6427, 6617-6696)
//   * unpack-accumulate          packed src -> strided dst with _acc
//       (_acc_packed_handler comex.c:4238-4268)
// A packed buffer is just a strided side whose strides are the running
// products count[0]*count[1]*...; see gaamd_packed_strides().
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace gaamd {

constexpr int kMaxLevels = 7;       // odometer arrays are int[7] in comex.c:1273
constexpr int kOpCopy = 0;          // byte copy (put/get/pack/unpack)

// q = n / d for 0 <= n < 2^31 with one mul-hi, an add and a shift
// (round-up magic number, Granlund & Montgomery).  Shared host/device.
struct FastDiv {
    uint32_t d, m, s;
    __host__ __device__ inline uint32_t div(uint32_t n) const {
#if defined(__HIP_DEVICE_COMPILE__)
        uint32_t hi = __umulhi(n, m);
#else
        uint32_t hi = (uint32_t)(((uint64_t)n * m) >> 32);
#endif
        return (uint32_t)(((uint64_t)hi + n) >> s);
    }
};
FastDiv make_fastdiv(uint32_t d);

struct alignas(16) Scale16 { uint64_t w[2]; };

struct Desc {
    const char *src;
    char *dst;
    int64_t s_str[kMaxLevels];   // byte stride of level j+1 (stride[j])
    int64_t d_str[kMaxLevels];
    FastDiv cnt[kMaxLevels];     // count[j+1]
    int32_t levels;              // stride_levels in this launch
    uint32_t rows;               // rows covered by this launch
    uint32_t row0;               // global index of the first row
    uint32_t nvec;               // W-byte vectors per row
    FastDiv nvec_div;
    uint32_t chunks;             // row chunks per row (row kernel)
    FastDiv chunk_div;
    uint64_t items;              // work items in this launch
    uint32_t align_mask;         // 2-D rows kernel: chunk alignment of dst (0 = off)
    Scale16 scale;
};

enum KernelKind { KK_AUTO = 0, KK_ROWS = 1, KK_FLAT = 2, KK_SERIAL = 3, KK_ORDERED = 4 };
constexpr int kKinds = 5;

// Run-time knobs.  Only shipped choices remain: the variants rounds 1-2 measured
// as losing (U = 2/4 vectors per thread, 256-thread row blocks, plain instead of
// non-temporal accesses, the looping kernel where the loop-free one applies, the
// 256 x 2 flat shape, 16-byte vectors at misaligned bases -- DESIGN.md §4) are
// no longer compiled; their probes live under tools/.
struct Tuning {
    int kind = KK_AUTO;     // force a kernel family
    int block = 0;          // threads per block of the rows kernels {64, 128}; 0 = auto
    int flat_max_nvec = 127;// rows with at most this many vectors use the flat kernel
    int align = 1;          // 2-D rows kernel: start chunks on chunk-aligned dst addresses (misaligned rows)
    int flat_line_min = 40; // rows off 128 B lines on both sides with at least this many vectors: rows kernel (0 = off)
    // ordered rows sharing bytes only column-wise: 2 (default) column slices, rows loaded by
    // every wave of a workgroup and applied in order from LDS (k_ordered_cols_lds); 1 one lane
    // per column slice loading its own rows (k_ordered_cols); 0 the one-workgroup kernel
    int ordered_cols = 2;
    // io-vectors of at most kIovLdsMax pairs whose destinations may repeat: 1 (default) the
    // one-workgroup LDS kernel, 0 the hashed three-launch path (kept for A/B and fallback)
    int iov_lds = 1;
};
Tuning &tuning();

struct LaunchInfo {
    int kind;      // KernelKind actually used
    int width;     // vector width in bytes
    int unroll;
    int launches;
    uint64_t blocks;
    int block;     // threads per block (rows kernels)
    int levels;    // stride levels after dropping count-1 levels and merging contiguous ones
    int aligned;   // 1: chunk grid shifted to chunk-aligned dst addresses
    int sys;       // 1: source read with system-scope loads (a peer GPU's memory)
};

// Enqueue `op` (kOpCopy or COMEX_ACC_*) over the strided patch.  src/dst
// must be device-accessible.  Returns 0 or a negative error code; never
// touches the host copy of the data.  `info` may be null.
// `src_peer`: src lies in another GPU's HBM (IPC mapping): it is read with
// system-scope loads (gaamd_kernels.hip vload_sys); a geometry whose rows'
// order matters returns kErrPeerOrdered, and the caller packs the rows into
// local memory first.
constexpr int kErrPeerOrdered = -10;
int launch_strided(int op, const void *scale, const void *src, const int *src_stride,
                   void *dst, const int *dst_stride, const int *count, int stride_levels,
                   hipStream_t stream, LaunchInfo *info,
                   uint64_t row_begin = 0, uint64_t row_end = ~0ull, bool plan_only = false,
                   bool src_peer = false);

// byte span [lo, hi) of one side relative to its base pointer
void side_span_host(const int *stride, const int *count, int stride_levels, int64_t row_bytes,
                    int64_t *lo, int64_t *hi);

int elem_size(int op);            // bytes per element for op; 1 for copy; 0 if unknown

// comex_rmw: fetch-and-add (swap == 0) or swap of one 4- or 8-byte word at
// `addr` (device-accessible); the old value lands in *out_dev (8 bytes)
int launch_rmw(int swap, void *addr, int bytes, uint64_t val, uint64_t *out_dev, hipStream_t stream);
// one lane stores v into *flag_dev (pinned host memory) after the stream's earlier work
int launch_flag(uint64_t *flag_dev, uint64_t v, hipStream_t stream);
// segment tags (segments.cpp): the tag of granule g (g * kSegGranule bytes into a
// block) for the block key `key` (granule 0's tag is the key itself)
constexpr uint64_t kSegGranule = 2ull << 20;
__host__ __device__ inline uint64_t seg_granule_tag(uint64_t key, uint32_t g) {
    return key ^ ((uint64_t)g * 0x9E3779B97F4A7C15ull);
}
// where a block's end tag lies: the last 8-byte-aligned word (an aligned 64-bit
// access even when bytes % 8 != 0, e.g. a float block of an odd count)
__host__ __device__ inline uint64_t seg_end_tag_off(uint64_t bytes) { return (bytes - 8) & ~7ull; }
// granule tags of a block of `bytes` (>= 16): every granule whose 8-byte tag ends at
// or before the end tag, so no two tags share a byte (a block of 2 MiB + 12 bytes has
// one granule tag, at 0, and its end tag at 2 MiB)
__host__ __device__ inline uint32_t seg_granule_count(uint64_t bytes) {
    return (uint32_t)((seg_end_tag_off(bytes) - 8) / kSegGranule + 1);
}
// write every granule's tag and the end tag (key_end, at seg_end_tag_off) of a block
int launch_seg_tags(void *p, uint64_t bytes, uint64_t key, uint64_t key_end, hipStream_t stream);
// check them through a mapping (system-scope loads); out_dev[2] (device memory,
// preset {0, ~0u}): mismatches, and the first bad granule (granule count = the end tag)
int launch_seg_check(const void *p, uint64_t bytes, uint64_t key, uint64_t key_end, uint32_t *out_dev,
                     hipStream_t stream);
LaunchInfo *last_launch_info();   // most recent launch_strided (any caller)
unsigned long long kernel_count(int kind);   // launch_strided launches so far, by KernelKind (< kKinds)

// I/O-vector descriptor: n pairs of `bytes`; a side is a device array of n
// addresses (list) or, when the list is null, base + i*bytes (packed)
struct IovDesc {
    const uint64_t *src_list;
    const uint64_t *dst_list;
    const char *src_base;
    char *dst_base;
    int32_t bytes;
    uint32_t n;
    uint32_t nvec, items;   // filled by launch_iov
    FastDiv nvec_div;
    const uint32_t *run_key;   // launch_iov_runs: destinations sorted ((dst - dlo) / bytes)
    const uint32_t *run_perm;  //   and the pair index of each sorted position
};
// `align_or` = OR of every listed address (the launcher cannot read device lists);
// `serial` applies the pairs one by one in order (overlapping destinations)
// `src_peer`: the sources lie in a peer GPU's memory (byte copy only: getv)
int launch_iov(int op, const void *scale, IovDesc d, uint64_t align_or, bool serial, hipStream_t stream,
               bool src_peer = false);
// Pairs whose destinations may repeat (GA scatter-accumulate with repeated
// subscripts), without a host-side overlap check: the destinations are sorted on
// the GPU (stable radix sort of (dst - dlo) / bytes, so equal destinations keep
// their input order) and one lane per distinct destination applies its pairs in
// input order -- the reference's pair order wherever it matters.  Requires a
// device dst list, every dst - dlo a multiple of d.bytes, (dhi - dlo) / bytes
// < 2^32, d.bytes <= kIovRunsMaxBytes, and no source inside a destination.
constexpr int kIovRunsMaxBytes = 256;
size_t iov_runs_work_bytes(uint32_t n);
struct IovPartState;   // the partitioned path's deferred overflow (below)
struct IovHash;   // the hashed path's table (one per calling thread; kept across calls)
// mask: the table of a hashed launch whose conflicts overflowed (iov_hash_overflowed):
// the pairs it applied already are skipped
int launch_iov_runs(int op, const void *scale, IovDesc d, uint64_t align_or, uint64_t dlo, uint64_t units,
                    void *work, size_t work_bytes, hipStream_t stream, bool src_peer = false,
                    const IovHash *mask = nullptr, const IovPartState *pmask = nullptr);
// The same contract as launch_iov_runs without the sort for up to 2^19 pairs: a
// hash table finds the destinations with more than one pair; pairs alone on
// theirs are applied at once, the rest (up to 8192) sorted by (destination,
// index) in one workgroup's LDS and applied in index order.  Returns 1 when n is
// outside its range (use launch_iov_runs).  After the stream has completed the
// launch, iov_hash_overflowed(h) true means more conflicting pairs than the LDS
// holds: none of those was applied -- run launch_iov_runs(..., mask = h) next.
// The caller serialises its launches on one IovHash (the table is reused).
// dst_in / src_in (optional, device-mapped pinned memory): the lists not yet in HBM --
// the first kernel copies them to d.dst_list / d.src_list on its way (no upload launch);
// when this returns 1 nothing was launched and the caller uploads them itself.
IovHash *iov_hash_create();
int launch_iov_hashed(IovHash *h, int op, const void *scale, IovDesc d, uint64_t align_or, uint64_t dlo,
                      uint64_t units, hipStream_t stream, bool src_peer = false, const uint64_t *dst_in = nullptr,
                      const uint64_t *src_in = nullptr);
bool iov_hash_overflowed(const IovHash *h);
// The same contract with the ordering held in LDS; d.dst_list / d.src_list may point
// into mapped pinned memory (read once).  Below kIovLdsRoute pairs, or without scratch,
// ONE launch of one workgroup (k_iov_lds, up to kIovLdsMax pairs); from kIovLdsRoute
// to kIovPartMax pairs with `scratch` (HBM, iov_lds_scratch_bytes(n)), two launches:
// the keys into hash-partition buckets (k_iov_keyof), then one workgroup per partition
// orders and applies its pairs (k_iov_part).  Returns 1 when n is outside its range.
// Calls from one thread must be ordered (each completes before the next starts): the
// partition counters are per thread and zero between calls.
// A partition of more than its bucket's pairs (heavy repeats) is done in windows of the
// input by its workgroup: n / 1024 windows, so only up to kIovPartWindowMax pairs.  Larger
// calls pass `defer` with a mapped pinned flag: such partitions are then left untouched
// (counters kept), the flag raised, and after the stream completed the caller applies
// them with launch_iov_runs(..., pmask = defer) (which zeroes the counters again).
struct IovPartState {
    uint32_t *flag_dev = nullptr;   // in: device view of a zeroed mapped pinned word
    uint32_t *counts = nullptr;     // out: the call's partition counters
    uint32_t lg = 0;                // out: log2 of its partitions
};
constexpr uint32_t kIovPartWindowMax = 1u << 16;
void iov_part_release();   // comex_finalize: the partition counters (streams idle)
constexpr uint32_t kIovLdsMax = 16384;
constexpr uint32_t kIovLdsRoute = 1024;
constexpr uint32_t kIovPartMax = 1u << 22;
size_t iov_lds_scratch_bytes(uint32_t n);   // keys and partition buckets (~68 B a pair)
int launch_iov_lds(int op, const void *scale, IovDesc d, uint64_t align_or, uint64_t dlo, uint64_t units,
                   hipStream_t stream, bool src_peer = false, void *scratch = nullptr,
                   IovPartState *defer = nullptr);

}  // namespace gaamd
