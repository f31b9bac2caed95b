// gaamd_kernels.hip -- gfx950 kernels for GA/ComEx strided pack/unpack and
// typed accumulate (dst += alpha*src), plus their host-side launcher.
//
// Reference semantics (paths relative to the GA tree):
//   _acc            comex/src-common/acc.h:106-154   (HAVE_BLAS=0 loops 137-143)
//   odometer        comex/src-mpi-pr/comex.c:1293-1327 (pack), 1354-1383
//                   (unpack), 4222-4266 (server unpack-acc), 6924-6961 (nb_accs)
//
// Design (CDNA4, bandwidth-bound, no MFMA):
//   * Row r of the patch sits at sum_j digit_j(r)*stride[j] with digit_j the
//     mixed-radix digits of r over count[1..L], count[1] fastest -- exactly the
//     rows the reference odometer visits, in the same order.  Digits come from
//     FastDiv (one mul-hi per level) instead of the reference's per-row `%`.
//   * ROWS kernel (long rows): one work item = one chunk of BS*U vectors of one
//     row; the row decode is wave-uniform (SGPRs), each lane streams U
//     independent W-byte vectors (W = 16 where alignment allows:
//     global_load_dwordx4), all loads issued before the first FP op.
//   * FLAT kernel (short rows, < 128 vectors): vectors of all rows are flattened
//     so every lane of a wave has work; each lane decodes its own row.
//   * ORDERED kernel: where rows truly share bytes (dst rows with each other,
//     or a src row with a dst row: found exactly by classify_rows), one
//     16-wave workgroup applies the rows in the reference's order, each row
//     wave-parallel.
//   * SERIAL kernel: one lane walks rows and elements in reference order; only
//     for a src run that starts inside its own dst run below it (a recurrence
//     inside one _acc loop).
//   * Alpha travels in the kernel argument block (SGPRs), not LDS.
//   * FP contraction is OFF (pragma below + -ffp-contract=off): the reference
//     computes round(round(a*b)+c) with no FMA, so must we, bit for bit.
//     Integer types accumulate in unsigned arithmetic (wraparound, like the
//     reference's -fwrapv behaviour).
#pragma clang fp contract(off)

#include "gaamd_kernels.h"
#include "gaamd_device.hpp"
#include <string.h>
#include <algorithm>
#include <type_traits>
#include <atomic>
#include <vector>
#include <utility>
#include <mutex>
#include <cmath>

namespace gaamd {

// ---------------------------------------------------------------------------
// host helpers
FastDiv make_fastdiv(uint32_t d) {
    FastDiv f;
    f.d = d ? d : 1;
    uint32_t l = 0;
    while ((1ull << l) < f.d) ++l;
    f.s = l;
    f.m = (uint32_t)((((1ull << 32) * ((1ull << l) - f.d)) / f.d) + 1);
    return f;
}

static Tuning g_tuning;
Tuning &tuning() { return g_tuning; }
static std::atomic<unsigned long long> g_kind_count[kKinds];
unsigned long long kernel_count(int kind) { return (kind >= 0 && kind < kKinds) ? g_kind_count[kind].load() : 0; }

int elem_size(int op) {
    switch (op) {
    case kOpCopy: return 1;
    case 37: return 4;   // COMEX_ACC_INT
    case 38: return 8;   // COMEX_ACC_DBL
    case 39: return 4;   // COMEX_ACC_FLT
    case 40: return 8;   // COMEX_ACC_CPL
    case 41: return 16;  // COMEX_ACC_DCP
    case 42: return 8;   // COMEX_ACC_LNG
    default: return 0;
    }
}


// ---------------------------------------------------------------------------
// row decode: byte offsets of row r on both sides (mixed radix over count[1..L]).
// LV > 0: exactly LV levels known at compile time (only those fields are read,
// which keeps the kernel's SGPR footprint small); LV == 0: runtime d.levels.
template <int LV>
__device__ __forceinline__ void row_offsets(const Desc &d, uint32_t r, int64_t &so, int64_t &dof) {
    so = 0;
    dof = 0;
    constexpr int N = LV > 0 ? LV : kMaxLevels;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        if (LV == 0 && j >= d.levels) continue;   // (not `break`: keeps the loop unrollable)
        const uint32_t q = d.cnt[j].div(r);
        const uint32_t dig = r - q * d.cnt[j].d;
        so += (int64_t)dig * d.s_str[j];
        dof += (int64_t)dig * d.d_str[j];
        r = q;
    }
}

// Stores of the streaming kernels are non-temporal, like their loads.  Round 6 tried
// default-policy stores: a stand-alone probe (tools/short_rows_probe.hip, constant
// data, profiles/r06/short_rows/) read them faster on every row length, but the
// library built with them lost on every row length but the shortest, on one stream and
// on two alike (64-byte rows 0.36-0.39 against 0.41-0.43, 16 KiB rows 0.72-0.76 against
// 0.79-0.81, interleaved in one call, profiles/r06/store_policy_ab/; the headline 0.75
// against 0.80 over 300 steps, profiles/r06/plain_stores/).  Rows of at most 32 bytes
// take the flat kernel's SHORT form instead: plain loads and non-temporal stores, 0.337
// against 0.283.
constexpr bool kNtStore = true;

// the U vectors of one thread: all loads first, then the ops and the stores.
// `full` (wave-uniform) says the whole chunk lies inside the row, so the
// vectors need no predicate and their addresses fold into immediate offsets.
// SYS: the source lies in a peer GPU's memory -> system-scope source loads
template <class OP, int W, int U, int BS, bool SYS = false>
__device__ __forceinline__ void chunk_op(const char *sp, char *dp, int64_t v0, uint32_t nvec, bool full,
                                         const OP &op) {
    typedef typename Vec<W>::T V;
    V a[U], b[U];
    const char *s0 = sp + v0 * W;
    char *d0 = dp + v0 * W;
    if (full) {
        if constexpr (SYS) {
            // the local dst loads first: each system-scope (volatile) source load is
            // followed by a wait for every load in flight (vload_sys)
            if constexpr (OP::kReadsDst) {
#pragma unroll
                for (int k = 0; k < U; ++k) b[k] = vload<W, true>(d0 + k * BS * W);
            }
#pragma unroll
            for (int k = 0; k < U; ++k) a[k] = vload_sys<W>(s0 + k * BS * W);
        } else {
#pragma unroll
            for (int k = 0; k < U; ++k) {
                a[k] = vload<W, true>(s0 + k * BS * W);
                if constexpr (OP::kReadsDst) b[k] = vload<W, true>(d0 + k * BS * W);
            }
        }
#pragma unroll
        for (int k = 0; k < U; ++k) vstore<W, kNtStore>(d0 + k * BS * W, op.template apply<W>(b[k], a[k]));
        return;
    }
    // row head/tail: one vector at a time (keeps the register budget of the full path)
    for (int k = 0; k < U; ++k) {
        if ((uint64_t)(v0 + k * BS) >= (uint64_t)nvec) continue;   // negative or past the row
        V x, y;
        if constexpr (OP::kReadsDst) y = vload<W, true>(d0 + k * BS * W);
        if constexpr (SYS) x = vload_sys<W>(s0 + k * BS * W);
        else x = vload<W, true>(s0 + k * BS * W);
        if constexpr (!OP::kReadsDst) y = x;
        vstore<W, kNtStore>(d0 + k * BS * W, op.template apply<W>(y, x));
    }
}

// ---------------------------------------------------------------------------
// ROWS kernel (N-D): work item w = (row, chunk); chunk = BS*U vectors of a row.
template <class OP, int W, int U, int BS, int LV, bool SYS = false>
__global__ __launch_bounds__(BS) void k_rows(const Desc d, const OP op) {
    for (uint32_t w = blockIdx.x; w < (uint32_t)d.items; w += gridDim.x) {
        const uint32_t rl = d.chunk_div.div(w);
        const uint32_t chunk = w - rl * d.chunks;
        int64_t so, dof;
        row_offsets<LV>(d, d.row0 + rl, so, dof);
        const uint32_t c0 = chunk * (uint32_t)(BS * U);
        chunk_op<OP, W, U, BS, SYS>(d.src + so, d.dst + dof, (int64_t)c0 + threadIdx.x, d.nvec,
                                    c0 + BS * U <= d.nvec, op);
    }
}

// ROWS2 kernel: the common <= 1 stride-level case (2-D patches, contiguous
// runs).  Row r sits at r*stride on each side -- no digit division -- and the
// small argument block keeps the kernel at ~32 SGPRs (full occupancy).
struct Desc2 {
    const char *src;
    char *dst;
    int64_t s_str, d_str;
    uint32_t row0, nvec, chunks, items;
    FastDiv chunk_div;
    uint32_t align_mask;   // != 0: chunk boundaries at dst addresses = 0 mod (mask+1)
};

template <class OP, int W, int U, int BS, bool SYS = false>
__global__ __launch_bounds__(BS) void k_rows2(const Desc2 d, const OP op) {
    for (uint32_t w = blockIdx.x; w < d.items; w += gridDim.x) {
        const uint32_t rl = d.chunk_div.div(w);
        const uint32_t chunk = w - rl * d.chunks;
        const int64_t r = (int64_t)(d.row0 + rl);
        const char *sp = d.src + r * d.s_str;
        char *dp = d.dst + r * d.d_str;
        // shift the chunk grid so that chunks start on aligned dst addresses
        const int64_t shift = (int64_t)(((uintptr_t)dp & d.align_mask) / W);
        const int64_t c0 = (int64_t)chunk * (BS * U) - shift;
        const bool full = c0 >= 0 && c0 + BS * U <= (int64_t)d.nvec;
        chunk_op<OP, W, U, BS, SYS>(sp, dp, c0 + threadIdx.x, d.nvec, full, op);
    }
}

// DIRECT 2-D kernel: the common case of ROWS2 where every row is a whole number
// of chunks and the grid has one block per chunk -- no loop, no bounds test, and
// one kernel-argument fetch (s_load_dwordx8 + x4 issued together before the
// first wait).  ROWS2 fetches its loop bound first and the rest after a wait:
// one more scalar-cache round trip at the head of each of the 64 Ki waves of a
// headline launch, which measured 2-3 % of the launch (tools/hbm_ceiling.hip
// vs k_rows2).
struct Desc2D {
    const char *src;
    char *dst;
    int64_t s_str, d_str;
    FastDiv chunk_div;   // chunks per row
    uint32_t row0;
};

// SYS: the source lies in a peer GPU's memory (the owner's direct-source route):
// one system-scope load per lane, issued after the local dst load (vload_sys)
template <class OP, int W, int BS, bool SYS = false>
__global__ __launch_bounds__(BS) void k_rows2d(const Desc2D d, const OP op) {
    const uint32_t w = blockIdx.x;
    const uint32_t rl = d.chunk_div.div(w);
    const uint32_t chunk = w - rl * d.chunk_div.d;
    const int64_t r = (int64_t)(d.row0 + rl);
    const int64_t v = (int64_t)chunk * BS + threadIdx.x;
    const char *sp = d.src + r * d.s_str + v * W;
    char *dp = d.dst + r * d.d_str + v * W;
    typename Vec<W>::T a, b;
    if constexpr (SYS) {
        if constexpr (OP::kReadsDst) b = vload<W, true>(dp);
        a = vload_sys<W>(sp);
        if constexpr (!OP::kReadsDst) b = a;
    } else {
        a = vload<W, true>(sp);
        b = a;
        if constexpr (OP::kReadsDst) b = vload<W, true>(dp);
    }
    vstore<W, kNtStore>(dp, op.template apply<W>(b, a));
}

// DIRECT N-D kernel (2 or 3 stride levels, every row whole chunks): as
// k_rows2d, with the row decoded by LV compile-time FastDiv digits from a
// compact argument block (C4: 3-D double complex, 4 KiB rows).
template <int LV>
struct DescND {
    const char *src;
    char *dst;
    int64_t s_str[LV], d_str[LV];
    FastDiv cnt[LV];
    FastDiv chunk_div;
    uint32_t row0;
};

template <class OP, int W, int BS, int LV>
__global__ __launch_bounds__(BS) void k_rowsnd(const DescND<LV> d, const OP op) {
    const uint32_t w = blockIdx.x;
    const uint32_t rl = d.chunk_div.div(w);
    const uint32_t chunk = w - rl * d.chunk_div.d;
    uint32_t r = d.row0 + rl;
    int64_t so = 0, dof = 0;
#pragma unroll
    for (int j = 0; j < LV; ++j) {
        const uint32_t q = d.cnt[j].div(r);
        const uint32_t dig = r - q * d.cnt[j].d;
        so += (int64_t)dig * d.s_str[j];
        dof += (int64_t)dig * d.d_str[j];
        r = q;
    }
    const int64_t v = (int64_t)chunk * BS + threadIdx.x;
    const char *sp = d.src + so + v * W;
    char *dp = d.dst + dof + v * W;
    typename Vec<W>::T a = vload<W, true>(sp), b = a;
    if constexpr (OP::kReadsDst) b = vload<W, true>(dp);
    vstore<W, kNtStore>(dp, op.template apply<W>(b, a));
}

// FLAT kernel: vectors of all rows flattened, each lane decodes its own row;
// non-temporal loads (+12-24 % on 64 B-1 KiB rows, profiles/r01/flat_nt_ab.jsonl), stores
// as kNtStore -- or, SHORT (rows of at most 32 bytes), plain loads and non-temporal stores.
template <class OP, int W, int U, int BS, int LV, bool SHORT = false>
__global__ __launch_bounds__(BS) void k_flat(const Desc d, const OP op) {
    constexpr bool NT = !SHORT, NTS = SHORT ? true : kNtStore;
    typedef typename Vec<W>::T V;
    const uint32_t span = (uint32_t)BS * U;
    for (uint32_t base = blockIdx.x * span; base < (uint32_t)d.items; base += gridDim.x * span) {
        V a[U], b[U];
        char *dps[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const uint32_t g = base + threadIdx.x + (uint32_t)(k * BS);
            dps[k] = nullptr;
            if (g < (uint32_t)d.items) {
                const uint32_t rl = d.nvec_div.div(g);
                const uint32_t v = g - rl * d.nvec;
                int64_t so, dof;
                row_offsets<LV>(d, d.row0 + rl, so, dof);
                dps[k] = d.dst + dof + (size_t)v * W;
                a[k] = vload<W, NT>(d.src + so + (size_t)v * W);
                if constexpr (OP::kReadsDst) b[k] = vload<W, NT>(dps[k]);
            }
        }
#pragma unroll
        for (int k = 0; k < U; ++k)
            if (dps[k]) vstore<W, NTS>(dps[k], op.template apply<W>(b[k], a[k]));
    }
}

// SERIAL kernel: the reference's own order (row by row, element by element).
// Only for a source run that reads bytes its own row wrote earlier in the same
// _acc loop (src starting inside the row's dst, below it): a recurrence.
template <class OP, int W>
__global__ __launch_bounds__(64) void k_serial(const Desc d, const OP op) {
    if (threadIdx.x != 0) return;
    for (uint32_t r = 0; r < d.rows; ++r) {
        int64_t so, dof;
        row_offsets<0>(d, d.row0 + r, so, dof);
        const uint64_t n = (uint64_t)d.nvec * W / OP::kElem;
        for (uint64_t m = 0; m < n; ++m)
            op.serial_elem(d.dst + dof + m * OP::kElem, d.src + so + m * OP::kElem);
    }
}

// ORDERED kernel: rows whose bytes truly overlap at DIFFERENT offsets (dst rows
// sharing bytes with each other, or a src row sharing bytes with a dst row) in
// the reference's row order (comex.c:6936-6961), each row wave-parallel.  One
// workgroup of 16 waves: a chunk of OB*U vectors is loaded completely (every
// load of the chunk before any of its stores: a src run starting above its own
// dst run reads the old bytes, as the reference's ascending _acc loop does),
// then stored; the stores are drained (vmcnt(0)) and the workgroup synchronised
// before the next chunk or row loads.  Visibility rule: __syncthreads() is a
// workgroup-scope release + barrier + acquire, which LLVM's AMDGPU memory model
// lowers on gfx942/gfx950 (no threadgroup split, the HIP default) to
// `s_waitcnt vmcnt(0)` + `s_barrier`: all waves of a workgroup share one CU's
// write-through L1, so a store completed before the barrier is seen by every
// load of the workgroup after it.
constexpr int kOrderedBS = 1024;
template <class OP, int W, int U>
__global__ __launch_bounds__(kOrderedBS) void k_ordered(const Desc d, const OP op) {
    typedef typename Vec<W>::T V;
    for (uint32_t r = 0; r < d.rows; ++r) {
        int64_t so, dof;
        row_offsets<0>(d, d.row0 + r, so, dof);
        const char *sp = d.src + so;
        char *dp = d.dst + dof;
        for (uint32_t c0 = 0; c0 < d.nvec; c0 += (uint32_t)(kOrderedBS * U)) {
            V a[U], b[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const uint32_t v = c0 + (uint32_t)(k * kOrderedBS) + threadIdx.x;
                if (v < d.nvec) {
                    a[k] = vload<W, true>(sp + (size_t)v * W);
                    b[k] = a[k];
                    if constexpr (OP::kReadsDst) b[k] = vload<W, true>(dp + (size_t)v * W);
                }
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const uint32_t v = c0 + (uint32_t)(k * kOrderedBS) + threadIdx.x;
                if (v < d.nvec) vstore<W, false>(dp + (size_t)v * W, op.template apply<W>(b[k], a[k]));
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
    }
}

// COLUMN-ORDERED kernel: rows that share bytes only at the SAME offset -- every
// pair of overlapping rows (dst/dst, src/dst) starts at the same address, e.g.
// many rows into one destination run (a zero dst stride: a column reduction),
// or a src row that IS an earlier dst row.  Then element x of a row depends only
// on element x of earlier rows, so the reference's order (rows in odometer
// order, comex.c:6936-6961) holds per column: one lane owns one W-byte column
// slice of the run for the whole call and walks every row in order; lanes and
// workgroups are independent (one wave per workgroup, nvec/64 workgroups).
//   PIPE (no src row meets any dst row): the src loads of P rows are issued
//   together, and the dst vector stays in a register while consecutive rows
//   hit the same dst run (stored when the run changes, and at the end) -- the
//   same operations in the same order as the reference, held in a register.
//   !PIPE (a src row is a dst row): load, apply, store per row; a lane's load
//   after its own store to the same address returns that store (single-thread
//   program order, which the memory model guarantees without fences).
template <class OP, int W, bool PIPE, int LV = 0>
__global__ __launch_bounds__(64) void k_ordered_cols(const Desc d, const OP op) {
    typedef typename Vec<W>::T V;
    // src loads in flight per lane (PIPE): 256 B, 64 VGPRs -- a column reduction has
    // only row-width / W lanes (one wave per SIMD at most), so each lane keeps many
    // independent loads in flight (P = 16 at W = 8 read 0.66 TB/s algorithmic on a
    // 64 KiB x 2048 reduction: latency-bound)
    constexpr int P = (LV == 1 && W == 8) ? 64 : (W >= 16 ? 16 : 32);
    const uint32_t v = blockIdx.x * 64u + threadIdx.x;
    if (v >= d.nvec) return;
    const int64_t xo = (int64_t)v * W;
    if constexpr (!PIPE) {
        for (uint32_t r = 0; r < d.rows; ++r) {
            int64_t so, dof;
            row_offsets<0>(d, d.row0 + r, so, dof);
            const V x = vload<W, false>(d.src + so + xo);
            V y = x;
            if constexpr (OP::kReadsDst) y = vload<W, false>(d.dst + dof + xo);
            vstore<W, false>(d.dst + dof + xo, op.template apply<W>(y, x));
        }
    } else {
        V acc = {};
        int64_t cur = 0;    // dst offset whose value `acc` holds, if `held`
        bool held = false;
        for (uint32_t r0 = 0; r0 < d.rows; r0 += P) {
            V s[P];
            int64_t dofs[P];
#pragma unroll
            for (int k = 0; k < P; ++k) {
                if (r0 + k < d.rows) {
                    int64_t so;
                    row_offsets<LV>(d, d.row0 + r0 + k, so, dofs[k]);
                    s[k] = vload<W, true>(d.src + so + xo);
                }
            }
#pragma unroll
            for (int k = 0; k < P; ++k) {
                if (r0 + k >= d.rows) continue;
                if (!held || dofs[k] != cur) {
                    if (held) vstore<W, false>(d.dst + cur + xo, acc);
                    cur = dofs[k];
                    held = true;
                    acc = s[k];
                    if constexpr (OP::kReadsDst) acc = vload<W, false>(d.dst + cur + xo);
                }
                acc = op.template apply<W>(acc, s[k]);
            }
        }
        if (held) vstore<W, false>(d.dst + cur + xo, acc);
    }
}

// COLUMN-ORDERED, LDS-staged (the PIPE geometries).  The
// one-lane-per-column kernel above is latency-bound: a column reduction has only
// row-width / W lanes (8192 at 64 KiB rows: one wave per two CUs), each with at
// most 63 loads in flight (vmcnt) -- 0.62-0.65 TB/s of real HBM traffic.  Here a
// workgroup owns CW column slices (CW*W contiguous bytes of every row) and splits
// the work by role:
//   * waves 1..KC_NW-1 LOAD: each issues KC_P 16-byte loads per lane per tile (a
//     load instruction covers RPI rows of the workgroup's piece), unconditionally
//     (rows past the last load the last one again: straight-line code, so the loads
//     issue back to back), computes the source-only part of the operation (op.pre:
//     the products a*src, the (re, im) of a complex product) and writes it into
//     one of two LDS tiles;
//   * wave 0 APPLIES: its first CW lanes walk the other tile's rows IN ORDER,
//     adding each row's pre-computed increment to the column value held in a
//     register (stored when the dst run changes and at the end) -- the reference's
//     operations, in its order per column (comex.c:6936-6961, acc.h:137-143); pre
//     then add is the same two roundings as apply.
// The applier is one wave and walks every row, so its instructions per row set the
// kernel's time (a 2048-row f64 column reduction at ~100 cycles per row: 90 us).
// Hence the split of the products onto the loaders, and a fast path for the common
// geometry -- every row into ONE dst run (all dst strides zero): no per-row offset
// or run test, one LDS read + one add per row, 16 rows per batch.
// One barrier per tile: the loaders fill tile i+1 while wave 0 applies tile i.
// Measured read rate of this access pattern (tools/piece_probe.hip, 256 workgroups
// each reading 256-byte pieces of 2048 rows with 64 KiB in flight): 5.4 TB/s.
constexpr int KC_NW = 8;                 // waves per workgroup: 1 applier + 7 loaders
constexpr int KC_P = 8;                  // 16-byte loads per loader lane per tile (56 KiB tiles)
template <class OP, int W, int LV, int CW>
__global__ __launch_bounds__(KC_NW * 64) void k_ordered_cols_lds(const Desc d, const OP op) {
    typedef typename Vec<W>::T V;
    typedef typename Vec<16>::T V16;
    constexpr int SPL = 16 / W;                      // column slices per 16-byte load
    constexpr int LPR = CW / SPL;                    // loader lanes per row piece
    constexpr int RPI = 64 / LPR;                    // rows per load instruction
    constexpr int T = (KC_NW - 1) * KC_P * RPI;      // rows per tile
    static_assert(CW % SPL == 0 && 64 % LPR == 0, "column group of whole 16-byte loads");
    __shared__ __attribute__((aligned(16))) V tile[2][T * CW];   // [buffer][row][column]
    // the wave index through readfirstlane: the compiler then knows the role branch
    // (and every value inside the applier's) is wave-uniform -- scalar branches
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t c = lane % CW;                    // the applier lane's column slice
    const uint32_t col0 = blockIdx.x * (uint32_t)CW, col = col0 + c;
    // every lane works on a valid address (clamped column; its values are never stored)
    const int64_t xl = (int64_t)min(col, d.nvec - 1u) * W;
    const uint32_t ntiles = (d.rows + (uint32_t)T - 1) / (uint32_t)T;
    const bool full = col0 + (uint32_t)CW <= d.nvec;   // no partial slice group (workgroup-uniform)
    auto load_store = [&](uint32_t tl, int buf) {    // loader waves: tile `tl` into tile[buf]
        const uint32_t lw = wave - 1, sub = lane / (uint32_t)LPR, s0 = (lane % (uint32_t)LPR) * SPL;
        if (full) {
            const int64_t xo = (int64_t)(col0 + s0) * W;
            V16 s[KC_P];
#pragma unroll
            for (int k = 0; k < KC_P; ++k) {
                const uint32_t r = min(tl * (uint32_t)T + (lw * KC_P + (uint32_t)k) * RPI + sub, d.rows - 1u);
                int64_t so, dof;
                row_offsets<LV>(d, d.row0 + r, so, dof);
                s[k] = vload<16, true>(d.src + so + xo);
            }
#pragma unroll
            for (int k = 0; k < KC_P; ++k)
                *reinterpret_cast<V16 *>(&tile[buf][((lw * KC_P + (uint32_t)k) * RPI + sub) * CW + s0]) =
                    op.template pre<16>(s[k]);
        } else {
            // the last workgroup of a row whose slice count is not a multiple of CW:
            // W-byte loads of clamped slices (never past the row's last byte)
#pragma unroll
            for (int k = 0; k < KC_P; ++k) {
                const uint32_t r = min(tl * (uint32_t)T + (lw * KC_P + (uint32_t)k) * RPI + sub, d.rows - 1u);
                int64_t so, dof;
                row_offsets<LV>(d, d.row0 + r, so, dof);
                V v[SPL];
#pragma unroll
                for (int j = 0; j < SPL; ++j)
                    v[j] = vload<W, true>(d.src + so + (int64_t)min(col0 + s0 + (uint32_t)j, d.nvec - 1u) * W);
#pragma unroll
                for (int j = 0; j < SPL; ++j)
                    tile[buf][((lw * KC_P + (uint32_t)k) * RPI + sub) * CW + s0 + j] = op.template pre<W>(v[j]);
            }
        }
    };
    const bool lane_ok = lane < (uint32_t)CW && col < d.nvec;
    bool one_run = true;                             // every row into one dst run
    for (int j = 0; j < d.levels; ++j) one_run = one_run && d.d_str[j] == 0;
    V acc = {};
    int64_t cur = 0;
    bool held = false;
    if (wave == 0 && one_run) {
        int64_t so;
        row_offsets<LV>(d, d.row0, so, cur);
        held = true;
        if constexpr (OP::kReadsDst) acc = vload<W, false>(d.dst + cur + xl);
    }
    auto apply_row = [&](uint32_t r, const V &x) {   // applier: row r of the patch (wave-uniform)
        int64_t so, dof;
        row_offsets<LV>(d, d.row0 + r, so, dof);
        if (!held || dof != cur) {
            if (held && lane_ok) vstore<W, false>(d.dst + cur + xl, acc);
            cur = dof;
            held = true;
            acc = x;
            if constexpr (OP::kReadsDst) acc = vload<W, false>(d.dst + cur + xl);
        }
        acc = op.template add<W>(acc, x);
    };
    if (wave != 0) load_store(0, 0);
    __syncthreads();
    for (uint32_t i = 0; i < ntiles; ++i) {
        const int buf = (int)(i & 1);
        if (wave != 0) {
            if (i + 1 < ntiles) load_store(i + 1, buf ^ 1);
        } else {
            const uint32_t r0 = i * (uint32_t)T;
            const uint32_t n = min((uint32_t)T, d.rows - r0);
            uint32_t t = 0;
            if (one_run) {
                constexpr int B = 16;
                for (; t + B <= n; t += B) {
                    V x[B];
#pragma unroll
                    for (int j = 0; j < B; ++j) x[j] = tile[buf][(t + j) * CW + c];
#pragma unroll
                    for (int j = 0; j < B; ++j) acc = op.template add<W>(acc, x[j]);
                }
                for (; t < n; ++t) acc = op.template add<W>(acc, tile[buf][t * CW + c]);
            } else {
                constexpr int B = 8;
                for (; t + B <= n; t += B) {
                    V x[B];
#pragma unroll
                    for (int j = 0; j < B; ++j) x[j] = tile[buf][(t + j) * CW + c];
#pragma unroll
                    for (int j = 0; j < B; ++j) apply_row(r0 + t + j, x[j]);
                }
                for (; t < n; ++t) apply_row(r0 + t, tile[buf][t * CW + c]);
            }
        }
        __syncthreads();
    }
    if (held && lane_ok) vstore<W, false>(d.dst + cur + xl, acc);
}

// COLUMN REDUCTION OF INTEGERS, rows split over workgroups:
// for COMEX_ACC_INT / _LNG the reference's per-row `A += B*C` wraps (unsigned
// arithmetic here, -fwrapv in the oracle), so a dst element's final value is its
// initial value plus the wrapped sum of its rows' products in ANY order.  A
// workgroup takes R consecutive rows of 256 element columns: the R loads of a
// lane are issued together (row-major streaming of the source, every row read in
// full 256-element pieces), the products of consecutive rows hitting the same dst
// run are summed in a register, and each run's partial goes into dst with one
// device-scope atomic add (the launcher takes this path only for a dst in HBM).
constexpr int kColsAtomicRows = 64;
template <class OP, int LV>
__global__ __launch_bounds__(256) void k_cols_atomic(const Desc d, const OP op) {
    typedef decltype(op.s) A;                      // uint32_t (INT) / uint64_t (LNG)
    constexpr int R = kColsAtomicRows;
    const uint32_t v = blockIdx.x * 256u + threadIdx.x;
    if (v >= d.nvec) return;
    const uint32_t rb = blockIdx.y * (uint32_t)R;
    const uint32_t n = min((uint32_t)R, d.rows - rb);
    const int64_t xo = (int64_t)v * sizeof(A);
    A x[R];
    int64_t dofs[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {                  // rows past the last load the last one again
        int64_t so;
        row_offsets<LV>(d, d.row0 + min(rb + (uint32_t)k, d.rows - 1u), so, dofs[k]);
        x[k] = __builtin_nontemporal_load(reinterpret_cast<const A *>(d.src + so + xo));
    }
    A part = 0;
    int64_t cur = dofs[0];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        if ((uint32_t)k >= n) break;
        if (dofs[k] != cur) {
            __hip_atomic_fetch_add(reinterpret_cast<A *>(d.dst + cur + xo), part, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            cur = dofs[k];
            part = 0;
        }
        A prod = x[k] * op.s;
        part = part + prod;
    }
    __hip_atomic_fetch_add(reinterpret_cast<A *>(d.dst + cur + xo), part, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The pure column reduction -- every row into ONE dst run (all dst strides of the
// row levels zero; the headline integer case of VERDICT r3 item 5).  What bounds it
// is how HBM is read, not arithmetic: a workgroup per 64 columns (512-byte row
// pieces at the row stride) reached 2.7 TB/s, 256-byte pieces 1.5 TB/s -- every
// piece opens DRAM pages for a fraction of their bytes.  So a workgroup here reads
// 4 KiB of each row (256 lanes x 16 bytes, the four waves side by side on the same
// row), over a slice of R rows with 16 rows in flight per lane; the grid is (row
// width / 4 KiB) x (row slices), and each lane adds its slice's partial sums into
// dst with device-scope atomic adds (wrapping integer sums are exact in any order;
// the launcher takes this path only for a 16-byte-aligned source and a dst in HBM).
constexpr int kColsSumP = 16;          // rows in flight per lane
constexpr int kColsSumTarget = 1024;   // workgroups to aim for (256: 4.53, 512: 4.19, 1024: 4.87-4.91 TB/s)
constexpr int kColsSumMinRows = 32;    // rows per slice at least
// row slices for a grid of gx column chunks over `rows` rows (the plan and the
// dispatcher agree through this)
static inline uint32_t cols_sum_slices(uint32_t gx, uint32_t rows) {
    uint32_t s = (kColsSumTarget + gx - 1) / gx;
    const uint32_t smax = (rows + kColsSumMinRows - 1) / kColsSumMinRows;
    if (s > smax) s = smax;
    if (s > 65535u) s = 65535u;
    return s ? s : 1;
}
template <class OP, int LV>
__global__ __launch_bounds__(256) void k_cols_sum(const Desc d, const OP op, uint32_t R) {
    typedef decltype(op.s) A;                      // uint32_t (INT) / uint64_t (LNG)
    typedef typename Vec<16>::T V;
    constexpr int E = 16 / (int)sizeof(A);
    constexpr int P = kColsSumP;
    const uint32_t v = blockIdx.x * 256u + threadIdx.x;   // this lane's 16-byte column vector
    const int64_t xo = (int64_t)min(v, d.nvec - 1u) * 16;
    const uint32_t rb = blockIdx.y * R, re = min(rb + R, d.rows);
    A part[E];
#pragma unroll
    for (int e = 0; e < E; ++e) part[e] = 0;
    for (uint32_t r0 = rb; r0 < re; r0 += P) {
        V x[P];
#pragma unroll
        for (int k = 0; k < P; ++k) {              // rows past the slice load its last row again
            int64_t so, dof;
            row_offsets<LV>(d, d.row0 + min(r0 + (uint32_t)k, re - 1u), so, dof);
            x[k] = vload<16, true>(d.src + so + xo);
        }
#pragma unroll
        for (int k = 0; k < P; ++k) {
            A y[E];
            __builtin_memcpy(y, &x[k], 16);
            if (r0 + (uint32_t)k < re) {
#pragma unroll
                for (int e = 0; e < E; ++e) part[e] = part[e] + y[e] * op.s;
            }
        }
    }
    if (v >= d.nvec) return;
    int64_t so, dof;
    row_offsets<LV>(d, d.row0, so, dof);           // the one dst run
    A *dp = reinterpret_cast<A *>(d.dst + dof + xo);
#pragma unroll
    for (int e = 0; e < E; ++e)
        __hip_atomic_fetch_add(dp + e, part[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// host launch plumbing
//
// Instantiation policy (only shipped choices are compiled): every
// (op, W) pair gets the rows kernels with one-wave and 128-thread blocks, one
// 16-byte vector per thread per stream (U = 16 / W vectors of narrower widths),
// non-temporal accesses; the flat kernel in one shape per width; the ordered,
// column-ordered and serial kernels; and one system-scope-source rows kernel
// (runtime levels, 256 threads) for sources in a peer GPU's memory.

// what the launcher decided for one call (the dispatcher's template selector)
struct Plan {
    int kind;        // KK_ROWS / KK_FLAT / KK_SERIAL / KK_ORDERED
    int W, U, BS;
    int variant;     // KK_ORDERED: 0 one workgroup, 1 column slices (pipelined), 2 column slices (in place),
                     // 3 integer column reduction with rows split over workgroups (atomic partials),
                     // 4 integer column reduction into one dst run (a workgroup per 64 columns, LDS sum)
    bool sys;        // KK_ROWS: source in a peer GPU's memory (system-scope loads)
    int cw;          // variant 1: columns per workgroup of the LDS-staged kernel (0: one lane per column)
};

// LDS-staged column kernel: column slices per workgroup -- 64 when that still
// gives >= 256 workgroups (one per CU), else the narrow form: one 128-byte line
// per row segment (16 slices of 8 B, 32 of 4 B; a 16-byte element keeps 16).
// Built for W = 4/8 and for 16-byte elements (W = 16); the column path never uses
// 16-byte vectors for smaller elements, and W = 1/2 keep one lane per column.
// One workgroup fits a CU (two 56 KiB LDS tiles) and its applier wave walks every
// row whatever CW is, so a launch takes about ceil(workgroups / CUs) applier
// passes: CW is the narrowest of 16/32/64 slices that keeps the workgroups within
// one pass over the 256 CUs (8192 slices of a 64 KiB f64 row: 32), never below one
// 128-byte line per row segment.
static int cols_per_group(uint32_t nvec, int W) {
    if (W != 4 && W != 8 && W != 16) return 0;
    int cw = W == 4 ? 32 : 16;
    while (cw < 64 && (nvec + (uint32_t)cw - 1) / (uint32_t)cw > 256u) cw *= 2;
    return cw;
}

template <class OP, int W, int LV>
static void go_cols_lds(const Desc &d, const OP &op, int cw, uint64_t blocks, hipStream_t st) {
    if constexpr ((W == 4 || W == 8) || (W == 16 && OP::kElem == 16)) {
        if (cw == 64)
            hipLaunchKernelGGL((k_ordered_cols_lds<OP, W, LV, 64>), dim3((uint32_t)blocks), dim3(KC_NW * 64), 0, st, d,
                               op);
        else if (cw == 32)
            hipLaunchKernelGGL((k_ordered_cols_lds<OP, W, LV, 32>), dim3((uint32_t)blocks), dim3(KC_NW * 64), 0, st, d,
                               op);
        else if constexpr (W >= 8)
            hipLaunchKernelGGL((k_ordered_cols_lds<OP, W, LV, 16>), dim3((uint32_t)blocks), dim3(KC_NW * 64), 0, st, d,
                               op);
    }
}

// flat kernel shape: one-wave blocks of one 16-byte vector per lane (+3.5-5 % on
// 128 B-1 KiB rows over 256 x 2, profiles/r01/sweep_flat_shape.jsonl); narrower
// vectors 256 threads x 4
static int flat_block_threads(int W) { return W == 16 ? 64 : 256; }
static uint64_t flat_block_items(int W) { return W == 16 ? 64 : 256ull * 4; }

// vectors per thread: 16 B per thread per stream (8 B for 1- and 2-byte vectors).
// unroll_for is the same table at run time: the launcher sizes its chunks with it,
// so it must agree with what the kernels are instantiated with (it once said 16
// for W = 1, and byte-wide rows kernels skipped half of every chunk: a put of odd-
// length rows longer than the flat kernel's limit; tests/test_gpu_fuzz.py).
template <int W> struct DefaultU { static constexpr int value = W == 16 ? 1 : (W == 8 ? 2 : (W == 4 ? 4 : 8)); };
static int unroll_for(int W) {
    switch (W) {
    case 16: return DefaultU<16>::value;
    case 8: return DefaultU<8>::value;
    case 4: return DefaultU<4>::value;
    case 2: return DefaultU<2>::value;
    default: return DefaultU<1>::value;
    }
}
constexpr int kSysBS = 256;   // peer-source rows kernel block

template <class OP, int W, int BS, bool SYS = false>
static hipError_t go_rows2(const Desc &d, const OP &op, uint64_t blocks, hipStream_t st) {
    constexpr int U = DefaultU<W>::value;
    Desc2 e;
    e.src = d.src;
    e.dst = d.dst;
    e.s_str = d.levels ? d.s_str[0] : 0;
    e.d_str = d.levels ? d.d_str[0] : 0;
    e.row0 = d.row0;
    e.nvec = d.nvec;
    e.chunks = d.chunks;
    e.items = (uint32_t)d.items;
    e.chunk_div = d.chunk_div;
    e.align_mask = d.align_mask;
    if constexpr (U == 1) {
        // whole chunks, one block each: the loop-free kernel
        if (!d.align_mask && blocks == e.items && d.nvec % (uint32_t)BS == 0) {
            Desc2D f;
            f.src = d.src;
            f.dst = d.dst;
            f.s_str = e.s_str;
            f.d_str = e.d_str;
            f.chunk_div = d.chunk_div;
            f.row0 = d.row0;
            hipLaunchKernelGGL((k_rows2d<OP, W, BS, SYS>), dim3((uint32_t)blocks), dim3(BS), 0, st, f, op);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((k_rows2<OP, W, U, BS, SYS>), dim3((uint32_t)blocks), dim3(BS), 0, st, e, op);
    return hipGetLastError();
}

template <class OP, int W, int LV, int BS>
static hipError_t go_rows_nd(const Desc &d, const OP &op, uint64_t blocks, hipStream_t st) {
    constexpr int U = DefaultU<W>::value;
    if constexpr (U == 1 && (LV == 2 || LV == 3)) {
        if (blocks == d.items && d.nvec % (uint32_t)BS == 0) {
            DescND<LV> f;
            f.src = d.src;
            f.dst = d.dst;
            for (int j = 0; j < LV; ++j) {
                f.s_str[j] = d.s_str[j];
                f.d_str[j] = d.d_str[j];
                f.cnt[j] = d.cnt[j];
            }
            f.chunk_div = d.chunk_div;
            f.row0 = d.row0;
            hipLaunchKernelGGL((k_rowsnd<OP, W, BS, LV>), dim3((uint32_t)blocks), dim3(BS), 0, st, f, op);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((k_rows<OP, W, U, BS, LV>), dim3((uint32_t)blocks), dim3(BS), 0, st, d, op);
    return hipGetLastError();
}
template <class OP, int W, int LV>
static hipError_t go_rows_nd(const Desc &d, const OP &op, uint64_t blocks, int BS, hipStream_t st) {
    if (BS == 64) return go_rows_nd<OP, W, LV, 64>(d, op, blocks, st);
    return go_rows_nd<OP, W, LV, 128>(d, op, blocks, st);
}

template <class OP, int W>
static hipError_t dispatch_w(const Plan &p, const Desc &d, const OP &op, uint64_t blocks, hipStream_t st) {
    if constexpr (W < OP::kElem) {
        return hipErrorInvalidValue;
    } else {
        if (p.kind == KK_SERIAL) {
            hipLaunchKernelGGL((k_serial<OP, W>), dim3(1), dim3(64), 0, st, d, op);
            return hipGetLastError();
        }
        if (p.kind == KK_ORDERED) {
            if (p.variant == 4) {           // integers into one dst run: 4 KiB row pieces, atomic partials
                if constexpr (std::is_same<OP, AccInt>::value || std::is_same<OP, AccLng>::value) {
                    if constexpr (W == 16) {
                        const uint32_t gx = (d.nvec + 255u) / 256u, sl = cols_sum_slices(gx, d.rows);
                        const uint32_t R = (d.rows + sl - 1) / sl;
                        const dim3 grid(gx, sl);
                        if (d.levels == 1) hipLaunchKernelGGL((k_cols_sum<OP, 1>), grid, dim3(256), 0, st, d, op, R);
                        else hipLaunchKernelGGL((k_cols_sum<OP, 0>), grid, dim3(256), 0, st, d, op, R);
                        return hipGetLastError();
                    }
                }
                return hipErrorInvalidValue;
            }
            if (p.variant == 3) {           // integers: rows split over workgroups, atomic partials
                if constexpr (std::is_same<OP, AccInt>::value || std::is_same<OP, AccLng>::value) {
                    if constexpr (W == OP::kElem) {
                        const dim3 grid((d.nvec + 255u) / 256u, (d.rows + kColsAtomicRows - 1) / kColsAtomicRows);
                        if (d.levels == 1) hipLaunchKernelGGL((k_cols_atomic<OP, 1>), grid, dim3(256), 0, st, d, op);
                        else hipLaunchKernelGGL((k_cols_atomic<OP, 0>), grid, dim3(256), 0, st, d, op);
                        return hipGetLastError();
                    }
                }
                return hipErrorInvalidValue;
            }
            if (p.variant == 1 && p.cw) {   // LDS-staged column slices
                if (d.levels == 1) go_cols_lds<OP, W, 1>(d, op, p.cw, blocks, st);
                else go_cols_lds<OP, W, 0>(d, op, p.cw, blocks, st);
                return hipGetLastError();
            }
            if (p.variant == 1 && d.levels == 1)   // 2-D: the row offset is one multiply
                hipLaunchKernelGGL((k_ordered_cols<OP, W, true, 1>), dim3((uint32_t)blocks), dim3(64), 0, st, d, op);
            else if (p.variant == 1)
                hipLaunchKernelGGL((k_ordered_cols<OP, W, true>), dim3((uint32_t)blocks), dim3(64), 0, st, d, op);
            else if (p.variant == 2)
                hipLaunchKernelGGL((k_ordered_cols<OP, W, false>), dim3((uint32_t)blocks), dim3(64), 0, st, d, op);
            else   // 64 bytes per thread per stream: 64 KiB chunks, one load round trip each
                hipLaunchKernelGGL((k_ordered<OP, W, 4 * DefaultU<W>::value>), dim3(1), dim3(kOrderedBS), 0, st, d, op);
            return hipGetLastError();
        }
        if (p.sys) {
            // <= 1 stride level (GA 2-D patches, packed chunks): the 2-D kernels with
            // system-scope source loads; deeper patches the generic rows kernel
            if (d.levels <= 1) {
                if (p.BS == 64) return go_rows2<OP, W, 64, true>(d, op, blocks, st);
                return go_rows2<OP, W, 128, true>(d, op, blocks, st);
            }
            hipLaunchKernelGGL((k_rows<OP, W, DefaultU<W>::value, kSysBS, 0, true>), dim3((uint32_t)blocks),
                               dim3(kSysBS), 0, st, d, op);
            return hipGetLastError();
        }
        if (p.kind == KK_FLAT) {
            constexpr int UF = (W == 16) ? 1 : 4;
            constexpr int FB = (W == 16) ? 64 : 256;
            if (d.levels == 1 && (uint64_t)d.nvec * W <= 32)
                hipLaunchKernelGGL((k_flat<OP, W, UF, FB, 1, true>), dim3((uint32_t)blocks), dim3(FB), 0, st, d, op);
            else if (d.levels == 1)
                hipLaunchKernelGGL((k_flat<OP, W, UF, FB, 1>), dim3((uint32_t)blocks), dim3(FB), 0, st, d, op);
            else if (d.levels == 2)
                hipLaunchKernelGGL((k_flat<OP, W, UF, FB, 2>), dim3((uint32_t)blocks), dim3(FB), 0, st, d, op);
            else
                hipLaunchKernelGGL((k_flat<OP, W, UF, FB, 0>), dim3((uint32_t)blocks), dim3(FB), 0, st, d, op);
            return hipGetLastError();
        }
        if (d.levels == 2) return go_rows_nd<OP, W, 2>(d, op, blocks, p.BS, st);
        if (d.levels == 3) return go_rows_nd<OP, W, 3>(d, op, blocks, p.BS, st);
        if (d.levels > 3) return go_rows_nd<OP, W, 0>(d, op, blocks, p.BS, st);
        if (p.BS == 64) return go_rows2<OP, W, 64>(d, op, blocks, st);
        return go_rows2<OP, W, 128>(d, op, blocks, st);
    }
}

template <class OP>
static hipError_t dispatch_op(const Plan &p, const Desc &d, const OP &op, uint64_t blocks, hipStream_t st) {
    switch (p.W) {
    case 16: return dispatch_w<OP, 16>(p, d, op, blocks, st);
    case 8: return dispatch_w<OP, 8>(p, d, op, blocks, st);
    case 4: return dispatch_w<OP, 4>(p, d, op, blocks, st);
    case 2: return dispatch_w<OP, 2>(p, d, op, blocks, st);
    case 1: return dispatch_w<OP, 1>(p, d, op, blocks, st);
    }
    return hipErrorInvalidValue;
}

static hipError_t dispatch(int op, const void *scale, const Plan &p, const Desc &d, uint64_t blocks, hipStream_t st) {
    switch (op) {
    case kOpCopy: return dispatch_op(p, d, CopyOp{}, blocks, st);
    case 37: { AccInt o; int32_t s; memcpy(&s, scale, 4); o.s = (uint32_t)s; return dispatch_op(p, d, o, blocks, st); }
    case 42: { AccLng o; int64_t s; memcpy(&s, scale, 8); o.s = (uint64_t)s; return dispatch_op(p, d, o, blocks, st); }
    case 39: { AccFlt o; memcpy(&o.s, scale, 4); return dispatch_op(p, d, o, blocks, st); }
    case 38: { AccDbl o; memcpy(&o.s, scale, 8); return dispatch_op(p, d, o, blocks, st); }
    case 40: { AccCpl o; float s[2]; memcpy(s, scale, 8); o.sr = s[0]; o.si = s[1]; return dispatch_op(p, d, o, blocks, st); }
    case 41: { AccDcp o; double s[2]; memcpy(s, scale, 16); o.sr = s[0]; o.si = s[1]; return dispatch_op(p, d, o, blocks, st); }
    }
    return hipErrorInvalidValue;
}


// Do two distinct rows of one side touch a common byte?  Sufficient test for
// "no": with levels sorted by |stride|, each stride covers the full extent of
// everything below it (the row itself is the innermost extent).
static bool rows_may_overlap(const int64_t *str, const uint32_t *cnt, int L, int64_t row_bytes) {
    int64_t s[kMaxLevels];
    uint32_t c[kMaxLevels];
    int n = 0;
    for (int j = 0; j < L; ++j)
        if (cnt[j] > 1) { s[n] = str[j] < 0 ? -str[j] : str[j]; c[n] = cnt[j]; ++n; }
    for (int i = 1; i < n; ++i)   // insertion sort by stride
        for (int k = i; k > 0 && s[k] < s[k - 1]; --k) { std::swap(s[k], s[k - 1]); std::swap(c[k], c[k - 1]); }
    int64_t extent = row_bytes;
    for (int i = 0; i < n; ++i) {
        if (s[i] < extent) return true;
        extent = s[i] * (int64_t)(c[i] - 1) + extent;
    }
    return false;
}

static void side_span(const int64_t *str, const uint32_t *cnt, int L, int64_t row_bytes, int64_t &lo, int64_t &hi) {
    lo = 0;
    hi = row_bytes;
    for (int j = 0; j < L; ++j) {
        const int64_t e = str[j] * (int64_t)(cnt[j] ? cnt[j] - 1 : 0);
        if (e < 0) lo += e; else hi += e;
    }
}

// Byte span [lo, hi) of rows [rb, re) of one side (re > rb).  Digits of the
// levels above the highest level k where rb and re-1 differ are fixed; the
// level-k digit runs monotonically from digit_k(rb) to digit_k(re-1); the
// levels below k may take any value.  Exact for one level, a tight bound above.
static void range_span(const int64_t *str, const uint32_t *cnt, int L, int64_t row_bytes, uint64_t rb, uint64_t re,
                       int64_t &lo, int64_t &hi) {
    uint32_t da[kMaxLevels], db[kMaxLevels];
    uint64_t a = rb, b = re - 1;
    for (int j = 0; j < L; ++j) {
        const uint32_t c = cnt[j] ? cnt[j] : 1;
        da[j] = (uint32_t)(a % c);
        db[j] = (uint32_t)(b % c);
        a /= c;
        b /= c;
    }
    int k = -1;
    for (int j = L - 1; j >= 0; --j)
        if (da[j] != db[j]) { k = j; break; }
    int64_t base = 0;
    for (int j = k + 1; j < L; ++j) base += (int64_t)da[j] * str[j];
    lo = base;
    hi = base + row_bytes;
    if (k >= 0) {
        const int64_t e0 = (int64_t)da[k] * str[k], e1 = (int64_t)db[k] * str[k];
        lo += std::min(e0, e1);
        hi += std::max(e0, e1);
        for (int j = 0; j < k; ++j) {
            const int64_t e = str[j] * (int64_t)(cnt[j] ? cnt[j] - 1 : 0);
            if (e < 0) lo += e; else hi += e;
        }
    }
}

// Byte offset of row r of one side (odometer digits over the levels).
static int64_t row_start(const int64_t *str, const uint32_t *cnt, int L, uint64_t r) {
    int64_t o = 0;
    for (int j = 0; j < L; ++j) {
        const uint32_t c = cnt[j] ? cnt[j] : 1;
        o += (int64_t)(r % c) * str[j];
        r /= c;
    }
    return o;
}

// How the rows of one call may be scheduled.  The reference applies them
// strictly in odometer order, each row in ascending element order (comex.c:
// 6936-6961 -> acc.h:137-143), so where bytes are shared the order decides the
// result:
//   OV_NONE     no byte of a dst row is touched by any other row (src or dst):
//               any order gives the reference's bytes -> the parallel kernels;
//   OV_ORDERED  dst rows share bytes with each other, or a src row shares bytes
//               with a dst row, but no src run starts inside its own dst run
//               below it -> rows in order, each row wave-parallel (k_ordered);
//   OV_SERIAL   some row's src run starts below its dst run and reaches into it
//               (s < d < s + row): element m reads bytes the same _acc loop
//               wrote at m' < m, a recurrence -> one lane in reference order.
//               (acc.h's loop reads each src element whole before its
//               statements -- restrict, acc.h:106-122 -- so a src run at or
//               above its dst run, in place included, only ever reads bytes
//               not yet written: no recurrence there.)
//   OV_COLS     order matters, but every two rows that share bytes start at the
//               same address (dst rows coincide -- a zero or repeated dst
//               stride -- and no src row meets a dst row): element x depends
//               only on element x of earlier rows -> column slices, each walked
//               in row order (k_ordered_cols, pipelined);
//   OV_COLS_SRC as OV_COLS, but some src row IS another row's dst run (same
//               start): column slices without the src prefetch.
// Exact (row intervals of both sides, sorted) up to kExactRows rows in the
// call; above that a bound on spans and on the per-row dst - src distance.
enum { OV_NONE = 0, OV_ORDERED = 1, OV_SERIAL = 2, OV_COLS = 3, OV_COLS_SRC = 4 };
constexpr uint64_t kExactRows = 1ull << 18;

static int classify_rows_exact(int64_t sb, const int64_t *ss, int64_t db, const int64_t *ds, const uint32_t *cn,
                               int L, int64_t rb, uint64_t r0, uint64_t r1) {
    const uint64_t n = r1 - r0;
    // spans of the rows this call touches: a chunked caller (remote pack /
    // unpack-acc) passes a row range and a packed base rebased so that row r0
    // lands at its slice -- the full-range span of such a side reaches far
    // outside the slice and would falsely meet the other side
    int64_t slo, shi, dlo, dhi;
    range_span(ss, cn, L, rb, r0, r1, slo, shi);
    range_span(ds, cn, L, rb, r0, r1, dlo, dhi);
    const bool same_layout = sb == db && !memcmp(ss, ds, sizeof(int64_t) * L);
    const bool spans_meet = !same_layout && sb + slo < db + dhi && db + dlo < sb + shi;
    const bool dst_may = n > 1 && rows_may_overlap(ds, cn, L, rb);
    if (!spans_meet && !dst_may) return OV_NONE;
    if (L == 1 && ss[0] == ds[0]) {
        // 2-D with one stride S on both sides (every GA patch of one array into
        // another patch of it): src row i is dst row i moved by delta = sb - db, and
        // src row i meets dst row j iff |delta + (i - j) S| < rb -- closed form
        const int64_t S = ss[0], delta = sb - db;
        if (delta < 0 && -delta < rb) return OV_SERIAL;         // d - s in (0, rb) on every row
        if (n > 1 && S == 0) {                                  // every dst row the same run
            if (delta == 0) return OV_COLS_SRC;                 // ... and every src row too
            return (delta < rb) ? OV_ORDERED : OV_COLS;         // a src run shifted into it, or apart
        }
        if (n > 1 && (S < 0 ? -S : S) < rb) return OV_ORDERED;  // dst rows share bytes at other offsets
        if (!spans_meet) return OV_NONE;
        const int64_t kmax = (int64_t)n - 1;
        const int64_t kc = S ? (int64_t)std::floor(-(double)delta / (double)S) : 0;
        bool same_start = false;
        for (int64_t k = kc - 1; k <= kc + 2; ++k) {
            if (k < -kmax || k > kmax) continue;
            const int64_t diff = delta + k * S;
            if (diff > -rb && diff < rb && !(k == 0 && diff == 0)) {
                if (diff != 0) return OV_ORDERED;
                same_start = true;                              // src row i == dst row i + k
            }
        }
        return same_start ? OV_COLS_SRC : OV_NONE;
    }
    if (n > kExactRows) {
        // bound: dst - src of a row is (db - sb) + sum_j digit_j * (ds_j - ss_j)
        int64_t lo = db - sb, hi = db - sb;
        for (int j = 0; j < L; ++j) {
            const int64_t e = (ds[j] - ss[j]) * (int64_t)(cn[j] ? cn[j] - 1 : 0);
            if (e < 0) lo += e; else hi += e;
        }
        if (spans_meet && hi > 0 && lo < rb) return OV_SERIAL;
        return OV_ORDERED;
    }
    std::vector<std::pair<int64_t, uint32_t>> S(spans_meet ? n : 0), D(n);
    for (uint64_t i = 0; i < n; ++i) {
        const int64_t s = sb + row_start(ss, cn, L, r0 + i), d = db + row_start(ds, cn, L, r0 + i);
        if (s < d && d < s + rb) return OV_SERIAL;
        D[i] = {d, (uint32_t)i};
        if (spans_meet) S[i] = {s, (uint32_t)i};
    }
    std::sort(D.begin(), D.end());
    bool dst_same = false;   // two dst rows at one start (and none at another overlapping offset)
    for (uint64_t k = 1; k < n; ++k) {
        if (D[k].first < D[k - 1].first + rb) {
            if (D[k].first != D[k - 1].first) return OV_ORDERED;
            dst_same = true;
        }
    }
    bool src_same = same_layout && dst_same;   // src row r' is the dst run of another row r
    if (spans_meet) {
        std::sort(S.begin(), S.end());
        for (const auto &x : D) {
            // src rows with a start in (d - rb, d + rb) share bytes with this dst row;
            // only the row's own src at the same address (dst = dst + a*dst) is harmless
            auto it = std::lower_bound(S.begin(), S.end(), std::make_pair(x.first - rb + 1, (uint32_t)0));
            for (; it != S.end() && it->first < x.first + rb; ++it) {
                if (it->first != x.first) return OV_ORDERED;
                if (it->second != x.second) src_same = true;
            }
        }
    }
    if (src_same) return OV_COLS_SRC;
    return dst_same ? OV_COLS : OV_NONE;
}

// The sorted-interval analysis costs O(rows log rows) of host time (~0.1 ms at
// 4096 rows) -- more than a headline launch -- and callers repeat geometries
// (the same GA patches, rotating buffers): its answers are kept in a small
// direct-mapped cache keyed by the whole geometry.
struct ClassifyKey {
    int64_t sb, db, rb;
    uint64_t r0, r1;
    int32_t L, pad;
    int64_t ss[kMaxLevels], ds[kMaxLevels];
    uint32_t cn[kMaxLevels];
    bool operator==(const ClassifyKey &o) const { return !memcmp(this, &o, sizeof(*this)); }
};
static std::mutex g_cls_mu;
static ClassifyKey g_cls_key[64];
static int g_cls_val[64];
static bool g_cls_used[64];

static int classify_rows(int64_t sb, const int64_t *ss, int64_t db, const int64_t *ds, const uint32_t *cn, int L,
                         int64_t rb, uint64_t r0, uint64_t r1) {
    ClassifyKey k;
    memset(&k, 0, sizeof(k));
    k.sb = sb;
    k.db = db;
    k.rb = rb;
    k.r0 = r0;
    k.r1 = r1;
    k.L = L;
    for (int j = 0; j < L; ++j) {
        k.ss[j] = ss[j];
        k.ds[j] = ds[j];
        k.cn[j] = cn[j];
    }
    uint64_t h = 1469598103934665603ull;
    const unsigned char *p = reinterpret_cast<const unsigned char *>(&k);
    for (size_t i = 0; i < sizeof(k); ++i) h = (h ^ p[i]) * 1099511628211ull;
    const int slot = (int)(h & 63);
    {
        std::lock_guard<std::mutex> g(g_cls_mu);
        if (g_cls_used[slot] && g_cls_key[slot] == k) return g_cls_val[slot];
    }
    const int v = classify_rows_exact(sb, ss, db, ds, cn, L, rb, r0, r1);
    std::lock_guard<std::mutex> g(g_cls_mu);
    g_cls_key[slot] = k;
    g_cls_val[slot] = v;
    g_cls_used[slot] = true;
    return v;
}

void side_span_host(const int *stride, const int *count, int stride_levels, int64_t row_bytes,
                    int64_t *lo, int64_t *hi) {
    int64_t str[kMaxLevels];
    uint32_t cnt[kMaxLevels];
    for (int j = 0; j < stride_levels && j < kMaxLevels; ++j) {
        str[j] = stride[j];
        cnt[j] = count[j + 1] < 0 ? 0 : (uint32_t)count[j + 1];
    }
    side_span(str, cnt, stride_levels, row_bytes, *lo, *hi);
}

int launch_strided(int op, const void *scale, const void *src, const int *src_stride,
                   void *dst, const int *dst_stride, const int *count, int stride_levels,
                   hipStream_t stream, LaunchInfo *info, uint64_t row_begin, uint64_t row_end, bool plan_only,
                   bool src_peer) {
    const Tuning &tn = g_tuning;
    if (info) memset(info, 0, sizeof(*info));
    if (stride_levels < 0 || stride_levels > kMaxLevels) return -2;
    if (!count || count[0] <= 0) return -3;
    const int esz = elem_size(op);
    if (!esz) return -4;
    if (op != kOpCopy && !scale) return -5;
    if (stride_levels > 0 && (!src_stride || !dst_stride)) return -6;

    // _acc processes bytes/sizeof(T) whole elements (acc.h:122)
    int64_t row_bytes = (op == kOpCopy) ? count[0] : (int64_t)(count[0] / esz) * esz;
    uint64_t rows = 1;
    for (int j = 1; j <= stride_levels; ++j) {
        if (count[j] < 0) return -3;
        rows *= (uint64_t)count[j];
    }
    if (rows == 0 || row_bytes == 0) return 0;   // nothing to do (reference loops 0 times)
    if (rows >= (1ull << 31)) return -7;
    if (row_end > rows) row_end = rows;
    if (row_begin >= row_end) return 0;
    const bool partial = row_begin != 0 || row_end != rows;

    // working copy of the levels; drop count==1 levels, merge contiguous ones
    int64_t ss[kMaxLevels], ds[kMaxLevels];
    uint32_t cn[kMaxLevels];
    int L = 0;
    for (int j = 0; j < stride_levels; ++j) {
        if (count[j + 1] == 1) continue;
        ss[L] = src_stride[j];
        ds[L] = dst_stride[j];
        cn[L] = (uint32_t)count[j + 1];
        ++L;
    }
    // merge level into the row when rows are back to back on both sides (only
    // when the row is whole elements, so _acc truncation is unchanged), and level
    // j+1 into level j when it continues it on both sides.  Both keep the
    // reference's visiting order of every byte (a merged row is the rows it
    // replaces, in order), so the ordering analysis below sees the same problem.
    while (!partial && L > 0 && ss[0] == row_bytes && ds[0] == row_bytes && (count[0] % esz) == 0 &&
           row_bytes * (int64_t)cn[0] < (1ll << 31)) {
        row_bytes *= cn[0];
        for (int j = 1; j < L; ++j) { ss[j - 1] = ss[j]; ds[j - 1] = ds[j]; cn[j - 1] = cn[j]; }
        --L;
    }
    for (int j = 0; j + 1 < L;) {
        if (ss[j + 1] == ss[j] * (int64_t)cn[j] && ds[j + 1] == ds[j] * (int64_t)cn[j] &&
            (uint64_t)cn[j] * cn[j + 1] < (1ull << 31)) {
            cn[j] *= cn[j + 1];
            for (int k = j + 1; k + 1 < L; ++k) { ss[k] = ss[k + 1]; ds[k] = ds[k + 1]; cn[k] = cn[k + 1]; }
            --L;
        } else {
            ++j;
        }
    }
    rows = 1;
    for (int j = 0; j < L; ++j) rows *= cn[j];
    if (!partial) row_end = rows;

    // ordering / aliasing: the reference applies rows strictly in order
    const int ov = classify_rows((int64_t)(uintptr_t)src, ss, (int64_t)(uintptr_t)dst, ds, cn, L, row_bytes,
                                 row_begin, row_end);
    // a source in a peer GPU's memory is read with system-scope loads by one rows
    // kernel; any order-dependent geometry is left to the caller, which packs
    // the rows into local memory first (the rows of src and dst then never meet)
    if (src_peer && ov != OV_NONE) return -10;
    const bool serial = !src_peer && (ov == OV_SERIAL || tn.kind == KK_SERIAL);
    const bool cols = !serial && tn.ordered_cols && (ov == OV_COLS || ov == OV_COLS_SRC);
    const bool ordered = !src_peer && !serial && (ov != OV_NONE || tn.kind == KK_ORDERED);

    // vector width: largest power of two <= 16 dividing every address and stride
    uint64_t a = (uint64_t)(uintptr_t)src | (uint64_t)(uintptr_t)dst | (uint64_t)row_bytes | 16;
    for (int j = 0; j < L; ++j) a |= (uint64_t)ss[j] | (uint64_t)ds[j];
    int W = (int)lowbit(a);
    if (W > 16) W = 16;
    // elements below their natural alignment (a Fortran complex*16 array is only
    // 8-byte aligned): one element per vector, read and written with dword-
    // aligned multi-dword accesses, which global memory serves at any dword
    // alignment; below 4 bytes the launcher refuses
    if (W < esz) {
        if (W < 4) return -8;
        W = esz;
    }
    if (serial) W = esz;
    // column slices: 8-byte lanes where the element allows (twice the lanes of
    // 16-byte vectors on a column reduction, whose parallelism is the row width)
    if (cols && W > 8 && esz <= 8) W = 8;
    // integer column reductions (COMEX_ACC_INT / _LNG, coinciding dst rows, no src row
    // meeting a dst row): rows split over workgroups with atomic partials -- wrapping
    // integer sums are exact in any order; device-scope atomics need the dst in HBM
    bool cols_atomic = false, cols_sum = false;
    if (cols && ov == OV_COLS && (op == 37 || op == 42) && tn.ordered_cols == 2 &&
        ((uint64_t)(uintptr_t)dst & (esz - 1)) == 0) {
        hipPointerAttribute_t at;
        memset(&at, 0, sizeof(at));
        bool hbm = false;
        if (hipPointerGetAttributes(&at, dst) == hipSuccess) hbm = at.type == hipMemoryTypeDevice;
        else (void)hipGetLastError();
        // every row into one dst run (the dst strides of all row levels zero), source
        // rows in whole 16-byte vectors: 4 KiB row pieces per workgroup
        uint64_t sa = (uint64_t)(uintptr_t)src | row_bytes;
        bool one_run = true;
        for (int j = 0; j < L; ++j) {
            one_run = one_run && ds[j] == 0;
            sa |= (uint64_t)ss[j];
        }
        cols_sum = hbm && one_run && (sa & 15) == 0;
        cols_atomic = hbm && !cols_sum && (row_end - row_begin) <= (uint64_t)kColsAtomicRows * 65535u;
    }
    if (cols_sum) W = 16;
    if (cols_atomic) W = esz;

    Desc d;
    memset(&d, 0, sizeof(d));
    d.src = (const char *)src;
    d.dst = (char *)dst;
    d.levels = L;
    for (int j = 0; j < L; ++j) {
        d.s_str[j] = ss[j];
        d.d_str[j] = ds[j];
        d.cnt[j] = make_fastdiv(cn[j]);
    }
    d.nvec = (uint32_t)(row_bytes / W);
    d.nvec_div = make_fastdiv(d.nvec);

    Plan p;
    memset(&p, 0, sizeof(p));
    int kind = serial ? KK_SERIAL : (ordered ? KK_ORDERED : (src_peer ? KK_ROWS : tn.kind));
    if (kind == KK_AUTO) {
        kind = ((int64_t)d.nvec <= tn.flat_max_nvec) ? KK_FLAT : KK_ROWS;
        // rows that start off 128-byte lines on both sides: the flat kernel's waves cut rows
        // (and their partial lines) at arbitrary vectors, the rows kernel keeps a row in one
        // block: rows kernel from flat_line_min vectors up (+9-28 % at 640 B-2 KiB rows
        // with ld = 2 x row + 16 B; line-aligned rows stay flat, which leads there by up to
        // 18 %: profiles/r01/flat_vs_rows_grid.jsonl)
        if (kind == KK_FLAT && tn.flat_line_min > 0 && (int64_t)d.nvec >= tn.flat_line_min) {
            uint64_t sa = (uint64_t)(uintptr_t)src, da = (uint64_t)(uintptr_t)dst;
            for (int j = 0; j < L; ++j) {
                sa |= (uint64_t)ss[j];
                da |= (uint64_t)ds[j];
            }
            if ((sa & 127) && (da & 127)) kind = KK_ROWS;
        }
    }
    // rows kernels: small blocks retire and free their CU slots independently;
    // on the headline shape 64/128/256/512/1024 threads measured
    // 6338/6268/6171/6020/5951 GB/s in a stand-alone probe (tools/h_shape_probe.hip).
    int block = tn.block;
    if (block != 64 && block != 128) {
        // auto: one-wave blocks when every row starts 4 KiB-aligned on both sides,
        // 128 threads otherwise (H-shape ld sweep, profiles/r01/sweep_ld_block.jsonl:
        // 64 leads by 1-6 % at ld 8192/8704/12288 and C3 by 4 %, 128 leads by 5-10 %
        // at ld 8194..8320, whose rows start off 4 KiB boundaries)
        uint64_t al = (uint64_t)(uintptr_t)src | (uint64_t)(uintptr_t)dst;
        for (int j = 0; j < L; ++j) al |= (uint64_t)ss[j] | (uint64_t)ds[j];
        block = (al & 4095) ? 128 : 64;
    }
    // the (U, BS) the dispatcher will pick -- chunking must agree with it
    const int U = unroll_for(W), BS = (src_peer && L > 1) ? kSysBS : block;
    p.kind = kind;
    p.W = W;
    p.U = U;
    p.BS = BS;
    p.sys = src_peer;
    p.variant = (kind == KK_ORDERED && cols) ? (cols_sum ? 4 : (cols_atomic ? 3 : (ov == OV_COLS ? 1 : 2))) : 0;
    p.cw = (p.variant == 1 && tn.ordered_cols == 2 && (W <= 8 || esz == 16)) ? cols_per_group(d.nvec, W) : 0;
    const uint32_t per_chunk = (uint32_t)BS * (uint32_t)U;
    d.align_mask = 0;
    if (tn.align && kind == KK_ROWS && L <= 1 && d.nvec >= 2 * per_chunk) {
        d.align_mask = per_chunk * (uint32_t)W - 1;   // a chunk spans per_chunk*W bytes
        // rows whose start is not chunk-aligned need one more (partial) chunk
        bool any = ((uintptr_t)dst & d.align_mask) != 0;
        for (int j = 0; j < L; ++j) any = any || (ds[j] & (int64_t)d.align_mask) != 0;
        if (!any) d.align_mask = 0;
    }
    d.chunks = (d.nvec + per_chunk - 1 + (d.align_mask ? per_chunk - 1 : 0)) / per_chunk;
    d.chunk_div = make_fastdiv(d.chunks);

    const uint64_t lim = (1ull << 31) - 1;
    uint64_t rows_per_launch = rows;
    if (kind == KK_ROWS) rows_per_launch = std::min<uint64_t>(rows, lim / d.chunks);
    if (kind == KK_FLAT) rows_per_launch = std::min<uint64_t>(rows, lim / d.nvec);
    if (kind == KK_SERIAL || kind == KK_ORDERED) rows_per_launch = rows;
    if (rows_per_launch == 0) return -9;

    int launches = 0;
    uint64_t total_blocks = 0;
    for (uint64_t r0 = row_begin; r0 < row_end; r0 += rows_per_launch) {
        const uint64_t nr = std::min<uint64_t>(rows_per_launch, row_end - r0);
        d.row0 = (uint32_t)r0;
        d.rows = (uint32_t)nr;
        uint64_t blocks = 1;
        if (kind == KK_ROWS) {
            d.items = nr * d.chunks;
            blocks = d.items;
            if (src_peer && L > 1 && blocks > 65536) blocks = 65536;   // grid-stride loop
        } else if (kind == KK_FLAT) {
            d.items = nr * d.nvec;
            const uint64_t per = flat_block_items(W);
            blocks = (d.items + per - 1) / per;
        } else {
            d.items = nr;
            if (p.variant == 4) {   // (4 KiB row pieces) x (row slices); the dispatcher builds the 2-D grid
                const uint32_t gx = (d.nvec + 255u) / 256u;
                blocks = (uint64_t)gx * cols_sum_slices(gx, (uint32_t)nr);
            }
            else if (p.variant == 3)   // (256-column chunks) x (row groups); the dispatcher builds the 2-D grid
                blocks = (uint64_t)((d.nvec + 255u) / 256u) * ((nr + kColsAtomicRows - 1) / kColsAtomicRows);
            else if (p.cw) blocks = (d.nvec + (uint32_t)p.cw - 1) / (uint32_t)p.cw;   // CW column slices per workgroup
            else if (p.variant) blocks = (d.nvec + 63u) / 64u;                   // one wave per 64 column slices
        }
        if (blocks > lim) blocks = lim;
        if (!plan_only) {
            hipError_t e = dispatch(op, scale, p, d, blocks, stream);
            if (e != hipSuccess) return -100 - (int)e;
        }
        ++launches;
        total_blocks += blocks;
    }
    if (!plan_only) g_kind_count[kind] += (unsigned long long)launches;
    if (info) {
        info->kind = kind;
        info->width = W;
        info->unroll = (kind == KK_ROWS) ? U : (kind == KK_ORDERED ? p.variant : 0);
        info->launches = launches;
        info->blocks = total_blocks;
        info->block = (kind == KK_ROWS) ? BS
                      : (kind == KK_FLAT ? flat_block_threads(W)
                                         : ((kind == KK_ORDERED && !p.variant) ? kOrderedBS
                                            : (p.variant == 4 || p.variant == 3 ? 256 : (p.cw ? KC_NW * 64 : 64))));
        info->levels = L;
        info->aligned = d.align_mask ? 1 : 0;
        info->sys = src_peer ? 1 : 0;
    }
    return 0;
}

}  // namespace gaamd
