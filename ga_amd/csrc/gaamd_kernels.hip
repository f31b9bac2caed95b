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
//   * SERIAL kernel: one lane walks rows and elements in reference order; used
//     only when dst rows overlap each other or src overlaps dst, where the
//     reference result depends on its sequential order.
//   * Alpha travels in the kernel argument block (SGPRs), not LDS.
//   * FP contraction is OFF (pragma below + -ffp-contract=off): the reference
//     computes round(round(a*b)+c) with no FMA, so must we, bit for bit.
//     Integer types accumulate in unsigned arithmetic (wraparound, like the
//     reference's -fwrapv behaviour).
#pragma clang fp contract(off)

#include "gaamd_kernels.h"
#include <string.h>
#include <algorithm>

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
// vectors
template <int W> struct Vec;
template <> struct Vec<16> { typedef uint32_t __attribute__((ext_vector_type(4))) T; };
template <> struct Vec<8>  { typedef uint32_t __attribute__((ext_vector_type(2))) T; };
template <> struct Vec<4>  { typedef uint32_t T; };
template <> struct Vec<2>  { typedef uint16_t T; };
template <> struct Vec<1>  { typedef uint8_t T; };

template <int W, bool NT>
__device__ __forceinline__ typename Vec<W>::T vload(const char *p) {
    typedef typename Vec<W>::T V;
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const V *>(p));
    else return *reinterpret_cast<const V *>(p);
}
template <int W, bool NT>
__device__ __forceinline__ void vstore(char *p, typename Vec<W>::T v) {
    typedef typename Vec<W>::T V;
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<V *>(p));
    else *reinterpret_cast<V *>(p) = v;
}

// ---------------------------------------------------------------------------
// element operations on one W-byte vector
struct CopyOp {
    static constexpr int kElem = 1;
    static constexpr bool kReadsDst = false;
    template <int W>
    __device__ __forceinline__ typename Vec<W>::T apply(typename Vec<W>::T, typename Vec<W>::T s) const { return s; }
};

// dst += src*scale, acc.h:46 IADD_SCALE_REG; integers in unsigned arithmetic.
template <typename T, typename A>
struct AccReal {
    static constexpr int kElem = sizeof(T);
    static constexpr bool kReadsDst = true;
    A s;
    template <int W>
    __device__ __forceinline__ typename Vec<W>::T apply(typename Vec<W>::T dv, typename Vec<W>::T sv) const {
        constexpr int N = W / (int)sizeof(T);
        union { typename Vec<W>::T v; A t[N]; } a, b;
        a.v = dv; b.v = sv;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            A prod = b.t[i] * s;
            a.t[i] = a.t[i] + prod;
        }
        return a.v;
    }
};

// acc.h:47-49 IADD_SCALE_CPL with B = src, C = scale:
//   A.real += (B.real*C.real) - (B.imag*C.imag)
//   A.imag += (B.real*C.imag) + (B.imag*C.real)
template <typename R>
struct AccCplx {
    static constexpr int kElem = 2 * sizeof(R);
    static constexpr bool kReadsDst = true;
    R sr, si;
    template <int W>
    __device__ __forceinline__ typename Vec<W>::T apply(typename Vec<W>::T dv, typename Vec<W>::T sv) const {
        constexpr int N = W / (int)(2 * sizeof(R));
        union { typename Vec<W>::T v; R t[2 * N]; } a, b;
        a.v = dv; b.v = sv;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const R br = b.t[2 * i], bi = b.t[2 * i + 1];
            R p1 = br * sr;
            R p2 = bi * si;
            R re = p1 - p2;
            R p3 = br * si;
            R p4 = bi * sr;
            R im = p3 + p4;
            a.t[2 * i] = a.t[2 * i] + re;
            a.t[2 * i + 1] = a.t[2 * i + 1] + im;
        }
        return a.v;
    }
};

typedef AccReal<int32_t, uint32_t> AccInt;
typedef AccReal<int64_t, uint64_t> AccLng;
typedef AccReal<float, float> AccFlt;
typedef AccReal<double, double> AccDbl;
typedef AccCplx<float> AccCpl;
typedef AccCplx<double> AccDcp;

// ---------------------------------------------------------------------------
// row decode: byte offsets of row r on both sides (mixed radix over count[1..L])
__device__ __forceinline__ void row_offsets(const Desc &d, uint32_t r, int64_t &so, int64_t &dof) {
    so = 0;
    dof = 0;
#pragma unroll
    for (int j = 0; j < kMaxLevels; ++j) {
        if (j >= d.levels) break;
        const uint32_t q = d.cnt[j].div(r);
        const uint32_t dig = r - q * d.cnt[j].d;
        so += (int64_t)dig * d.s_str[j];
        dof += (int64_t)dig * d.d_str[j];
        r = q;
    }
}

// ---------------------------------------------------------------------------
// ROWS kernel: work item w = (row, chunk); chunk = BS*U vectors of that row.
template <class OP, int W, int U, int BS, bool NT>
__global__ __launch_bounds__(BS) void k_rows(const Desc d, const OP op) {
    typedef typename Vec<W>::T V;
    for (uint64_t w = blockIdx.x; w < d.items; w += gridDim.x) {
        const uint32_t rl = d.chunk_div.div((uint32_t)w);
        const uint32_t chunk = (uint32_t)w - rl * d.chunks;
        int64_t so, dof;
        row_offsets(d, d.row0 + rl, so, dof);
        const char *sp = d.src + so;
        char *dp = d.dst + dof;
        const uint32_t v0 = chunk * (uint32_t)(BS * U) + threadIdx.x;
        V a[U], b[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const uint32_t v = v0 + (uint32_t)(k * BS);
            if (v < d.nvec) {
                a[k] = vload<W, NT>(sp + (size_t)v * W);
                if constexpr (OP::kReadsDst) b[k] = vload<W, NT>(dp + (size_t)v * W);
            }
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const uint32_t v = v0 + (uint32_t)(k * BS);
            if (v < d.nvec) vstore<W, NT>(dp + (size_t)v * W, op.template apply<W>(b[k], a[k]));
        }
    }
}

// FLAT kernel: vectors of all rows flattened, each lane decodes its own row.
template <class OP, int W, int U, int BS>
__global__ __launch_bounds__(BS) void k_flat(const Desc d, const OP op) {
    typedef typename Vec<W>::T V;
    const uint64_t span = (uint64_t)BS * U;
    for (uint64_t base = (uint64_t)blockIdx.x * span; base < d.items; base += (uint64_t)gridDim.x * span) {
        V a[U], b[U];
        char *dps[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const uint64_t g = base + threadIdx.x + (uint64_t)k * BS;
            dps[k] = nullptr;
            if (g < d.items) {
                const uint32_t rl = d.nvec_div.div((uint32_t)g);
                const uint32_t v = (uint32_t)g - rl * d.nvec;
                int64_t so, dof;
                row_offsets(d, d.row0 + rl, so, dof);
                dps[k] = d.dst + dof + (size_t)v * W;
                a[k] = vload<W, false>(d.src + so + (size_t)v * W);
                if constexpr (OP::kReadsDst) b[k] = vload<W, false>(dps[k]);
            }
        }
#pragma unroll
        for (int k = 0; k < U; ++k)
            if (dps[k]) vstore<W, false>(dps[k], op.template apply<W>(b[k], a[k]));
    }
}

// SERIAL kernel: the reference's own order (row by row, element by element).
template <class OP, int W>
__global__ __launch_bounds__(64) void k_serial(const Desc d, const OP op) {
    if (threadIdx.x != 0) return;
    for (uint32_t r = 0; r < d.rows; ++r) {
        int64_t so, dof;
        row_offsets(d, d.row0 + r, so, dof);
        for (uint32_t v = 0; v < d.nvec; ++v) {
            char *dp = d.dst + dof + (size_t)v * W;
            typename Vec<W>::T a = vload<W, false>(d.src + so + (size_t)v * W);
            typename Vec<W>::T b = a;
            if constexpr (OP::kReadsDst) b = vload<W, false>(dp);
            vstore<W, false>(dp, op.template apply<W>(b, a));
        }
    }
}

// ---------------------------------------------------------------------------
// host launch plumbing
static int unroll_for(int W, int u16) {
    switch (W) {
    case 16: return u16;
    case 8: return 8;
    default: return 16;
    }
}

template <class OP, int W, int U>
static hipError_t go_rows(const Desc &d, const OP &op, uint64_t blocks, int nt, hipStream_t st) {
    if (nt) hipLaunchKernelGGL((k_rows<OP, W, U, 256, true>), dim3((uint32_t)blocks), dim3(256), 0, st, d, op);
    else hipLaunchKernelGGL((k_rows<OP, W, U, 256, false>), dim3((uint32_t)blocks), dim3(256), 0, st, d, op);
    return hipGetLastError();
}

template <class OP, int W>
static hipError_t dispatch_w(int kind, int U, int nt, const Desc &d, const OP &op, uint64_t blocks, hipStream_t st) {
    if constexpr (W < OP::kElem) {
        return hipErrorInvalidValue;
    } else {
        if (kind == KK_SERIAL) {
            hipLaunchKernelGGL((k_serial<OP, W>), dim3(1), dim3(64), 0, st, d, op);
            return hipGetLastError();
        }
        if (kind == KK_FLAT) {
            constexpr int UF = (W == 16) ? 2 : 4;
            hipLaunchKernelGGL((k_flat<OP, W, UF, 256>), dim3((uint32_t)blocks), dim3(256), 0, st, d, op);
            return hipGetLastError();
        }
        if constexpr (W == 16) {
            if (U == 2) return go_rows<OP, W, 2>(d, op, blocks, nt, st);
            if (U == 8) return go_rows<OP, W, 8>(d, op, blocks, nt, st);
            return go_rows<OP, W, 4>(d, op, blocks, nt, st);
        } else if constexpr (W == 8) {
            return go_rows<OP, W, 8>(d, op, blocks, 0, st);
        } else {
            return go_rows<OP, W, 16>(d, op, blocks, 0, st);
        }
    }
}

template <class OP>
static hipError_t dispatch_op(int W, int kind, int U, int nt, const Desc &d, const OP &op, uint64_t blocks, hipStream_t st) {
    switch (W) {
    case 16: return dispatch_w<OP, 16>(kind, U, nt, d, op, blocks, st);
    case 8: return dispatch_w<OP, 8>(kind, U, nt, d, op, blocks, st);
    case 4: return dispatch_w<OP, 4>(kind, U, nt, d, op, blocks, st);
    case 2: return dispatch_w<OP, 2>(kind, U, nt, d, op, blocks, st);
    case 1: return dispatch_w<OP, 1>(kind, U, nt, d, op, blocks, st);
    }
    return hipErrorInvalidValue;
}

static hipError_t dispatch(int op, const void *scale, int W, int kind, int U, int nt,
                           const Desc &d, uint64_t blocks, hipStream_t st) {
    switch (op) {
    case kOpCopy: return dispatch_op(W, kind, U, nt, d, CopyOp{}, blocks, st);
    case 37: { AccInt o; int32_t s; memcpy(&s, scale, 4); o.s = (uint32_t)s; return dispatch_op(W, kind, U, nt, d, o, blocks, st); }
    case 42: { AccLng o; int64_t s; memcpy(&s, scale, 8); o.s = (uint64_t)s; return dispatch_op(W, kind, U, nt, d, o, blocks, st); }
    case 39: { AccFlt o; memcpy(&o.s, scale, 4); return dispatch_op(W, kind, U, nt, d, o, blocks, st); }
    case 38: { AccDbl o; memcpy(&o.s, scale, 8); return dispatch_op(W, kind, U, nt, d, o, blocks, st); }
    case 40: { AccCpl o; float s[2]; memcpy(s, scale, 8); o.sr = s[0]; o.si = s[1]; return dispatch_op(W, kind, U, nt, d, o, blocks, st); }
    case 41: { AccDcp o; double s[2]; memcpy(s, scale, 16); o.sr = s[0]; o.si = s[1]; return dispatch_op(W, kind, U, nt, d, o, blocks, st); }
    }
    return hipErrorInvalidValue;
}

static inline uint64_t lowbit(uint64_t x) { return x & (~x + 1); }

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
                   hipStream_t stream, LaunchInfo *info, uint64_t row_begin, uint64_t row_end) {
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
    // ordering / aliasing: the reference applies rows strictly in order
    const bool dst_overlap = rows_may_overlap(ds, cn, L, row_bytes);
    bool src_dst_overlap = false;
    {
        int64_t slo, shi, dlo, dhi;
        side_span(ss, cn, L, row_bytes, slo, shi);
        side_span(ds, cn, L, row_bytes, dlo, dhi);
        const int64_t sb = (int64_t)(uintptr_t)src, db = (int64_t)(uintptr_t)dst;
        const bool same_layout = (src == dst) && !memcmp(ss, ds, sizeof(int64_t) * L);
        if (!same_layout && sb + slo < db + dhi && db + dlo < sb + shi) src_dst_overlap = true;
    }
    const bool serial = dst_overlap || src_dst_overlap || tn.kind == KK_SERIAL;

    if (!serial) {
        // merge level into the row when rows are back to back on both sides
        // (only when the row is whole elements, so _acc truncation is unchanged)
        while (!partial && L > 0 && ss[0] == row_bytes && ds[0] == row_bytes && (count[0] % esz) == 0 &&
               row_bytes * (int64_t)cn[0] < (1ll << 31)) {
            row_bytes *= cn[0];
            for (int j = 1; j < L; ++j) { ss[j - 1] = ss[j]; ds[j - 1] = ds[j]; cn[j - 1] = cn[j]; }
            --L;
        }
        // merge level j+1 into level j when it continues it on both sides
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
    }
    rows = 1;
    for (int j = 0; j < L; ++j) rows *= cn[j];
    if (!partial) row_end = rows;

    // vector width: largest power of two <= 16 dividing every address and stride
    uint64_t a = (uint64_t)(uintptr_t)src | (uint64_t)(uintptr_t)dst | (uint64_t)row_bytes | 16;
    for (int j = 0; j < L; ++j) a |= (uint64_t)ss[j] | (uint64_t)ds[j];
    int W = (int)lowbit(a);
    if (W > 16) W = 16;
    if (W < esz) return -8;   // elements not naturally aligned
    if (serial) W = esz;

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

    int kind = serial ? KK_SERIAL : tn.kind;
    if (kind == KK_AUTO) kind = ((int64_t)d.nvec <= tn.flat_max_nvec) ? KK_FLAT : KK_ROWS;
    const int U = unroll_for(W, tn.unroll16);
    const uint32_t per_chunk = 256u * (uint32_t)U;
    d.chunks = (d.nvec + per_chunk - 1) / per_chunk;
    d.chunk_div = make_fastdiv(d.chunks);

    const uint64_t lim = (1ull << 31) - 1;
    uint64_t rows_per_launch = rows;
    if (kind == KK_ROWS) rows_per_launch = std::min<uint64_t>(rows, lim / d.chunks);
    if (kind == KK_FLAT) rows_per_launch = std::min<uint64_t>(rows, lim / d.nvec);
    if (kind == KK_SERIAL) rows_per_launch = rows;
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
        } else if (kind == KK_FLAT) {
            d.items = nr * d.nvec;
            const int UF = (W == 16) ? 2 : 4;
            blocks = (d.items + 256ull * UF - 1) / (256ull * UF);
        } else {
            d.items = nr;
        }
        if (tn.max_grid > 0 && blocks > (uint64_t)tn.max_grid) blocks = (uint64_t)tn.max_grid;
        if (blocks > lim) blocks = lim;
        hipError_t e = dispatch(op, scale, W, kind, U, tn.nontemporal, d, blocks, stream);
        if (e != hipSuccess) return -100 - (int)e;
        ++launches;
        total_blocks += blocks;
    }
    if (info) {
        info->kind = kind;
        info->width = W;
        info->unroll = (kind == KK_ROWS) ? U : 0;
        info->launches = launches;
        info->blocks = total_blocks;
    }
    return 0;
}

}  // namespace gaamd
