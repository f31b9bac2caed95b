// gaamd_device.hpp -- device building blocks shared by the kernel files:
// W-byte vectors and their loads/stores (plain, non-temporal, system-scope),
// and the element operations -- copy, and the reference's _acc per type
// (comex/src-common/acc.h:46-49, 106-154) with FP contraction off.
#pragma once
#include "gaamd_kernels.h"
#include <string.h>
#include <type_traits>

#pragma clang fp contract(off)

namespace gaamd {

// lowest set bit (host and device)
__host__ __device__ inline uint64_t lowbit(uint64_t x) { return x & (~x + 1); }

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

// System-scope loads for bytes that live in ANOTHER GPU's HBM (a peer's staging
// or segment reached through its IPC mapping).  They must be served coherently at
// system scope: a line of the peer's memory this GPU's L2 still holds from an
// earlier read (MTYPE NC) must not be returned stale.  On gfx950 (LLVM's AMDGPU
// memory model, the GFX942 family) both a relaxed system-scope atomic load and a
// volatile load lower to `global_load_* sc0 sc1`; only the volatile form comes
// in every width, so W = 4/8/16 is ONE `global_load_dword{,x2,x4} ... sc0 sc1`
// (round 3 issued a system-scope dword per 4 bytes).  The
// memory model follows a volatile load with `s_waitcnt vmcnt(0)` (volatile
// accesses keep their order), so callers issue their other loads BEFORE the
// system-scope one: they are then in flight together.  Every vector the launcher
// builds is naturally aligned at its width W.  1/2-byte vectors stay atomic loads.
template <int W>
__device__ __forceinline__ typename Vec<W>::T vload_sys(const char *p) {
    typedef typename Vec<W>::T V;
    if constexpr (W == 1) {
        return __hip_atomic_load(reinterpret_cast<const uint8_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if constexpr (W == 2) {
        return __hip_atomic_load(reinterpret_cast<const uint16_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
        // through a global (addrspace 1) pointer: a generic one becomes flat_load
        typedef const volatile __attribute__((address_space(1))) V GV;
        return *(GV *)(p);
    }
}
template <int W, bool NT>
__device__ __forceinline__ void vstore(char *p, typename Vec<W>::T v) {
    typedef typename Vec<W>::T V;
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<V *>(p));
    else *reinterpret_cast<V *>(p) = v;
}

// ---------------------------------------------------------------------------
// element operations on one W-byte vector
// Each op also has serial_elem(dp, sp): one element through memory, for the
// one-lane kernel (src element read whole, then the statements of acc.h:46-49:
// the reference declares dst/src `restrict` and its compiled loop reads B once
// per element, acc.h:106-122).
struct CopyOp {
    static constexpr int kElem = 1;
    static constexpr bool kReadsDst = false;
    template <int W>
    __device__ __forceinline__ typename Vec<W>::T apply(typename Vec<W>::T, typename Vec<W>::T s) const { return s; }
    // apply() split into its source-only part and the combine (k_ordered_cols_lds:
    // loaders compute pre(src), the applier's chain is add(dst, pre(src)))
    template <int W>
    __device__ __forceinline__ typename Vec<W>::T pre(typename Vec<W>::T s) const { return s; }
    template <int W>
    __device__ __forceinline__ typename Vec<W>::T add(typename Vec<W>::T, typename Vec<W>::T i) const { return i; }
    __device__ __forceinline__ void serial_elem(char *dp, const char *sp) const { *dp = *sp; }
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
    // the same operations split: pre = the products, add = the sums (bit-identical)
    template <int W>
    __device__ __forceinline__ typename Vec<W>::T pre(typename Vec<W>::T sv) const {
        constexpr int N = W / (int)sizeof(T);
        union { typename Vec<W>::T v; A t[N]; } b;
        b.v = sv;
#pragma unroll
        for (int i = 0; i < N; ++i) b.t[i] = b.t[i] * s;
        return b.v;
    }
    template <int W>
    __device__ __forceinline__ typename Vec<W>::T add(typename Vec<W>::T dv, typename Vec<W>::T iv) const {
        constexpr int N = W / (int)sizeof(T);
        union { typename Vec<W>::T v; A t[N]; } a, b;
        a.v = dv; b.v = iv;
#pragma unroll
        for (int i = 0; i < N; ++i) a.t[i] = a.t[i] + b.t[i];
        return a.v;
    }
    __device__ __forceinline__ void serial_elem(char *dp, const char *sp) const {
        A *it = reinterpret_cast<A *>(dp);
        const A *v = reinterpret_cast<const A *>(sp);
        A prod = *v * s;
        *it = *it + prod;
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
    // the same operations split: pre = (re, im) of each source element, add = the sums
    template <int W>
    __device__ __forceinline__ typename Vec<W>::T pre(typename Vec<W>::T sv) const {
        constexpr int N = W / (int)(2 * sizeof(R));
        union { typename Vec<W>::T v; R t[2 * N]; } b;
        b.v = sv;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const R br = b.t[2 * i], bi = b.t[2 * i + 1];
            R p1 = br * sr;
            R p2 = bi * si;
            R re = p1 - p2;
            R p3 = br * si;
            R p4 = bi * sr;
            R im = p3 + p4;
            b.t[2 * i] = re;
            b.t[2 * i + 1] = im;
        }
        return b.v;
    }
    template <int W>
    __device__ __forceinline__ typename Vec<W>::T add(typename Vec<W>::T dv, typename Vec<W>::T iv) const {
        constexpr int N = W / (int)sizeof(R);
        union { typename Vec<W>::T v; R t[N]; } a, b;
        a.v = dv; b.v = iv;
#pragma unroll
        for (int i = 0; i < N; ++i) a.t[i] = a.t[i] + b.t[i];
        return a.v;
    }
    __device__ __forceinline__ void serial_elem(char *dp, const char *sp) const {
        R *it = reinterpret_cast<R *>(dp);
        const R *v = reinterpret_cast<const R *>(sp);
        const R br = v[0], bi = v[1];
        R p1 = br * sr;
        R p2 = bi * si;
        R re = p1 - p2;
        it[0] = it[0] + re;
        R p3 = br * si;
        R p4 = bi * sr;
        R im = p3 + p4;
        it[1] = it[1] + im;
    }
};

typedef AccReal<int32_t, uint32_t> AccInt;
typedef AccReal<int64_t, uint64_t> AccLng;
typedef AccReal<float, float> AccFlt;
typedef AccReal<double, double> AccDbl;
typedef AccCplx<float> AccCpl;
typedef AccCplx<double> AccDcp;

}  // namespace gaamd
