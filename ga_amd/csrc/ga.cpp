// ga.cpp -- the Global Arrays caller of the accumulate path (SURVEY.md §8(a)
// row a15) over the MI355X ARMCI/ComEx runtime.
//
// Reference (paths in the GA tree):
//   NGA_Create / NGA_Create_irreg / NGA_Acc ...  global/src/capi.c:164-265, 2079-2089
//     (C order, 0-based  ->  Fortran order, 1-based: COPYC2F/COPYINDEX_C2F capi.c:54-61)
//   process grid            ddb, ddb_h2, ddb_ex, dd_ev, dd_su  global/src/decomp.c:125-758
//   block map               pnga_allocate  global/src/base.c:2550-2630
//   owner iteration         gai_iterator_*  global/src/iterator.c:188-771 (REGULAR)
//   ngai_acc_common         global/src/onesided.c:1334-1453: per owner
//       pbuf = buf + size*gam_ComputePatchIndex (onesided.c:330-337)
//       count = gam_ComputeCount, count[0] *= size (base.h:341-344)
//       stride_loc/stride_rem = gam_setstride (base.h:322-331)
//       remote owners first, then SMP-local; ARMCI_NbAccS for all but the last
//   statistics              GAstat.numacc, GAbytes.acctot/accloc (onesided.c:1372-1419)
// Each rank's block is column-major with the block's extents as leading
// dimensions (no ghosts), in one comex_malloc segment per array (HBM).
//
// This file is its own library, libga_amd_ga.so, linked against libga_amd.so
// and calling it only through the public C ABI (comex.h, armci.h, ga_amd.h) --
// the same position global/src has over libarmci.  libga_amd.so itself exports
// only comex_*/ARMCI_*/armci_*/gaamd_* names (as libarmci does, capi.c:14-27),
// so a real GA, which defines NGA_*/GA_* itself (global/src/capi.c:2079-2089),
// links against it without a second definition of its own entry points.
// built with -fvisibility=hidden: only the names the headers declare are exported
#pragma GCC visibility push(default)
#include "../../include/ga.h"
#include "../../include/armci.h"
#include "../../include/comex.h"
#include "../../include/ga_amd.h"
#pragma GCC visibility pop
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <functional>
#include <thread>
#include <string>
#include <vector>

namespace gaamd_ga {

// GA_Error / pnga_error: message, then abort through the runtime (comex_error ->
// the reference's MPI_Abort, comex_impl.h:52-76)
[[noreturn]] static void fatal(const char *fmt, ...) {
    char buf[768];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    char msg[800];
    snprintf(msg, sizeof(msg), "ga_amd GA: %s", buf);
    comex_error(msg, 1);
    abort();   // comex_error does not return
}

static int my_rank() {
    int me = 0;
    comex_group_rank(COMEX_GROUP_WORLD, &me);
    return me;
}

static int world_size() {
    int n = 1;
    comex_group_size(COMEX_GROUP_WORLD, &n);
    return n;
}

struct GArray {
    bool live = false;
    int type = 0, ndim = 0, elemsize = 0, optype = 0;
    std::string name;
    long dims[GA_MAX_DIM] = {0};        // Fortran order
    int nblock[GA_MAX_DIM] = {0};       // blocks (processes) per dimension
    std::vector<long> map[GA_MAX_DIM];  // 1-based first index of every block
    std::vector<void *> ptr;            // each rank's block (owner's address space)
    int nproc_grid = 0;
};

static std::vector<GArray> g_arrays;
static struct {
    long numacc = 0, numput = 0, numget = 0, numsca = 0, numgat = 0;
    double acctot = 0, accloc = 0, scatot = 0, scaloc = 0, gattot = 0, gatloc = 0;
} g_stat;

static GArray &arr(int g_a) {
    if (g_a < 1 || g_a > (int)g_arrays.size() || !g_arrays[g_a - 1].live) fatal("invalid global array handle %d", g_a);
    return g_arrays[g_a - 1];
}

static int type_size(int type, int *optype) {
    switch (type) {   // onesided.c:1362-1368
    case C_DBL: *optype = COMEX_ACC_DBL; return 8;
    case C_FLOAT: *optype = COMEX_ACC_FLT; return 4;
    case C_DCPL: *optype = COMEX_ACC_DCP; return 16;
    case C_SCPL: *optype = COMEX_ACC_CPL; return 8;
    case C_INT: *optype = COMEX_ACC_INT; return 4;
    case C_LONG: *optype = COMEX_ACC_LNG; return 8;
    }
    fatal("type %d not supported", type);
}

// ---- process grid: decomp.c restated ---------------------------------------
// dd_ev (decomp.c:711-722): load-balance ratio of a grid
static double dd_ev(int ndims, const long *ardims, const long *pedims) {
    double t = 1.0;
    for (int k = 0; k < ndims; k++) {
        const double q = (double)((ardims[k] / pedims[k]) * pedims[k]);
        t = t * (q / (double)ardims[k]);
    }
    return t;
}

// dd_su (decomp.c:730-738)
static void dd_su(int ndims, const long *ardims, const long *pedims, long *blk) {
    for (int i = 0; i < ndims; i++) {
        blk[i] = ardims[i] / pedims[i];
        if (blk[i] < 1) blk[i] = 1;
    }
}

// ddb_ex (decomp.c:213-333): exhaustive search over factorisations of npes,
// best load balance first, then least communication volume
static void ddb_ex(int ndims, const long *ardims, long npes, double threshold, long *blk, long *pedims) {
    if (ndims == 1) {
        pedims[0] = npes;
        dd_su(1, ardims, pedims, blk);
        return;
    }
    std::vector<long> tard(ndims), tdims(ndims, 0), stack(ndims, 0);
    for (int i = 0; i < ndims; i++) if (blk[i] < 1) blk[i] = 1;
    for (int i = 0; i < ndims; i++) tard[i] = ardims[i] / blk[i];
    for (int i = 0; i < ndims; i++) if (tard[i] < 1) { tard[i] = 1; blk[i] = ardims[i]; }
    double blb = -1.0;
    long bev = 1;
    for (int i = 0; i < ndims; i++) bev *= tard[i];
    pedims[0] = npes;
    for (int i = 1; i < ndims; i++) pedims[i] = 1;
    tdims[0] = 0;
    stack[0] = npes;
    int pc = 0;
    bool done = false;
    do {
        if (pc == ndims - 1) {
            tdims[pc] = stack[pc];
            const double clb = dd_ev(ndims, tard.data(), tdims.data());
            long cev = 0;
            for (int k = 0; k < ndims; k++) {
                long r = 1;
                for (int j = 0; j < ndims; j++) if (j != k) r = r * (tard[j] / tdims[j]);
                cev = cev + r;
            }
            if (clb > blb || (clb == blb && cev < bev)) {
                for (int j = 0; j < ndims; j++) pedims[j] = tdims[j];
                blb = clb;
                bev = cev;
            }
            if (blb > threshold) break;
            tdims[pc] = 0;
            pc -= 1;
        } else {
            if (tdims[pc] == stack[pc]) {
                done = (pc == 0);
                tdims[pc] = 0;
                pc -= 1;
            } else {
                for (tdims[pc] += 1; stack[pc] % tdims[pc] != 0; tdims[pc] += 1) {}
                pc += 1;
                stack[pc] = npes;
                for (int i = 0; i < pc; i++) stack[pc] /= tdims[i];
                tdims[pc] = 0;
            }
        }
    } while (!done);
    dd_su(ndims, ardims, pedims, blk);
}

// ddb_h2 (decomp.c:611-703): deal the prime factors of npes to the axes
static void ddb_h2(int ndims, const long *ardims, long npes, double threshold, long bias, long *blk, long *pedims) {
    std::vector<long> tard(ndims);
    for (int i = 0; i < ndims; i++) if (blk[i] < 1) blk[i] = 1;
    for (int i = 0; i < ndims; i++) tard[i] = (ardims[i] + blk[i] - 1) / blk[i];
    for (int i = 0; i < ndims; i++) if (tard[i] < 1) { tard[i] = 1; blk[i] = ardims[i]; }
    std::vector<long> pdivs;
    for (long i = 1; i <= npes; i++) if (npes % i == 0) pdivs.push_back(i);
    long npdivs = (long)pdivs.size();
    if (npdivs > 1) {   // prime divisors with repetition
        long k = 1;
        do {
            long h = k + 1;
            for (long j = h; j < npdivs; j++)
                if (pdivs[j] % pdivs[k] == 0) pdivs[h++] = pdivs[j] / pdivs[k];
            npdivs = h;
            k = k + 1;
        } while (k < npdivs);
    }
    long istep = 1, istart = 0;
    if (bias > 0) { istep = -1; istart = ndims - 1; }
    for (int j = 0; j < ndims; j++) pedims[j] = 1;
    for (long k = npdivs - 1; k >= 1; k--) {
        const long p0 = pdivs[k];
        long h = istart;
        double q = (tard[istart] < p0 * pedims[istart]) ? 1.1
                   : (double)(tard[istart] % (p0 * pedims[istart])) / (double)tard[istart];
        for (int j = 1; j < ndims; j++) {
            const long ilook = (istart + istep * j) % ndims;
            const double w = (tard[ilook] < p0 * pedims[ilook]) ? 1.1
                             : (double)(tard[ilook] % (p0 * pedims[ilook])) / (double)tard[ilook];
            if (w < q) { q = w; h = ilook; }
        }
        pedims[h] *= p0;
        if (bias == 0) istart = (istart + 1) % ndims;
    }
    const double ub = dd_ev(ndims, tard.data(), pedims);
    if (ub < threshold) ddb_ex(ndims, tard.data(), npes, threshold, blk, pedims);
    dd_su(ndims, ardims, pedims, blk);
    for (int i = 0; i < ndims; i++) {
        if (pedims[i] <= 0) fatal("process dimension is zero: ddb_h2");
        blk[i] = (tard[i] + pedims[i] - 1) / pedims[i];
    }
}

// ddb (decomp.c:125-199): user-chunked axes first, ddb_h2 on the rest
static void ddb(int ndims, const long *ardims, long npes, long *blk, long *pedims) {
    const double threshold = 0.1;
    long tp = npes, count = 0;
    for (int i = ndims - 1; i >= 0; i--) {
        if (blk[i] <= 0) {
            pedims[i] = -1;
            count += 1;
        } else {
            long sp = (ardims[i] + blk[i] - 1) / blk[i];
            if (sp > tp) {
                sp = tp;
                tp = 1;
                pedims[i] = sp;
            } else {
                long j;
                for (j = sp; j < tp && (tp % j != 0); j++) {}
                pedims[i] = j;
                tp = tp / j;
            }
        }
    }
    if (count > 0) {
        std::vector<long> tardim, tblk(count, 1), tpedim(count, 0);
        for (int j = 0; j < ndims; j++) if (pedims[j] < 0) tardim.push_back(ardims[j]);
        ddb_h2((int)count, tardim.data(), tp, threshold, 0, tblk.data(), tpedim.data());
        for (int i = 0, j = 0; j < ndims; j++)
            if (pedims[j] < 0) { blk[j] = (tardim[i] + tpedim[i] - 1) / tpedim[i]; i++; }
        for (int i = 0, j = 0; j < ndims; j++) if (pedims[j] < 0) pedims[j] = tpedim[i++];
    }
}

// ---- allocation --------------------------------------------------------------
static long block_elems(const GArray &a, int proc, long *lo, long *hi) {
    // ga_ownsM_no_handle (base.h:153-180): proc -> block coordinates, dim 0 fastest
    long n = 1;
    int idx = proc;
    for (int d = 0; d < a.ndim; d++) {
        const int loc = idx % a.nblock[d];
        idx /= a.nblock[d];
        lo[d] = a.map[d][loc];
        hi[d] = (loc + 1 < a.nblock[d]) ? a.map[d][loc + 1] - 1 : a.dims[d];
        n *= std::max(0L, hi[d] - lo[d] + 1);
    }
    if (proc >= a.nproc_grid) {
        for (int d = 0; d < a.ndim; d++) { lo[d] = 0; hi[d] = -1; }
        return 0;
    }
    return n;
}

// a rank's own block: HBM is zeroed on the device; a host segment (COMEX_AMD_SEGMENT=host)
// the way pnga_zero does it, memset through the host pointer (global.nalg.c:94-129)
static void zero_block(void *p, size_t bytes) {
    if (!bytes) return;
    if (gaamd_segment_kind(p) == 2) memset(p, 0, bytes);
    else if (gaamd_memset(p, 0, bytes) != 0) fatal("zeroing a %zu-byte block failed", bytes);
}

static int allocate(GArray &a) {
    const int me = my_rank(), np = world_size();
    long lo[GA_MAX_DIM], hi[GA_MAX_DIM];
    a.nproc_grid = 1;
    for (int d = 0; d < a.ndim; d++) a.nproc_grid *= a.nblock[d];
    if (a.nproc_grid > np) fatal("distribution needs %d processes, have %d", a.nproc_grid, np);
    const long n = block_elems(a, me, lo, hi);
    a.ptr.assign(np, nullptr);
    if (comex_malloc(a.ptr.data(), (size_t)n * a.elemsize, COMEX_GROUP_WORLD) != COMEX_SUCCESS) return 0;
    zero_block(a.ptr[me], (size_t)n * a.elemsize);
    comex_barrier(COMEX_GROUP_WORLD);
    a.live = true;
    g_arrays.push_back(a);
    return (int)g_arrays.size();
}

// ---- owner iteration + the per-owner ARMCI call (ngai_*_common) ---------------
enum GaOp { GA_ACC, GA_PUT, GA_GET };

// skip != nullptr: the strided (every skip[d]-th element) variants,
// pnga_strided_acc/put/get (onesided.c:4225-4470).  nb != nullptr: the
// non-blocking variants (pnga_nbacc/nbput/nbget, onesided.c:685, 1300, 1481):
// every owner's transfer is non-blocking and its handle is returned.
static void patch_op(GaOp kind, int g_a, const long *lo, const long *hi, void *buf, const long *ld, void *alpha,
                     const long *skip = nullptr, std::vector<armci_hdl_t> *nb = nullptr) {
    GArray &a = arr(g_a);
    const int me = my_rank();
    const int nd = a.ndim, size = a.elemsize;
    for (int d = 0; d < nd; d++)
        if (lo[d] < 1 || hi[d] > a.dims[d] || lo[d] > hi[d]) fatal("patch out of range in dim %d", d);
    // blocks of every dimension that intersect [lo, hi] (pnga_locate_region)
    int b0[GA_MAX_DIM], b1[GA_MAX_DIM];
    for (int d = 0; d < nd; d++) {
        const std::vector<long> &m = a.map[d];
        b0[d] = (int)(std::upper_bound(m.begin(), m.end(), lo[d]) - m.begin()) - 1;
        b1[d] = (int)(std::upper_bound(m.begin(), m.end(), hi[d]) - m.begin()) - 1;
    }
    long elems = 1;
    for (int d = 0; d < nd; d++) elems *= hi[d] - lo[d] + 1;
    if (kind == GA_ACC) { g_stat.numacc++; g_stat.acctot += (double)size * elems; }
    else if (kind == GA_PUT) g_stat.numput++;
    else g_stat.numget++;

    struct Owner { int proc; long plo[GA_MAX_DIM], phi[GA_MAX_DIM], ldrem[GA_MAX_DIM], blo[GA_MAX_DIM]; };
    std::vector<Owner> owners;
    int bi[GA_MAX_DIM];
    for (int d = 0; d < nd; d++) bi[d] = b0[d];
    for (;;) {
        Owner o;
        int proc = 0, mul = 1;
        for (int d = 0; d < nd; d++) { proc += bi[d] * mul; mul *= a.nblock[d]; }
        long blo[GA_MAX_DIM], bhi[GA_MAX_DIM];
        block_elems(a, proc, blo, bhi);
        o.proc = proc;
        for (int d = 0; d < nd; d++) {
            o.plo[d] = std::max(lo[d], blo[d]);
            o.phi[d] = std::min(hi[d], bhi[d]);
            o.ldrem[d] = bhi[d] - blo[d] + 1;
            o.blo[d] = blo[d];
        }
        owners.push_back(o);
        int d = 0;
        while (d < nd && ++bi[d] > b1[d]) { bi[d] = b0[d]; ++d; }
        if (d == nd) break;
    }
    // remote owners first, then the local one (onesided.c:1387-1400); the
    // strided variants keep the iterator's order (gai_iterator_next)
    if (!skip)
        std::stable_partition(owners.begin(), owners.end(), [&](const Owner &o) { return o.proc != me; });
    std::vector<armci_hdl_t> hdl;
    for (size_t k = 0; k < owners.size(); ++k) {
        Owner &o = owners[k];
        int count[2 * GA_MAX_DIM], stride_rem[2 * GA_MAX_DIM], stride_loc[2 * GA_MAX_DIM];
        int levels = nd - 1;
        char *pbuf, *prem;
        if (skip) {
            // gai_correct_strided_patch (onesided.c:4051-4070): first/last selected element
            bool empty = false;
            for (int d = 0; d < nd; d++) {
                long delta = o.plo[d] - lo[d];
                if (delta % skip[d]) o.plo[d] = o.plo[d] - delta % skip[d] + skip[d];
                delta = o.phi[d] - lo[d];
                if (delta % skip[d]) o.phi[d] -= delta % skip[d];
                if (o.phi[d] < o.plo[d]) empty = true;
            }
            if (empty) continue;
            // gai_FindOffset(blo, plo, ldrem) (4204-4216): remote offset of plo
            long roff = 0, rf = 1;
            for (int d = 0; d < nd; d++) { roff += (o.plo[d] - o.blo[d]) * rf; if (d < nd - 1) rf *= o.ldrem[d]; }
            prem = (char *)a.ptr[o.proc] + (long)size * roff;
            // gai_ComputePatchIndexWithSkip (4178-4202): the local buffer holds only
            // the selected elements
            long idx = (o.plo[0] - lo[0]) / skip[0];
            for (int d = 0; d < nd - 1; d++) idx += ld[d] * ((o.plo[d + 1] - lo[d + 1]) / skip[d + 1]);
            pbuf = (char *)buf + (long)size * idx;
            // gai_ComputeCountWithSkip (4077-4100, the "#if 1" form): one element per
            // run, then the selected elements of every dimension as stride levels
            count[0] = size;
            for (int d = 0; d < nd; d++) count[d + 1] = (int)((o.phi[d] - o.plo[d]) / skip[d] + 1);
            levels = nd;
            // gai_SetStrideWithSkip (4135-4150, "#if 1"); the reference also reads
            // ld[ndim-1], past the ndim-1 given, for a stride it never passes on
            stride_rem[0] = stride_loc[0] = size;
            for (int d = 0; d < nd; d++) {
                stride_rem[d + 1] = stride_rem[d];
                stride_rem[d] *= (int)skip[d];
                stride_rem[d + 1] *= (int)o.ldrem[d];
                stride_loc[d + 1] = stride_loc[d];
                if (d < nd - 1) stride_loc[d + 1] *= (int)ld[d];
            }
        } else {
            // gam_ComputePatchIndex (onesided.c:330-337)
            long idx = o.plo[0] - lo[0], factor = 1;
            for (int d = 0; d < nd - 1; d++) { factor *= ld[d]; idx += factor * (o.plo[d + 1] - lo[d + 1]); }
            pbuf = (char *)buf + (long)size * idx;
            // remote address: owner's block base + offset of plo in its column-major block
            long roff = 0, rf = 1;
            for (int d = 0; d < nd; d++) { roff += (o.plo[d] - o.blo[d]) * rf; rf *= o.ldrem[d]; }
            prem = (char *)a.ptr[o.proc] + (long)size * roff;
            for (int d = 0; d < nd; d++) count[d] = (int)(o.phi[d] - o.plo[d] + 1);   // gam_ComputeCount
            count[0] *= size;
            stride_rem[0] = stride_loc[0] = size;                                       // gam_setstride
            for (int d = 0; d < nd - 1; d++) {
                stride_rem[d] *= (int)o.ldrem[d];
                stride_loc[d] *= (int)ld[d];
                stride_rem[d + 1] = stride_rem[d];
                stride_loc[d + 1] = stride_loc[d];
            }
        }
        if (kind == GA_ACC && o.proc == me) {
            long e = 1;
            for (int d = 0; d < nd; d++) e *= (o.phi[d] - o.plo[d]) / (skip ? skip[d] : 1) + 1;
            g_stat.accloc += (double)size * e;
        }
        const bool last = !nb && (skip || k + 1 == owners.size());
        armci_hdl_t h = -1;
        if (kind == GA_ACC) {
            if (last) ARMCI_AccS(a.optype, alpha, pbuf, stride_loc, prem, stride_rem, count, levels, o.proc);
            else ARMCI_NbAccS(a.optype, alpha, pbuf, stride_loc, prem, stride_rem, count, levels, o.proc, &h);
        } else if (kind == GA_PUT) {
            if (last) ARMCI_PutS(pbuf, stride_loc, prem, stride_rem, count, levels, o.proc);
            else ARMCI_NbPutS(pbuf, stride_loc, prem, stride_rem, count, levels, o.proc, &h);
        } else {
            if (last) ARMCI_GetS(prem, stride_rem, pbuf, stride_loc, count, levels, o.proc);
            else ARMCI_NbGetS(prem, stride_rem, pbuf, stride_loc, count, levels, o.proc, &h);
        }
        if (h >= 0) hdl.push_back(h);
    }
    if (nb) {
        nb->insert(nb->end(), hdl.begin(), hdl.end());
        return;
    }
    for (armci_hdl_t &h : hdl) ARMCI_Wait(&h);   // nga_wait_internal
    if (kind == GA_GET) comex_fence_all(COMEX_GROUP_WORLD);   // data is in `buf` on return
}

// ---- gather / scatter / scatter-accumulate --------------------------------
// gai_gatscat (onesided.c:2747-3370, the default build: USE_GATSCAT_NEW is not
// defined): locate the owner of every subscript (pnga_locate), group the
// elements by owner -- owners in ascending rank order, elements in input order
// within an owner -- and issue ONE ARMCI_GetV / PutV / AccV per owner with
// `bytes = elemsize` and the (local, remote) address pairs (gam_Loc_ptr).
// Repeated subscripts of a scatter-accumulate are applied in that order (the
// io-vector path applies the pairs of a repeated destination in input order).
enum GatScat { GS_GATHER, GS_SCATTER, GS_SCATTER_ACC };


// per-call buffers kept across calls: a scatter of millions of elements would
// otherwise page-fault its way through fresh arrays every call
template <class T> static T *grow(std::vector<T> &v, size_t n) {
    if (v.size() < n) v.resize(n);
    return v.data();
}

// Subscripts arrive in C order (capi.c:3026-3160: row-major, 0-based, as an
// array of pointers or one flat array); they are read in place, reversed and
// made 1-based per element rather than copied into a Fortran array first.
// Locating owners and grouping the pairs is a stable counting sort by owner,
// split over host threads for large calls: every thread locates a contiguous
// range of elements and counts per owner, the counts are prefix-summed owner
// by owner in thread order, and every thread locates its range again and writes
// the pairs at its own offsets -- owners ascending, input order within an owner,
// as with one thread.  Locating twice (a few integer operations per element) is
// cheaper than storing each element's owner and offset between the passes: the
// call is bound by host memory traffic, 32 bytes per element this way against 48
// (NGA_Scatter_acc_flat of 4 Mi elements: profiles/r05/scatter2, scatter3).
// host threads that locate owners and group pairs (one per 128 Ki elements, up to 8;
// the former COMEX_AMD_GS_THREADS knob, settled: the box's host share is 16 cores)
static int gs_threads() { return 8; }

struct GsCtx {
    const GArray *a;
    int *const *csubs;
    const int *cflat;
    const long *blo, *ext;   // every owner's block: first index and extents
    char *v;
    int size;
};

static inline void gs_locate(const GsCtx &c, long k, int *pr_out, long *off_out) {
    const GArray &a = *c.a;
    const int nd = a.ndim;
    const int *cs = c.csubs ? c.csubs[k] : c.cflat + k * nd;
    long sub[GA_MAX_DIM];
    int pr = 0, mul = 1;
    for (int d = 0; d < nd; d++) {   // locate(): the owner's block along each dimension
        sub[d] = (long)cs[nd - 1 - d] + 1;
        if (sub[d] < 1 || sub[d] > a.dims[d]) fatal("gather/scatter: invalid subscript of element %ld", k);
        if (a.nblock[d] > 1) {
            const std::vector<long> &m = a.map[d];
            pr += (int)(std::upper_bound(m.begin(), m.end(), sub[d]) - m.begin() - 1) * mul;
        }
        mul *= a.nblock[d];
    }
    long o = 0, f = 1;
    const long *bl = c.blo + (size_t)pr * nd, *ex = c.ext + (size_t)pr * nd;
    for (int d = 0; d < nd; d++) { o += (sub[d] - bl[d]) * f; f *= ex[d]; }
    *pr_out = pr;
    *off_out = o;
}

static void gatscat(GatScat op, int g_a, void *v, int *const *csubs, const int *cflat, long nv, void *alpha) {
    if (nv < 1) return;   // pnga_gather / pnga_scatter: nv < 1 returns
    GArray &a = arr(g_a);
    const int me = my_rank(), np = world_size();
    const int size = a.elemsize, nd = a.ndim;
    static std::vector<void *> s_loc, s_rem;
    std::vector<long> blo((size_t)a.nproc_grid * nd), ext((size_t)a.nproc_grid * nd);
    for (int p = 0; p < a.nproc_grid; ++p) {
        long lo[GA_MAX_DIM], hi[GA_MAX_DIM];
        block_elems(a, p, lo, hi);
        for (int d = 0; d < nd; ++d) {
            blo[(size_t)p * nd + d] = lo[d];
            ext[(size_t)p * nd + d] = hi[d] - lo[d] + 1;
        }
    }
    const GsCtx c{&a, csubs, cflat, blo.data(), ext.data(), (char *)v, size};
    void **loc = grow(s_loc, (size_t)nv), **rem = grow(s_rem, (size_t)nv);
    const int P = np;
    // one thread per 128 Ki elements, at most gs_threads() (COMEX_AMD_GS_THREADS, default 8)
    const int T = (int)std::max(1L, std::min<long>(gs_threads(), nv >> 17));
    std::vector<long> cnt((size_t)T * P, 0);   // cnt[t*P + p]: elements of thread t owned by p
    auto range = [&](int t, long *k0, long *k1) { *k0 = nv * t / T; *k1 = nv * (t + 1) / T; };
    auto locate = [&](int t) {
        long k0, k1;
        range(t, &k0, &k1);
        std::vector<long> ct(P, 0);   // thread-local: neighbours' counters share cache lines
        for (long k = k0; k < k1; k++) {
            int pr;
            long o;
            gs_locate(c, k, &pr, &o);
            ct[pr]++;
        }
        std::copy(ct.begin(), ct.end(), &cnt[(size_t)t * P]);
    };
    std::vector<long> pos((size_t)T * P);      // pos[t*P + p]: next slot of thread t's owner-p pairs
    auto place = [&](int t) {
        long k0, k1;
        range(t, &k0, &k1);
        std::vector<long> pt(&pos[(size_t)t * P], &pos[(size_t)t * P] + P);
        for (long k = k0; k < k1; k++) {
            int pr;
            long o;
            gs_locate(c, k, &pr, &o);
            const long j = pt[pr]++;
            loc[j] = c.v + (long)size * k;
            rem[j] = (char *)a.ptr[pr] + (long)size * o;
        }
    };
    auto run = [&](const std::function<void(int)> &fn) {   // on libga_amd's host worker pool
        if (T == 1) { fn(0); return; }
        if (gaamd_host_parallel(T, [](int t, void *f) { (*(const std::function<void(int)> *)f)(t); },
                                (void *)&fn))
            fatal("gather/scatter: host pool refused %d threads", T);
    };
    if (a.nproc_grid == 1) {
        // one block: every element is its owner's (rank 0 of the grid) -- no counting pass
        // (the placing pass still checks every subscript)
        for (int t = 0; t < T; ++t) {
            long k0, k1;
            range(t, &k0, &k1);
            cnt[(size_t)t * P] = k1 - k0;
        }
    } else {
        run(locate);
    }
    std::vector<long> nelem(P, 0), first(P, 0);
    long acc = 0;
    for (int p = 0; p < P; p++) {
        first[p] = acc;
        for (int t = 0; t < T; t++) {
            pos[(size_t)t * P + p] = acc;
            acc += cnt[(size_t)t * P + p];
        }
        nelem[p] = acc - first[p];
    }
    run(place);
    double &tot = op == GS_GATHER ? g_stat.gattot : g_stat.scatot;
    double &lcl = op == GS_GATHER ? g_stat.gatloc : g_stat.scaloc;
    (op == GS_GATHER ? g_stat.numgat : g_stat.numsca)++;
    tot += (double)size * nv;
    lcl += (double)size * nelem[me];
    for (int p = 0; p < np; p++) {
        if (!nelem[p]) continue;
        armci_giov_t desc;
        desc.bytes = size;
        desc.ptr_array_len = (int)nelem[p];
        int rc;
        if (op == GS_GATHER) {
            desc.src_ptr_array = &rem[first[p]];
            desc.dst_ptr_array = &loc[first[p]];
            rc = ARMCI_GetV(&desc, 1, p);
        } else {
            desc.src_ptr_array = &loc[first[p]];
            desc.dst_ptr_array = &rem[first[p]];
            rc = op == GS_SCATTER ? ARMCI_PutV(&desc, 1, p) : ARMCI_AccV(a.optype, alpha, &desc, 1, p);
        }
        if (rc) fatal("gather/scatter failed in armci (%d)", rc);
    }
    if (op == GS_GATHER) comex_fence_all(COMEX_GROUP_WORLD);   // data is in `v` on return
}

// C (row-major, 0-based) -> Fortran (column-major, 1-based): capi.c:54-61
static void c2f_index(int nd, const int *c, long *f) { for (int i = 0; i < nd; i++) f[nd - i - 1] = (long)c[i] + 1; }
static void c2f(int nd, const int *c, long *f) { for (int i = 0; i < nd; i++) f[nd - i - 1] = c[i]; }

}  // namespace gaamd_ga

using namespace gaamd_ga;

extern "C" {

int GA_Initialize(void) { return ARMCI_Init(); }
static void destroy(int g_a) {
    GArray &a = arr(g_a);
    comex_free(a.ptr[my_rank()], COMEX_GROUP_WORLD);
    a.live = false;
    a.ptr.clear();
}

void GA_Terminate(void) {
    for (size_t i = 0; i < g_arrays.size(); ++i)
        if (g_arrays[i].live) destroy((int)i + 1);
    ARMCI_Finalize();
}
int GA_Nodeid(void) { return my_rank(); }
int GA_Nnodes(void) { return world_size(); }
void GA_Sync(void) { comex_barrier(COMEX_GROUP_WORLD); }
void GA_Error(char *msg, int code) { comex_error(msg, code); }

int NGA_Create(int type, int ndim, int dims[], char *name, int chunk[]) {
    if (ndim < 1 || ndim > GA_MAX_DIM) return 0;
    GArray a;
    a.type = type;
    a.ndim = ndim;
    a.name = name ? name : "";
    a.elemsize = type_size(type, &a.optype);
    long fdims[GA_MAX_DIM], fchunk[GA_MAX_DIM] = {0};
    c2f(ndim, dims, fdims);
    if (chunk) c2f(ndim, chunk, fchunk);
    for (int d = 0; d < ndim; d++) {
        if (fdims[d] < 1) fatal("NGA_Create: dimension %d is %ld", d, fdims[d]);
        a.dims[d] = fdims[d];
    }
    // pnga_allocate (base.c:2550-2630)
    long blk[GA_MAX_DIM], pe[GA_MAX_DIM];
    if (fchunk[0] != 0)
        for (int d = 0; d < ndim; d++) blk[d] = std::min(fchunk[d], fdims[d]);
    else
        for (int d = 0; d < ndim; d++) blk[d] = -1;
    for (int d = 0; d < ndim; d++) if (fdims[d] == 1) blk[d] = 1;
    ddb(ndim, fdims, world_size(), blk, pe);
    for (int d = 0; d < ndim; d++) {
        long pcut;
        if (fchunk[d] > 1) {
            const long ddim = (fdims[d] - 1) / std::min(fchunk[d], fdims[d]) + 1;
            pcut = ddim - (blk[d] - 1) * pe[d];
        } else {
            pcut = fdims[d] - (blk[d] - 1) * pe[d];
        }
        long i = 0, nblock = 0;
        for (long p = 0; p < pe[d] && i < fdims[d]; p++, nblock++) {
            long b = blk[d];
            if (p >= pcut) b = b - 1;
            a.map[d].push_back(i + 1);
            if (fchunk[d] > 1) b *= std::min(fchunk[d], fdims[d]);
            i += b;
        }
        a.nblock[d] = (int)std::min(pe[d], nblock);
        a.map[d].resize(a.nblock[d]);
    }
    return allocate(a);
}

int NGA_Create_irreg(int type, int ndim, int dims[], char *name, int block[], int map[]) {
    if (ndim < 1 || ndim > GA_MAX_DIM) return 0;
    GArray a;
    a.type = type;
    a.ndim = ndim;
    a.name = name ? name : "";
    a.elemsize = type_size(type, &a.optype);
    long fdims[GA_MAX_DIM];
    c2f(ndim, dims, fdims);
    for (int d = 0; d < ndim; d++) a.dims[d] = fdims[d];
    // copy_map (capi.c): C dimension i's block starts follow those of i-1 in `map`
    int off[GA_MAX_DIM];
    for (int i = 0, o = 0; i < ndim; i++) { off[i] = o; o += block[i]; }
    for (int i = 0; i < ndim; i++) {
        const int fd = ndim - 1 - i;
        a.nblock[fd] = block[i];
        for (int k = 0; k < block[i]; k++) a.map[fd].push_back((long)map[off[i] + k] + 1);
    }
    return allocate(a);
}

void GA_Destroy(int g_a) { destroy(g_a); }

void GA_Zero(int g_a) {
    GArray &a = arr(g_a);
    const int me = my_rank();
    long lo[GA_MAX_DIM], hi[GA_MAX_DIM];
    const long n = block_elems(a, me, lo, hi);
    // pnga_zero (global.nalg.c:60-90) is collective and syncs first: no rank may
    // zero its block while another still reads or writes it
    comex_barrier(COMEX_GROUP_WORLD);
    zero_block(a.ptr[me], (size_t)n * a.elemsize);
    comex_barrier(COMEX_GROUP_WORLD);   // fences (syncs every library stream) + barrier
}

void NGA_Distribution(int g_a, int iproc, int lo[], int hi[]) {
    GArray &a = arr(g_a);
    long flo[GA_MAX_DIM], fhi[GA_MAX_DIM];
    block_elems(a, iproc, flo, fhi);
    for (int i = 0; i < a.ndim; i++) {   // COPYINDEX_F2C
        lo[a.ndim - i - 1] = (int)flo[i] - 1;
        hi[a.ndim - i - 1] = (int)fhi[i] - 1;
    }
}

// pnga_locate_num_blocks (base.c:5591-5627): the region is bounds-checked, and the
// count is only defined for block-cyclic distributions; an array with a map
// (NGA_Create's regular blocks or NGA_Create_irreg's) is GA's REGULAR type, for which
// the reference returns -1 -- so does this.
int NGA_Locate_num_blocks(int g_a, int lo[], int hi[]) {
    GArray &a = arr(g_a);
    long flo[GA_MAX_DIM], fhi[GA_MAX_DIM];
    c2f_index(a.ndim, lo, flo);
    c2f_index(a.ndim, hi, fhi);
    for (int d = 0; d < a.ndim; d++)
        if (flo[d] < 1 || fhi[d] > a.dims[d] || flo[d] > fhi[d]) fatal("Requested region out of bounds");
    return -1;
}

static void c_patch(GaOp kind, int g_a, int lo[], int hi[], void *buf, int ld[], void *alpha) {
    GArray &a = arr(g_a);
    long flo[GA_MAX_DIM], fhi[GA_MAX_DIM], fld[GA_MAX_DIM] = {0};
    c2f_index(a.ndim, lo, flo);
    c2f_index(a.ndim, hi, fhi);
    if (a.ndim > 1) c2f(a.ndim - 1, ld, fld);
    patch_op(kind, g_a, flo, fhi, buf, fld, alpha);
}

// ---- strided (skip) and non-blocking variants: capi.c:1990-2060, 2103-2190 ----
static void c_strided(GaOp kind, int g_a, int lo[], int hi[], int skip[], void *buf, int ld[], void *alpha) {
    GArray &a = arr(g_a);
    long flo[GA_MAX_DIM], fhi[GA_MAX_DIM], fld[GA_MAX_DIM] = {0}, fskip[GA_MAX_DIM];
    c2f_index(a.ndim, lo, flo);
    c2f_index(a.ndim, hi, fhi);
    if (a.ndim > 1) c2f(a.ndim - 1, ld, fld);
    c2f(a.ndim, skip, fskip);   // COPYC2F: reversed, no +1
    for (int d = 0; d < a.ndim; d++)
        if (fskip[d] < 1) fatal("nga_strided: invalid skip %ld along coordinate %d", fskip[d], d);
    patch_op(kind, g_a, flo, fhi, buf, fld, alpha, fskip);
}

void NGA_Strided_acc(int g_a, int lo[], int hi[], int skip[], void *buf, int ld[], void *alpha) {
    c_strided(GA_ACC, g_a, lo, hi, skip, buf, ld, alpha);
}
void NGA_Strided_put(int g_a, int lo[], int hi[], int skip[], void *buf, int ld[]) {
    c_strided(GA_PUT, g_a, lo, hi, skip, buf, ld, nullptr);
}
void NGA_Strided_get(int g_a, int lo[], int hi[], int skip[], void *buf, int ld[]) {
    c_strided(GA_GET, g_a, lo, hi, skip, buf, ld, nullptr);
    comex_fence_all(COMEX_GROUP_WORLD);
}

// GA non-blocking handle -> the ARMCI handles of its owners (the reference's
// gai_nbhdl agg lists, onesided.c:120-300); value = slot + 1, 0 = done
struct GaNb { bool used = false; bool get = false; std::vector<armci_hdl_t> h; };
static std::vector<GaNb> g_ga_nb;

static void c_nb(GaOp kind, int g_a, int lo[], int hi[], void *buf, int ld[], void *alpha, ga_nbhdl_t *nbhandle) {
    GArray &a = arr(g_a);
    long flo[GA_MAX_DIM], fhi[GA_MAX_DIM], fld[GA_MAX_DIM] = {0};
    c2f_index(a.ndim, lo, flo);
    c2f_index(a.ndim, hi, fhi);
    if (a.ndim > 1) c2f(a.ndim - 1, ld, fld);
    size_t slot = 0;
    while (slot < g_ga_nb.size() && g_ga_nb[slot].used) ++slot;
    if (slot == g_ga_nb.size()) g_ga_nb.emplace_back();
    GaNb &n = g_ga_nb[slot];
    n.used = true;
    n.get = kind == GA_GET;
    n.h.clear();
    patch_op(kind, g_a, flo, fhi, buf, fld, alpha, nullptr, &n.h);
    *nbhandle = (ga_nbhdl_t)(slot + 1);
}

void NGA_NbAcc(int g_a, int lo[], int hi[], void *buf, int ld[], void *alpha, ga_nbhdl_t *nbhandle) {
    c_nb(GA_ACC, g_a, lo, hi, buf, ld, alpha, nbhandle);
}
void NGA_NbPut(int g_a, int lo[], int hi[], void *buf, int ld[], ga_nbhdl_t *nbhandle) {
    c_nb(GA_PUT, g_a, lo, hi, buf, ld, nullptr, nbhandle);
}
void NGA_NbGet(int g_a, int lo[], int hi[], void *buf, int ld[], ga_nbhdl_t *nbhandle) {
    c_nb(GA_GET, g_a, lo, hi, buf, ld, nullptr, nbhandle);
}
void NGA_NbWait(ga_nbhdl_t *nbhandle) {   // pnga_nbwait -> nga_wait_internal (onesided.c:368)
    if (!nbhandle || *nbhandle <= 0 || (size_t)*nbhandle > g_ga_nb.size()) return;
    GaNb &n = g_ga_nb[(size_t)*nbhandle - 1];
    if (!n.used) return;
    for (armci_hdl_t &h : n.h) ARMCI_Wait(&h);
    if (n.get) comex_fence_all(COMEX_GROUP_WORLD);   // data is in `buf` on return
    n.h.clear();
    n.used = false;
    *nbhandle = 0;
}

void NGA_Acc(int g_a, int lo[], int hi[], void *buf, int ld[], void *alpha) { c_patch(GA_ACC, g_a, lo, hi, buf, ld, alpha); }
void NGA_Put(int g_a, int lo[], int hi[], void *buf, int ld[]) { c_patch(GA_PUT, g_a, lo, hi, buf, ld, nullptr); }
void NGA_Get(int g_a, int lo[], int hi[], void *buf, int ld[]) { c_patch(GA_GET, g_a, lo, hi, buf, ld, nullptr); }

void NGA_Access(int g_a, int lo[], int hi[], void *ptr, int ld[]) {
    GArray &a = arr(g_a);
    const int me = my_rank();
    long blo[GA_MAX_DIM], bhi[GA_MAX_DIM], flo[GA_MAX_DIM], fhi[GA_MAX_DIM];
    block_elems(a, me, blo, bhi);
    c2f_index(a.ndim, lo, flo);
    c2f_index(a.ndim, hi, fhi);
    long off = 0, f = 1;
    for (int d = 0; d < a.ndim; d++) {
        if (flo[d] < blo[d] || fhi[d] > bhi[d]) fatal("NGA_Access: patch not local");
        off += (flo[d] - blo[d]) * f;
        f *= bhi[d] - blo[d] + 1;
    }
    comex_fence_all(COMEX_GROUP_WORLD);   // pending writes land before the caller reads
    *(char **)ptr = (char *)a.ptr[me] + off * a.elemsize;
    for (int i = 0; i < a.ndim - 1; i++) ld[a.ndim - 2 - i] = (int)(bhi[i] - blo[i] + 1);
}

void NGA_Release(int g_a, int lo[], int hi[]) { (void)arr(g_a); (void)lo; (void)hi; }
void NGA_Release_update(int g_a, int lo[], int hi[]) { (void)arr(g_a); (void)lo; (void)hi; }

// capi.c:3026-3160 (NGA_Scatter*, NGA_Gather*): C subscripts, converted per element in gatscat
void NGA_Scatter(int g_a, void *v, int *subsArray[], int n) {
    gatscat(GS_SCATTER, g_a, v, subsArray, nullptr, n, nullptr);
}
void NGA_Scatter_flat(int g_a, void *v, int subsArray[], int n) {
    gatscat(GS_SCATTER, g_a, v, nullptr, subsArray, n, nullptr);
}
void NGA_Scatter_acc(int g_a, void *v, int *subsArray[], int n, void *alpha) {
    gatscat(GS_SCATTER_ACC, g_a, v, subsArray, nullptr, n, alpha);
}
void NGA_Scatter_acc_flat(int g_a, void *v, int subsArray[], int n, void *alpha) {
    gatscat(GS_SCATTER_ACC, g_a, v, nullptr, subsArray, n, alpha);
}
void NGA_Gather(int g_a, void *v, int *subsArray[], int n) {
    gatscat(GS_GATHER, g_a, v, subsArray, nullptr, n, nullptr);
}
void NGA_Gather_flat(int g_a, void *v, int subsArray[], int n) {
    gatscat(GS_GATHER, g_a, v, nullptr, subsArray, n, nullptr);
}

void GA_Get_proc_grid(int g_a, int dims[]) {
    GArray &a = arr(g_a);
    for (int i = 0; i < a.ndim; i++) dims[a.ndim - 1 - i] = a.nblock[i];
}

// The process grid NGA_Create picks for `npes` processes (C order), without
// allocating anything: host-only, used by the CPU tests of the restated ddb.
int gaamd_ga_proc_grid(int ndim, const int *dims, const int *chunk, int npes, int *grid) {
    if (ndim < 1 || ndim > GA_MAX_DIM || npes < 1) return -1;
    long fdims[GA_MAX_DIM], fchunk[GA_MAX_DIM] = {0}, blk[GA_MAX_DIM], pe[GA_MAX_DIM];
    c2f(ndim, dims, fdims);
    if (chunk) c2f(ndim, chunk, fchunk);
    if (fchunk[0] != 0)
        for (int d = 0; d < ndim; d++) blk[d] = std::min(fchunk[d], fdims[d]);
    else
        for (int d = 0; d < ndim; d++) blk[d] = -1;
    for (int d = 0; d < ndim; d++) if (fdims[d] == 1) blk[d] = 1;
    ddb(ndim, fdims, npes, blk, pe);
    for (int i = 0; i < ndim; i++) grid[ndim - 1 - i] = (int)pe[i];
    return 0;
}

void GA_Print_stats(void) {
    printf("[%d] GA statistics: acc calls %ld, put calls %ld, get calls %ld, scatter calls %ld, gather calls %ld\n",
           my_rank(), g_stat.numacc, g_stat.numput, g_stat.numget, g_stat.numsca, g_stat.numgat);
    printf("[%d] accumulate bytes total %.0f, local %.0f (%.1f%%)\n", my_rank(), g_stat.acctot, g_stat.accloc,
           g_stat.acctot > 0 ? 100.0 * g_stat.accloc / g_stat.acctot : 0.0);
}

}  // extern "C"
