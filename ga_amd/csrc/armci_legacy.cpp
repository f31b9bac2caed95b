// armci_legacy.cpp -- the legacy ARMCI accumulate kernels (include/armci_acc.h).
//
// Reference: armci/src/xfer/caccumulate.c (the c_?_accumulate_{1d,2d,2d_u}_
// loops) and armci_acc_2D (armci/src/xfer/strided.c:257-328), the legacy
// ARMCI's per-slab accumulate.  Each entry point here is one strided
// accumulate of the rows x cols patch on this rank -- the same GPU kernel as
// comex_accs -- with the reference's arithmetic: no FMA (-ffp-contract=off in
// the kernels), complex products in caccumulate.c's order, which equals
// comex acc.h's element for element.
#include "../../include/armci_acc.h"
#include "../../include/comex.h"
#include "runtime.hpp"

namespace {

int my_rank() {
    int me = 0;
    comex_group_rank(COMEX_GROUP_WORLD, &me);
    return me;
}

// A(ald, *) += alpha * B(bld, *) over rows x cols elements of `esz` bytes
void acc2d(int op, const void *alpha, int rows, int cols, void *A, int ald, const void *B, int bld, int esz) {
    if (rows <= 0 || cols <= 0) return;   // the reference's loops run zero times
    if (!gaamd::rt().initialized) gaamd::fatal("legacy ARMCI accumulate before ARMCI_Init");
    int count[2] = {rows * esz, cols};
    int ss[1] = {bld * esz}, ds[1] = {ald * esz};
    const int levels = cols > 1 ? 1 : 0;
    if (comex_accs(op, const_cast<void *>(alpha), const_cast<void *>(B), ss, A, ds, count, levels, my_rank(),
                   COMEX_GROUP_WORLD) != COMEX_SUCCESS)
        gaamd::fatal("legacy ARMCI accumulate failed");
}

constexpr int kInt = COMEX_ACC_INT, kDbl = COMEX_ACC_DBL, kFlt = COMEX_ACC_FLT, kCpl = COMEX_ACC_CPL,
              kDcp = COMEX_ACC_DCP, kLng = COMEX_ACC_LNG;

}  // namespace

extern "C" {

#define GA_LEGACY_1D(NAME, T, OP)                                   \
    void NAME(const T *alpha, T *A, const T *B, const int *rows) {  \
        acc2d(OP, alpha, *rows, 1, A, *rows, B, *rows, sizeof(T)); \
    }
GA_LEGACY_1D(c_d_accumulate_1d_, double, kDbl)
GA_LEGACY_1D(c_f_accumulate_1d_, float, kFlt)
GA_LEGACY_1D(c_c_accumulate_1d_, complex_t, kCpl)
GA_LEGACY_1D(c_z_accumulate_1d_, dcomplex_t, kDcp)
GA_LEGACY_1D(c_i_accumulate_1d_, int, kInt)
GA_LEGACY_1D(c_l_accumulate_1d_, long, kLng)
GA_LEGACY_1D(c_ll_accumulate_1d_, long long, kLng)
#undef GA_LEGACY_1D

#define GA_LEGACY_2D(NAME, T, OP)                                                                       \
    void NAME(const T *alpha, const int *rows, const int *cols, T *A, const int *ald, const T *B,       \
              const int *bld) {                                                                         \
        acc2d(OP, alpha, *rows, *cols, A, *ald, B, *bld, sizeof(T));                                    \
    }
GA_LEGACY_2D(c_d_accumulate_2d_, double, kDbl)
GA_LEGACY_2D(c_f_accumulate_2d_, float, kFlt)
GA_LEGACY_2D(c_c_accumulate_2d_, complex_t, kCpl)
GA_LEGACY_2D(c_z_accumulate_2d_, dcomplex_t, kDcp)
GA_LEGACY_2D(c_i_accumulate_2d_, int, kInt)
GA_LEGACY_2D(c_l_accumulate_2d_, long, kLng)
GA_LEGACY_2D(c_ll_accumulate_2d_, long long, kLng)
// caccumulate.c:385-700: unrolled by four in the reference; the same values
GA_LEGACY_2D(c_d_accumulate_2d_u_, double, kDbl)
GA_LEGACY_2D(c_f_accumulate_2d_u_, float, kFlt)
GA_LEGACY_2D(c_c_accumulate_2d_u_, complex_t, kCpl)
GA_LEGACY_2D(c_z_accumulate_2d_u_, dcomplex_t, kDcp)
GA_LEGACY_2D(c_i_accumulate_2d_u_, int, kInt)
GA_LEGACY_2D(c_l_accumulate_2d_u_, long, kLng)
GA_LEGACY_2D(c_ll_accumulate_2d_u_, long long, kLng)
#undef GA_LEGACY_2D

// strided.c:257-328
void armci_acc_2D(int op, void *scale, int proc, void *src_ptr, void *dst_ptr, int bytes, int cols, int src_stride,
                  int dst_stride, int lockit) {
    (void)lockit;
    if (proc != my_rank())
        gaamd::fatal("armci_acc_2D: proc %d is not this rank (legacy direct access is local only)", proc);
    int esz = 0;
    switch (op) {
    case kInt: esz = (int)sizeof(int); break;
    case kLng: esz = (int)sizeof(long); break;
    case kDbl: esz = (int)sizeof(double); break;
    case kDcp: esz = 2 * (int)sizeof(double); break;
    case kCpl: esz = 2 * (int)sizeof(float); break;
    case kFlt: esz = (int)sizeof(float); break;
    default: gaamd::fatal("ARMCI accumulate: operation not supported %d", op);
    }
    acc2d(op, scale, bytes / esz, cols, dst_ptr, dst_stride / esz, src_ptr, src_stride / esz, esz);
}

}  // extern "C"
