/*
 * comex_oracle.c -- CPU restatement of the GA/ComEx strided pack/unpack and
 * typed-accumulate path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * implementation in ga_amd/csrc.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product library never links,
 * calls or falls back to it.
 *
 * Every function restates one piece of the reference (paths relative to
 * /root/reference), keeping its loop order and expression order so results are
 * bit-identical to the reference CPU loops:
 *
 *   ora_acc              comex/src-common/acc.h:106-154 (HAVE_BLAS=0 branch,
 *                        loops 137-143, IADD_SCALE_REG/CPL macros 46-49)
 *   ora_packed_size      comex/src-mpi-pr/comex.c:1237-1264
 *   ora_pack             comex/src-mpi-pr/comex.c:1267-1328
 *   ora_unpack           comex/src-mpi-pr/comex.c:1331-1384
 *   ora_unpack_acc       comex/src-mpi-pr/comex.c:4238-4268 (_acc_packed_handler)
 *   ora_accs             comex/src-mpi-pr/comex.c:6890-6962 (nb_accs, self/SMP
 *                        per-row path) with nb_acc 6218-6260 -> _acc
 *   ora_accs_packed      comex.c:6965-7109 (nb_accs_packed: pack) followed by
 *                        the progress-rank unpack-accumulate 4238-4268
 *   ora_puts / ora_gets  comex.c:6342-6427 / 6617-6696 per-row memcpy odometer
 *   ora_check_contiguous comex/src-armci/armci.c:114-170
 *   ora_legacy_acc_2d    armci/src/xfer/caccumulate.c (c_?_accumulate_2d_:
 *                        97-121, 149-173, 202-217, 256-271, 333-382)
 *   ora_legacy_acc_2D    armci/src/xfer/strided.c:257-328 (armci_acc_2D: byte
 *                        counts and strides to elements by integer division)
 *   ora_splitmix64_*     synthetic input generator of SURVEY.md §8(d)
 *
 * Build flags (oracle/Makefile): -O2 -fwrapv -ffp-contract=off, no -march, so
 * there is no FMA and signed int overflow wraps as the reference's gcc build
 * does in practice.
 *
 * Parity pinning: ora_acc is checked bit-for-bit against the reference's own
 * _acc compiled from comex/src-common/acc.h (oracle/_ref, see Makefile) and
 * against the committed golden fixtures in tests/golden/ generated from it.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <assert.h>

#define ORA_ACC_INT 37
#define ORA_ACC_DBL 38
#define ORA_ACC_FLT 39
#define ORA_ACC_CPL 40
#define ORA_ACC_DCP 41
#define ORA_ACC_LNG 42

typedef struct { double real, imag; } ora_dcpl;
typedef struct { float real, imag; } ora_scpl;

/* acc.h:106-154, HAVE_BLAS == 0.  A += B*C for real types;
 * A.real += (B.real*C.real) - (B.imag*C.imag);
 * A.imag += (B.real*C.imag) + (B.imag*C.real)   for complex (B = src, C = scale).
 * acc.h declares dst/src `restrict` (acc.h:106-110, 121-122): the compiled loop
 * reads B once per element for both statements, so B is read into `b` first --
 * the same bytes as acc.h whenever src and dst do not overlap, and the compiled
 * reference's bytes (oracle/_ref, tests/golden alias cases) where a caller
 * aliases them (a patch accumulated onto itself), which restrict leaves to the
 * compiler. */
int ora_acc(int op, int bytes, void *dst, const void *src, const void *scale)
{
#define ORA_REG(CT)                                                           \
    {                                                                         \
        int m; const int m_lim = bytes / (int)sizeof(CT);                     \
        CT *it = (CT *)dst; const CT *v = (const CT *)src;                    \
        const CT s = *(const CT *)scale;                                      \
        for (m = 0; m < m_lim; ++m) { it[m] += v[m] * s; }                    \
    }
#define ORA_CPL(CT)                                                           \
    {                                                                         \
        int m; const int m_lim = bytes / (int)sizeof(CT);                     \
        CT *it = (CT *)dst; const CT *v = (const CT *)src;                    \
        const CT s = *(const CT *)scale;                                      \
        for (m = 0; m < m_lim; ++m) {                                         \
            const CT b = v[m];                                                \
            it[m].real += (b.real * s.real) - (b.imag * s.imag);              \
            it[m].imag += (b.real * s.imag) + (b.imag * s.real);              \
        }                                                                     \
    }
    switch (op) {
    case ORA_ACC_DBL: ORA_REG(double); break;
    case ORA_ACC_FLT: ORA_REG(float); break;
    case ORA_ACC_INT: ORA_REG(int); break;
    case ORA_ACC_LNG: ORA_REG(long); break;
    case ORA_ACC_DCP: ORA_CPL(ora_dcpl); break;
    case ORA_ACC_CPL: ORA_CPL(ora_scpl); break;
    default: return -1;
    }
#undef ORA_REG
#undef ORA_CPL
    return 0;
}

int ora_elem_size(int op)
{
    switch (op) {
    case ORA_ACC_DBL: return 8;
    case ORA_ACC_FLT: return 4;
    case ORA_ACC_INT: return 4;
    case ORA_ACC_LNG: return 8;
    case ORA_ACC_DCP: return 16;
    case ORA_ACC_CPL: return 8;
    default: return 0;
    }
}

/* comex.c:1237-1264 */
/* io-vector accumulate / copy to a self/SMP target: one _acc (or one memcpy) per
 * (src[i], dst[i]) pair, in pair order -- nb_accv / nb_putv / nb_getv for such
 * targets (comex.c:7327-7400 -> nb_acc 6228-6260, nb_put / nb_get) */
int ora_accv(int op, const void *scale, void *const *src, void *const *dst, long n, int bytes)
{
    long i;
    for (i = 0; i < n; i++)
        if (ora_acc(op, bytes, dst[i], src[i], scale)) return -1;
    return 0;
}

void ora_copyv(void *const *src, void *const *dst, long n, int bytes)
{
    long i;
    for (i = 0; i < n; i++) memcpy(dst[i], src[i], (size_t)bytes);
}

long ora_packed_size(const int *count, int stride_levels)
{
    long n1dim = 1;
    int i;
    for (i = 1; i <= stride_levels; i++) n1dim *= count[i];
    return n1dim * count[0];
}

/* The odometer shared by pack (1293-1327), unpack (1354-1383), the server
 * unpack-acc (4222-4266) and nb_accs/nb_puts/nb_gets: for row i, digit j
 * (1 <= j <= L) is bvalue[j]; the byte offset is sum_j bvalue[j]*stride[j-1].
 * bvalue[j] advances when (i+1) % bunit[j] == 0 and wraps past count[j]-1,
 * with bunit[1] = 1 and bunit[j] = bunit[j-1]*count[j-1].  Restated verbatim
 * (including the int-typed bunit products) so edge behaviour matches. */
typedef struct {
    int levels;
    int bvalue[8];
    int bunit[8];
    const int *count;
    const int *stride;
} ora_odo;

static void odo_init(ora_odo *o, const int *stride, const int *count, int levels)
{
    int i;
    o->levels = levels; o->count = count; o->stride = stride;
    o->bvalue[0] = 0; o->bvalue[1] = 0; o->bunit[0] = 1; o->bunit[1] = 1;
    for (i = 2; i <= levels; i++) {
        o->bvalue[i] = 0;
        o->bunit[i] = o->bunit[i - 1] * count[i - 1];
    }
}

static long odo_next(ora_odo *o, int i)
{
    long idx = 0;
    int j;
    for (j = 1; j <= o->levels; j++) {
        idx += (long)o->bvalue[j] * (long)o->stride[j - 1];
        if ((i + 1) % o->bunit[j] == 0) o->bvalue[j]++;
        if (o->bvalue[j] > (o->count[j] - 1)) o->bvalue[j] = 0;
    }
    return idx;
}

static int n1dim_of(const int *count, int levels)
{
    int n1dim = 1, i;
    for (i = 1; i <= levels; i++) n1dim *= count[i];
    return n1dim;
}

/* comex.c:1267-1328 -- caller provides the packed buffer (the reference
 * mallocs it); returns the packed size. */
long ora_pack(const char *src, const int *src_stride, const int *count,
              int stride_levels, char *packed)
{
    ora_odo o; int i; long packed_index = 0;
    const int n1dim = n1dim_of(count, stride_levels);
    odo_init(&o, src_stride, count, stride_levels);
    for (i = 0; i < n1dim; i++) {
        long src_idx = odo_next(&o, i);
        memcpy(&packed[packed_index], &src[src_idx], count[0]);
        packed_index += count[0];
    }
    return packed_index;
}

/* comex.c:1331-1384 */
long ora_unpack(const char *packed, char *dst, const int *dst_stride,
                const int *count, int stride_levels)
{
    ora_odo o; int i; long packed_index = 0;
    const int n1dim = n1dim_of(count, stride_levels);
    odo_init(&o, dst_stride, count, stride_levels);
    for (i = 0; i < n1dim; i++) {
        long dst_idx = odo_next(&o, i);
        memcpy(&dst[dst_idx], &packed[packed_index], count[0]);
        packed_index += count[0];
    }
    return packed_index;
}

/* comex.c:4238-4268: _acc of each packed row into the strided dst. */
long ora_unpack_acc(int op, const void *scale, const char *packed, char *dst,
                    const int *dst_stride, const int *count, int stride_levels)
{
    ora_odo o; int i; long packed_index = 0;
    const int n1dim = n1dim_of(count, stride_levels);
    odo_init(&o, dst_stride, count, stride_levels);
    for (i = 0; i < n1dim; i++) {
        long dst_idx = odo_next(&o, i);
        ora_acc(op, count[0], &dst[dst_idx], &packed[packed_index], scale);
        packed_index += count[0];
    }
    return packed_index;
}

/* comex.c:6890-6962 (+ nb_acc 6218-6260): stride_levels == 0 is one _acc of
 * count[0] bytes; otherwise one _acc per row in odometer order. */
int ora_accs(int op, const void *scale, const char *src, const int *src_stride,
             char *dst, const int *dst_stride, const int *count, int stride_levels)
{
    ora_odo so, dso; int i;
    if (stride_levels == 0) return ora_acc(op, count[0], dst, src, scale);
    {
        const int n1dim = n1dim_of(count, stride_levels);
        odo_init(&so, src_stride, count, stride_levels);
        odo_init(&dso, dst_stride, count, stride_levels);
        for (i = 0; i < n1dim; i++) {
            long src_idx = odo_next(&so, i);
            long dst_idx = odo_next(&dso, i);
            int rc = ora_acc(op, count[0], dst + dst_idx, src + src_idx, scale);
            if (rc) return rc;
        }
    }
    return 0;
}

/* comex.c:6965-7109 then 4238-4268: the off-node / ACC_SMP=0 route. */
int ora_accs_packed(int op, const void *scale, const char *src, const int *src_stride,
                    char *dst, const int *dst_stride, const int *count, int stride_levels)
{
    long size = ora_packed_size(count, stride_levels);
    char *buf = (char *)malloc(size > 0 ? (size_t)size : 1);
    if (!buf) return -1;
    ora_pack(src, src_stride, count, stride_levels, buf);
    ora_unpack_acc(op, scale, buf, dst, dst_stride, count, stride_levels);
    free(buf);
    return 0;
}

/* comex.c:6342-6427 (nb_puts, per-row nb_put = memcpy for self/SMP) and
 * 6617-6696 (nb_gets): same odometer on both sides, count[0] bytes per row. */
int ora_puts(const char *src, const int *src_stride, char *dst, const int *dst_stride,
             const int *count, int stride_levels)
{
    ora_odo so, dso; int i;
    if (stride_levels == 0) { memcpy(dst, src, count[0]); return 0; }
    {
        const int n1dim = n1dim_of(count, stride_levels);
        odo_init(&so, src_stride, count, stride_levels);
        odo_init(&dso, dst_stride, count, stride_levels);
        for (i = 0; i < n1dim; i++) {
            long src_idx = odo_next(&so, i);
            long dst_idx = odo_next(&dso, i);
            memcpy(dst + dst_idx, src + src_idx, count[0]);
        }
    }
    return 0;
}

int ora_gets(const char *src, const int *src_stride, char *dst, const int *dst_stride,
             const int *count, int stride_levels)
{
    return ora_puts(src, src_stride, dst, dst_stride, count, stride_levels);
}

/* comex/src-armci/armci.c:114-170 (the "#if 1" CMX-merge variant). */
int ora_check_contiguous(const int *src_stride, const int *dst_stride,
                         const int *count, int n_stride)
{
    int i, ret = 1, stridelen = 1, gap = 0;
    int src_ld[8], dst_ld[8];
    if (n_stride > 0) {
        src_ld[0] = src_stride[0];
        dst_ld[0] = dst_stride[0];
    }
    for (i = 1; i < n_stride; i++) {
        src_ld[i] = src_stride[i] / src_stride[i - 1];
        dst_ld[i] = dst_stride[i] / dst_stride[i - 1];
    }
    for (i = 0; i < n_stride; i++) {
        int tmp = stridelen * count[i];
        if (stridelen != 0 && tmp / stridelen != count[i]) { ret = 0; break; }
        stridelen = tmp;
        if ((count[i] < src_ld[i] || count[i] < dst_ld[i]) && gap == 1) {
            ret = 0; break;
        } else if ((count[i] < src_ld[i] || count[i] < dst_ld[i]) && gap == 0) {
            gap = 1;
        } else if (count[i] != 1 && gap == 1) {
            ret = 0; break;
        }
    }
    if (gap == 1 && ret == 1 && n_stride > 0) {
        if (count[n_stride] != 1) ret = 0;
    }
    return ret;
}

/* ---- synthetic inputs ---------------------------------- */
static inline uint64_t splitmix64_at(uint64_t seed, uint64_t i)
{
    /* state after (i+1) increments, so element i is independent of order */
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* f64 in [-1,1): ((x>>11) * 2^-53) * 2 - 1 */
void ora_fill_f64(double *p, long n, uint64_t seed)
{
    long i;
    for (i = 0; i < n; i++)
        p[i] = ((double)(splitmix64_at(seed, (uint64_t)i) >> 11) * 0x1.0p-53) * 2.0 - 1.0;
}

void ora_fill_f32(float *p, long n, uint64_t seed)
{
    long i;
    for (i = 0; i < n; i++)
        p[i] = ((float)(splitmix64_at(seed, (uint64_t)i) >> 40) * 0x1.0p-24f) * 2.0f - 1.0f;
}

/* integers uniform in [-2^20, 2^20) */
void ora_fill_i32(int32_t *p, long n, uint64_t seed)
{
    long i;
    for (i = 0; i < n; i++)
        p[i] = (int32_t)(splitmix64_at(seed, (uint64_t)i) >> 43) - (1 << 20);
}

void ora_fill_i64(int64_t *p, long n, uint64_t seed)
{
    long i;
    for (i = 0; i < n; i++)
        p[i] = (int64_t)(splitmix64_at(seed, (uint64_t)i) >> 43) - (1 << 20);
}

uint64_t ora_splitmix64(uint64_t seed, uint64_t i) { return splitmix64_at(seed, i); }

#include "mt_split.h"

/* P workers on P slabs of the patch (bench.py CPU baseline) */
int ora_accs_mt(int op, const void *scale, const char *src, const int *src_stride,
                char *dst, const int *dst_stride, const int *count, int stride_levels,
                int nthreads)
{
    return mt_accs(ora_accs, ora_elem_size(op), op, scale, src, src_stride, dst, dst_stride, count,
                   stride_levels, nthreads);
}

/* caccumulate.c: column-major A(ald, *) += alpha * B(bld, *), columns outer,
 * rows inner; complex real part alpha.r*B.r - alpha.i*B.i, imaginary part
 * alpha.i*B.r + alpha.r*B.i (183-184).  ld in elements. */
int ora_legacy_acc_2d(int op, const void *alpha, int rows, int cols, void *A, int ald, const void *B, int bld)
{
    int r, c;
#define ORA_LREG(T)                                                           \
    {                                                                         \
        const T a = *(const T *)alpha;                                        \
        T *x = (T *)A; const T *y = (const T *)B;                             \
        for (c = 0; c < cols; ++c)                                            \
            for (r = 0; r < rows; ++r)                                        \
                x[(long)c * ald + r] += a * y[(long)c * bld + r];             \
    }
#define ORA_LCPL(CT)                                                          \
    {                                                                         \
        const CT a = *(const CT *)alpha;                                      \
        CT *x = (CT *)A; const CT *y = (const CT *)B;                         \
        for (c = 0; c < cols; ++c)                                            \
            for (r = 0; r < rows; ++r) {                                      \
                const CT b = y[(long)c * bld + r];                            \
                x[(long)c * ald + r].real += a.real * b.real - a.imag * b.imag; \
                x[(long)c * ald + r].imag += a.imag * b.real + a.real * b.imag; \
            }                                                                 \
    }
    switch (op) {
    case ORA_ACC_DBL: ORA_LREG(double); break;
    case ORA_ACC_FLT: ORA_LREG(float); break;
    case ORA_ACC_INT: ORA_LREG(int); break;
    case ORA_ACC_LNG: ORA_LREG(long); break;
    case ORA_ACC_DCP: ORA_LCPL(ora_dcpl); break;
    case ORA_ACC_CPL: ORA_LCPL(ora_scpl); break;
    default: return -1;
    }
#undef ORA_LREG
#undef ORA_LCPL
    return 0;
}

/* strided.c:257-328: bytes / strides in bytes -> rows / leading dimensions in
 * elements (integer division), then the 2-D loop above */
int ora_legacy_acc_2D(int op, const void *scale, const void *src, void *dst, int bytes, int cols, int src_stride,
                      int dst_stride)
{
    const int esz = ora_elem_size(op);
    if (esz <= 0) return -1;
    return ora_legacy_acc_2d(op, scale, bytes / esz, cols, dst, dst_stride / esz, src, src_stride / esz);
}
