/* abi_client.c -- a plain C (C99) caller of the drop-in boundary, as GA's
 * global/src would be: includes include/comex.h, armci.h and ga.h, links
 * libga_amd_ga.so (ga.h) over libga_amd.so, and on a GPU box runs one strided accumulate through each of
 * comex_accs and ARMCI_AccS on a host patch, checked against the reference's
 * loop expression (acc.h:46 IADD_SCALE_REG: dst += src*scale, no FMA), plus an
 * NGA_Acc / NGA_Get round trip on a 1-rank GA.
 * Build (tests/test_abi.py does this): gcc -std=c99 -Wall -Werror -ffp-contract=off
 *   -Iinclude tests/c/abi_client.c -Lga_amd -lga_amd_ga -lga_amd -Wl,-rpath,<repo>/ga_amd
 * Run: ./abi_client  -> prints "abi_client OK" and exits 0. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "comex.h"
#include "armci.h"
#include "ga.h"

#define ROWS 37
#define COLS 53   /* doubles per row of the patch */
#define LDS 61    /* leading dimensions (doubles) */
#define LDD 67

static int check(const double *got, const double *src, const double *dst0, double alpha) {
    for (int r = 0; r < ROWS; ++r)
        for (int c = 0; c < COLS; ++c) {
            volatile double prod = src[r * LDS + c] * alpha;   /* round(src*alpha) */
            const double want = dst0[r * LDD + c] + prod;      /* then round(+dst) */
            if (memcmp(&got[r * LDD + c], &want, sizeof(double)) != 0) {
                fprintf(stderr, "mismatch at (%d,%d): %.17g vs %.17g\n", r, c, got[r * LDD + c], want);
                return 1;
            }
        }
    return 0;
}

int main(void) {
    static double src[ROWS * LDS], dst[ROWS * LDD], dst0[ROWS * LDD];
    for (int i = 0; i < ROWS * LDS; ++i) src[i] = (double)((i * 7919) % 1000) / 7.0 - 60.0;
    for (int i = 0; i < ROWS * LDD; ++i) dst0[i] = dst[i] = (double)((i * 104729) % 997) / 3.0;
    int stride[1] = {LDS * (int)sizeof(double)}, dstride[1] = {LDD * (int)sizeof(double)};
    int count[2] = {COLS * (int)sizeof(double), ROWS};
    double alpha = 0.7071067811865476;

    if (GA_Initialize() != 0) return 2;   /* -> ARMCI_Init -> comex_init */
    if (comex_accs(COMEX_ACC_DBL, &alpha, src, stride, dst, dstride, count, 1, 0, COMEX_GROUP_WORLD) != COMEX_SUCCESS)
        return 3;
    comex_fence_all(COMEX_GROUP_WORLD);
    if (check(dst, src, dst0, alpha)) return 4;

    memcpy(dst, dst0, sizeof(dst));
    if (ARMCI_AccS(ARMCI_ACC_DBL, &alpha, src, stride, dst, dstride, count, 1, 0) != 0) return 5;
    ARMCI_AllFence();
    if (check(dst, src, dst0, alpha)) return 6;

    /* GA: 1-rank array, accumulate a patch from host memory and read it back */
    int dims[2] = {ROWS + 5, COLS + 9};
    int g = NGA_Create(C_DBL, 2, dims, "abi", NULL);
    if (g <= 0) return 8;
    GA_Zero(g);
    int lo[2] = {2, 3}, hi[2] = {2 + ROWS - 1, 3 + COLS - 1}, ld[1] = {LDS};
    NGA_Acc(g, lo, hi, src, ld, &alpha);
    GA_Sync();
    static double back[ROWS * LDS];
    int ldb[1] = {LDS};
    NGA_Get(g, lo, hi, back, ldb);
    for (int r = 0; r < ROWS; ++r)
        for (int c = 0; c < COLS; ++c) {
            volatile double prod = src[r * LDS + c] * alpha;
            const double want = 0.0 + prod;
            if (memcmp(&back[r * LDS + c], &want, sizeof(double)) != 0) {
                fprintf(stderr, "GA mismatch at (%d,%d)\n", r, c);
                return 9;
            }
        }
    GA_Destroy(g);
    GA_Terminate();   /* -> ARMCI_Finalize -> comex_finalize */
    printf("abi_client OK\n");
    return 0;
}
