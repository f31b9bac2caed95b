/* ga_coexist.c -- a program that is its own Global Arrays layer, as a real GA
 * build is: it DEFINES GA_Initialize, NGA_Acc, GA_Destroy and GA_Terminate
 * itself (global/src/capi.c:2079-2089 defines NGA_Acc over pnga_acc), calls
 * the ARMCI API beneath them, and links libga_amd.so -- and only libga_amd.so,
 * the drop-in for libarmci (comex/src-armci/capi.c:14-27 exports only
 * ARMCI_* / PARMCI_* / armci_* names).  The link must not meet a second
 * definition of the program's own GA entry points, and the runtime must never
 * call back into them: every one counts its calls, and the counts must equal
 * the calls the program made.
 *
 * Build: gcc -std=c99 -Wall -Werror -ffp-contract=off -Iinclude tests/c/ga_coexist.c
 *          -rdynamic -Lga_amd -lga_amd -Wl,-rpath,<repo>/ga_amd -ldl
 *        (-rdynamic: the program exports its GA names, as libga.so would)
 * Run:   ./ga_coexist link   (no GPU: the program's names are the ones the
 *                             process resolves, libga_amd.so defines none)
 *        ./ga_coexist run    (GPU: GA_Initialize -> ARMCI_Init, NGA_Acc ->
 *                             ARMCI_AccS of a 2-D host patch into an ARMCI_Malloc
 *                             block, exact vs acc.h:46; GA_Terminate -> ARMCI_Finalize)
 * prints "ga_coexist OK" and exits 0. */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "armci.h"

#define ROWS 29
#define COLS 45   /* doubles per row of the patch */
#define LDS 51    /* leading dimension of the caller's buffer (doubles) */
#define LDB 64    /* leading dimension of the "block" (doubles) */

static int n_init, n_acc, n_destroy, n_terminate;
static void *g_block;   /* this program's one "array": a 1-rank block in an ARMCI segment */

/* ---- the program's own GA layer (same prototypes as include/ga.h) ---------- */
int GA_Initialize(void) {
    ++n_init;
    return ARMCI_Init();
}

static int create_block(void) {
    void *ptrs[1] = {NULL};
    if (ARMCI_Malloc(ptrs, (long)ROWS * LDB * (long)sizeof(double)) != 0) return 0;
    g_block = ptrs[0];
    return 1;
}

void NGA_Acc(int g_a, int lo[], int hi[], void *buf, int ld[], void *alpha) {
    (void)g_a;
    ++n_acc;
    /* C order: lo/hi = {row, col}; rows of the block are LDB doubles apart */
    int rows = hi[0] - lo[0] + 1, cols = hi[1] - lo[1] + 1;
    int src_stride[1] = {ld[0] * (int)sizeof(double)};
    int dst_stride[1] = {LDB * (int)sizeof(double)};
    int count[2] = {cols * (int)sizeof(double), rows};
    char *dst = (char *)g_block + ((long)lo[0] * LDB + lo[1]) * (long)sizeof(double);
    if (ARMCI_AccS(ARMCI_ACC_DBL, alpha, buf, src_stride, dst, dst_stride, count, 1, 0) != 0) {
        fprintf(stderr, "ARMCI_AccS failed\n");
        exit(11);
    }
}

void GA_Destroy(int g_a) {
    (void)g_a;
    ++n_destroy;
    if (g_block) ARMCI_Free(g_block);
    g_block = NULL;
}

void GA_Terminate(void) {
    ++n_terminate;
    ARMCI_Finalize();
}

/* the name the process resolves must be this program's */
static int resolves_here(const char *name, void *mine) {
    void *p = dlsym(RTLD_DEFAULT, name);
    if (p != mine) {
        fprintf(stderr, "%s resolves to %p, not the program's %p\n", name, p, mine);
        return 0;
    }
    Dl_info in;
    if (dladdr(p, &in) && in.dli_fname && strstr(in.dli_fname, "libga_amd")) {
        fprintf(stderr, "%s resolves into %s\n", name, in.dli_fname);
        return 0;
    }
    return 1;
}

int main(int argc, char **argv) {
    const int run = argc > 1 && !strcmp(argv[1], "run");
    if (!resolves_here("GA_Initialize", (void *)GA_Initialize) || !resolves_here("NGA_Acc", (void *)NGA_Acc) ||
        !resolves_here("GA_Destroy", (void *)GA_Destroy) || !resolves_here("GA_Terminate", (void *)GA_Terminate))
        return 2;
    /* libga_amd.so itself must neither define nor import a GA name */
    void *core = dlopen("libga_amd.so", RTLD_NOW | RTLD_NOLOAD);
    if (!core) {
        fprintf(stderr, "libga_amd.so is not loaded\n");
        return 3;
    }
    const char *ga_names[] = {"GA_Initialize", "NGA_Acc", "GA_Destroy", "GA_Terminate", "NGA_Create", "GA_Sync", 0};
    for (int i = 0; ga_names[i]; ++i) {
        void *p = dlsym(core, ga_names[i]);   /* searches libga_amd.so and its dependencies */
        Dl_info in;
        if (p && dladdr(p, &in) && in.dli_fname && strstr(in.dli_fname, "libga_amd")) {
            fprintf(stderr, "libga_amd.so defines %s (%s)\n", ga_names[i], in.dli_fname);
            return 4;
        }
    }
    if (!run) {
        printf("ga_coexist OK (link)\n");
        return 0;
    }

    static double src[ROWS * LDS], back[ROWS * LDB], block0[ROWS * LDB];
    for (int i = 0; i < ROWS * LDS; ++i) src[i] = (double)((i * 7919) % 1000) / 7.0 - 60.0;
    for (int i = 0; i < ROWS * LDB; ++i) block0[i] = (double)((i * 104729) % 997) / 3.0;
    double alpha = 0.7071067811865476;
    if (GA_Initialize() != 0) return 5;
    if (!create_block()) return 6;
    ARMCI_Put(block0, g_block, (int)sizeof(block0), 0);
    ARMCI_AllFence();
    int lo[2] = {0, 3}, hi[2] = {ROWS - 1, 3 + COLS - 1}, ld[1] = {LDS};
    NGA_Acc(1, lo, hi, src, ld, &alpha);
    ARMCI_AllFence();
    ARMCI_Get(g_block, back, (int)sizeof(back), 0);
    for (int r = 0; r < ROWS; ++r)
        for (int c = 0; c < LDB; ++c) {
            double want = block0[r * LDB + c];
            if (c >= 3 && c < 3 + COLS) {
                volatile double prod = src[r * LDS + (c - 3)] * alpha;   /* acc.h:46: round(src*a) */
                want = want + prod;                                    /* then round(+dst) */
            }
            if (memcmp(&back[r * LDB + c], &want, sizeof(double)) != 0) {
                fprintf(stderr, "mismatch at (%d,%d): %.17g vs %.17g\n", r, c, back[r * LDB + c], want);
                return 7;
            }
        }
    GA_Destroy(1);
    GA_Terminate();
    /* every call of the program's GA names came from the program itself */
    if (n_init != 1 || n_acc != 1 || n_destroy != 1 || n_terminate != 1) {
        fprintf(stderr, "GA entry points called %d/%d/%d/%d times (want 1/1/1/1): the runtime called back\n",
                n_init, n_acc, n_destroy, n_terminate);
        return 8;
    }
    printf("ga_coexist OK\n");
    return 0;
}
