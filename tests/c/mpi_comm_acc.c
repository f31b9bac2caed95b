/*
 * ARMCI_Init_mpi_comm over a sub-communicator on the GPU (VERDICT r2 item 7;
 * reference comex/src-armci/armci.c:427-440 -> comex_init_comm, comex.c:726-730;
 * GA_Initialize_comm, global/src/base.c:545).  MPI_COMM_WORLD (3 ranks) is split
 * into {0, 1} and {2}; each part initialises ARMCI over its own communicator, so
 * ARMCI_Malloc is collective over that part only (a world of 3 would wait for
 * the other part forever) and every rank accumulates into the next rank of its
 * part (rank 2: into itself).  Integer-valued f64 data: exact.
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include "armci.h"
#include "message.h"
#include "comex.h"

int main(int argc, char **argv) {
    MPI_Init(&argc, &argv);
    int wr;
    MPI_Comm_rank(MPI_COMM_WORLD, &wr);
    MPI_Comm part;
    MPI_Comm_split(MPI_COMM_WORLD, wr / 2, wr, &part);
    int pr, ps;
    MPI_Comm_rank(part, &pr);
    MPI_Comm_size(part, &ps);
    if (ARMCI_Init_mpi_comm(part) != 1) { printf("world %d: ARMCI_Init_mpi_comm failed\n", wr); MPI_Abort(MPI_COMM_WORLD, 1); }
    if (armci_msg_me() != pr || armci_msg_nproc() != ps) {
        printf("world %d: ARMCI rank/size %d/%d, part %d/%d\n", wr, armci_msg_me(), armci_msg_nproc(), pr, ps);
        MPI_Abort(MPI_COMM_WORLD, 2);
    }
    MPI_Comm wc;
    comex_group_comm(COMEX_GROUP_WORLD, &wc);
    int cmp = 0;
    MPI_Comm_compare(wc, part, &cmp);
    if (cmp != MPI_CONGRUENT) { printf("world %d: comex_group_comm(world) is not the part\n", wr); MPI_Abort(MPI_COMM_WORLD, 3); }
    const int n = 1 << 17;   /* 1 MiB of f64 */
    void **ptr = (void **)malloc(sizeof(void *) * (size_t)ps);
    if (ARMCI_Malloc(ptr, (armci_size_t)n * 8)) MPI_Abort(MPI_COMM_WORLD, 4);
    double *h = (double *)malloc((size_t)n * 8);
    for (int i = 0; i < n; ++i) h[i] = 0.0;
    ARMCI_Put(h, ptr[pr], n * 8, pr);
    ARMCI_Barrier();
    for (int i = 0; i < n; ++i) h[i] = (double)(i % 1000) + 1000.0 * (pr + 1);
    double two = 2.0;
    const int target = (pr + 1) % ps;
    ARMCI_Acc(ARMCI_ACC_DBL, &two, h, ptr[target], n * 8, target);
    ARMCI_Barrier();
    ARMCI_Get(ptr[pr], h, n * 8, pr);
    const int from = (pr + ps - 1) % ps;
    int bad = 0;
    for (int i = 0; i < n; ++i)
        if (h[i] != 2.0 * ((double)(i % 1000) + 1000.0 * (from + 1))) ++bad;
    ARMCI_Free(ptr[pr]);
    ARMCI_Finalize();
    printf("world %d part %d/%d: %s (%d bad)\n", wr, pr, ps, bad ? "WRONG" : "exact", bad);
    MPI_Finalize();
    return bad ? 5 : 0;
}
