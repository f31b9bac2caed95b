/*
 * comex_init_comm's bootstrap over a sub-communicator (VERDICT r2 item 7;
 * reference comex/src-mpi-pr/comex.c:726-730, comex/src-armci/armci.c:427-440,
 * global/src/base.c:545): MPI_COMM_WORLD is split into even and odd ranks, each
 * rank hands its half to gaamd_set_bootstrap_comm (the half of comex_init_comm
 * that needs no GPU), and the runtime's world must be that half -- its rank and
 * size, and allgathers/barriers that run over it only (gaamd_bootstrap_selftest
 * checks every allgathered word).  Run with MPICH's mpiexec; the library itself
 * links no MPI.
 */
#include <mpi.h>
#include <stdio.h>
#include "ga_amd.h"

int main(int argc, char **argv) {
    MPI_Init(&argc, &argv);
    int wr, ws;
    MPI_Comm_rank(MPI_COMM_WORLD, &wr);
    MPI_Comm_size(MPI_COMM_WORLD, &ws);
    MPI_Comm half;
    MPI_Comm_split(MPI_COMM_WORLD, wr % 2, wr, &half);
    int hr, hs;
    MPI_Comm_rank(half, &hr);
    MPI_Comm_size(half, &hs);
    int rc = gaamd_set_bootstrap_comm(half);
    if (rc) { printf("world %d: set_bootstrap_comm rc %d\n", wr, rc); MPI_Abort(MPI_COMM_WORLD, 1); }
    if (gaamd_rank() != hr || gaamd_size() != hs) {
        printf("world %d: runtime rank/size %d/%d, sub-communicator %d/%d\n", wr, gaamd_rank(), gaamd_size(), hr, hs);
        MPI_Abort(MPI_COMM_WORLD, 2);
    }
    rc = gaamd_bootstrap_selftest(3);
    if (rc) { printf("world %d: bootstrap selftest over the sub-communicator failed\n", wr); MPI_Abort(MPI_COMM_WORLD, 3); }
    printf("world %d -> sub %d/%d OK\n", wr, hr, hs);
    MPI_Finalize();
    return 0;
}
