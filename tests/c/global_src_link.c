/*
 * Link check: every ARMCI_* / armci_* function the reference GA layer calls
 * (the .c and .h files of /root/reference/global/src, default build) resolves in
 * libga_amd.so through include/armci.h and include/message.h.  The list was
 * taken from those sources by name; the calls compiled only under MPI
 * (collect.c: ARMCI_COMM_WORLD, armci_group_comm) or ENABLE_CHECKPOINT
 * (ga_ckpt.c, base.c:1191-1294: ARMCI_Ckpt*, ARMCI_Get_ft_group,
 * ARMCI_Get_world_group, armci_irecover, armci_set_spare_procs) are outside the
 * default build and are not provided.  ARMCI_INIT_HANDLE (nbutil.c:146) is a
 * macro of armci.h; ARMCI_PutS_flag__ (ghosts.c:2442) is GA's own function.
 *
 * Nothing is called: the table only takes each function's address, so the
 * program links and runs without a GPU.  Built twice by tests/test_abi.py: as
 * is, and with WITH_MPI (MPICH's <mpi.h> first), where the communicator entry
 * points (ARMCI_Init_mpi_comm, armci_group_comm, comex_init_comm,
 * comex_group_comm) are declared too and must resolve without an MPI library.
 */
#ifdef WITH_MPI
#include <mpi.h>
#endif
#include <stdio.h>
#include "armci.h"
#ifdef WITH_MPI
#include "comex.h"
#endif
#include "message.h"

typedef void (*fn_t)(void);

static const struct { const char *name; fn_t fn; } table[] = {
    {"armci_msg_snd", (fn_t)armci_msg_snd},
    {"armci_msg_rcv", (fn_t)armci_msg_rcv},
    {"ARMCI_PutS", (fn_t)ARMCI_PutS},
    {"ARMCI_PutS_flag", (fn_t)ARMCI_PutS_flag},
    {"ARMCI_GetS", (fn_t)ARMCI_GetS},
    {"ARMCI_PutV", (fn_t)ARMCI_PutV},
    {"ARMCI_GetV", (fn_t)ARMCI_GetV},
    {"armci_write_strided", (fn_t)armci_write_strided},
    {"armci_read_strided", (fn_t)armci_read_strided},
    {"armci_msg_sel_scope", (fn_t)armci_msg_sel_scope},
    {"armci_msg_gop_scope", (fn_t)armci_msg_gop_scope},
    {"ARMCI_Put", (fn_t)ARMCI_Put},
    {"armci_msg_fgop", (fn_t)armci_msg_fgop},
    {"armci_msg_dgop", (fn_t)armci_msg_dgop},
    {"ARMCI_Same_node", (fn_t)ARMCI_Same_node},
    {"ARMCI_NbGetS", (fn_t)ARMCI_NbGetS},
    {"ARMCI_Free", (fn_t)ARMCI_Free},
    {"ARMCI_AccV", (fn_t)ARMCI_AccV},
    {"armci_domain_my_id", (fn_t)armci_domain_my_id},
    {"armci_domain_id", (fn_t)armci_domain_id},
    {"ARMCI_NbPutS", (fn_t)ARMCI_NbPutS},
    {"ARMCI_Uses_shm", (fn_t)ARMCI_Uses_shm},
    {"ARMCI_Free_group", (fn_t)ARMCI_Free_group},
    {"armci_msg_me", (fn_t)armci_msg_me},
    {"armci_msg_lgop", (fn_t)armci_msg_lgop},
    {"armci_msg_igop", (fn_t)armci_msg_igop},
    {"armci_msg_barrier", (fn_t)armci_msg_barrier},
    {"armci_domain_same_id", (fn_t)armci_domain_same_id},
    {"ARMCI_Malloc_local", (fn_t)ARMCI_Malloc_local},
    {"ARMCI_Malloc", (fn_t)ARMCI_Malloc},
    {"ARMCI_Free_local", (fn_t)ARMCI_Free_local},
    {"ARMCI_AllFence", (fn_t)ARMCI_AllFence},
    {"ARMCI_AccS", (fn_t)ARMCI_AccS},
    {"armci_msg_group_gop_scope", (fn_t)armci_msg_group_gop_scope},
    {"armci_msg_group_fgop", (fn_t)armci_msg_group_fgop},
    {"armci_msg_group_dgop", (fn_t)armci_msg_group_dgop},
    {"armci_msg_group_bcast_scope", (fn_t)armci_msg_group_bcast_scope},
    {"armci_msg_group_barrier", (fn_t)armci_msg_group_barrier},
    {"armci_msg_bcast", (fn_t)armci_msg_bcast},
    {"ARMCI_WaitAll", (fn_t)ARMCI_WaitAll},
    {"ARMCI_Wait", (fn_t)ARMCI_Wait},
    {"ARMCI_NbAccS", (fn_t)ARMCI_NbAccS},
    {"ARMCI_Malloc_group", (fn_t)ARMCI_Malloc_group},
    {"ARMCI_Init_args", (fn_t)ARMCI_Init_args},
    {"ARMCI_Group_get_world", (fn_t)ARMCI_Group_get_world},
    {"ARMCI_Group_create", (fn_t)ARMCI_Group_create},
    {"ARMCI_GroupFence", (fn_t)ARMCI_GroupFence},
    {"ARMCI_Free_memdev", (fn_t)ARMCI_Free_memdev},
    {"ARMCI_Fence", (fn_t)ARMCI_Fence},
    {"ARMCI_Absolute_id", (fn_t)ARMCI_Absolute_id},
    {"armci_msg_nproc", (fn_t)armci_msg_nproc},
    {"armci_msg_llgop", (fn_t)armci_msg_llgop},
    {"armci_msg_group_llgop", (fn_t)armci_msg_group_llgop},
    {"armci_msg_group_lgop", (fn_t)armci_msg_group_lgop},
    {"armci_msg_group_igop", (fn_t)armci_msg_group_igop},
    {"armci_msg_bintree", (fn_t)armci_msg_bintree},
    {"armci_exchange_address_grp", (fn_t)armci_exchange_address_grp},
    {"armci_exchange_address", (fn_t)armci_exchange_address},
    {"armci_domain_nprocs", (fn_t)armci_domain_nprocs},
    {"armci_domain_glob_proc_id", (fn_t)armci_domain_glob_proc_id},
    {"armci_domain_count", (fn_t)armci_domain_count},
    {"ARMCI_Uses_shm_grp", (fn_t)ARMCI_Uses_shm_grp},
    {"ARMCI_Unlock", (fn_t)ARMCI_Unlock},
    {"ARMCI_Test", (fn_t)ARMCI_Test},
    {"ARMCI_Set_shm_limit", (fn_t)ARMCI_Set_shm_limit},
    {"ARMCI_Rmw", (fn_t)ARMCI_Rmw},
    {"ARMCI_Malloc_memdev", (fn_t)ARMCI_Malloc_memdev},
    {"ARMCI_Malloc_group_memdev", (fn_t)ARMCI_Malloc_group_memdev},
    {"ARMCI_Lock", (fn_t)ARMCI_Lock},
    {"ARMCI_Initialized", (fn_t)ARMCI_Initialized},
#ifdef WITH_MPI
    {"ARMCI_Init_mpi_comm", (fn_t)ARMCI_Init_mpi_comm},
    {"armci_group_comm", (fn_t)armci_group_comm},
    {"comex_init_comm", (fn_t)comex_init_comm},
    {"comex_group_comm", (fn_t)comex_group_comm},
#endif
    {"ARMCI_Init", (fn_t)ARMCI_Init},
    {"ARMCI_Group_set_default", (fn_t)ARMCI_Group_set_default},
    {"ARMCI_Group_free", (fn_t)ARMCI_Group_free},
    {"ARMCI_Finalize", (fn_t)ARMCI_Finalize},
    {"ARMCI_Error", (fn_t)ARMCI_Error},
    {"ARMCI_Destroy_mutexes", (fn_t)ARMCI_Destroy_mutexes},
    {"ARMCI_Create_mutexes", (fn_t)ARMCI_Create_mutexes},
    {"ARMCI_Cleanup", (fn_t)ARMCI_Cleanup},
};

int main(void) {
    armci_hdl_t h;
    int n = 0;
    ARMCI_INIT_HANDLE(&h);
    (void)h;
    for (size_t i = 0; i < sizeof(table) / sizeof(table[0]); ++i)
        if (table[i].fn) ++n;
    printf("global_src_link OK %d\n", n);
    return n == (int)(sizeof(table) / sizeof(table[0])) ? 0 : 1;
}
