"""ctypes binding of libga_amd.so (the C-ABI in include/comex.h, armci.h, message.h,
armci_acc.h, ga_amd.h) and of libga_amd_ga.so (include/ga.h, the GA caller layer
over libga_amd.so's public ABI).

Both are built in-tree (``ga_amd/``) by ``__graft_entry__.build()`` or
``make -C ga_amd/csrc``.  There is no fallback: if a library is missing, loading
raises, so a GPU test can never pass on a substitute path.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libga_amd.so")
GA_LIB_PATH = os.path.join(_HERE, "libga_amd_ga.so")
DIAG_LIB_PATH = os.path.join(_HERE, "libga_amd_diag.so")

c_int_p = ctypes.POINTER(ctypes.c_int)


class DoubleComplex(ctypes.Structure):   # include/ga.h (comex/src-common/acc.h:6-10)
    _fields_ = [("real", ctypes.c_double), ("imag", ctypes.c_double)]


class SingleComplex(ctypes.Structure):   # include/ga.h (acc.h:12-15)
    _fields_ = [("real", ctypes.c_float), ("imag", ctypes.c_float)]


c_void_pp = ctypes.POINTER(ctypes.c_void_p)

# name: (restype, [argtypes]) -- mirrors include/*.h exactly
SIGNATURES = {
    # comex.h
    "comex_init": (ctypes.c_int, []),
    "comex_init_args": (ctypes.c_int, [c_int_p, ctypes.c_void_p]),
    "comex_initialized": (ctypes.c_int, []),
    "comex_finalize": (ctypes.c_int, []),
    "comex_error": (None, [ctypes.c_char_p, ctypes.c_int]),
    "comex_group_create": (ctypes.c_int, [ctypes.c_int, c_int_p, ctypes.c_int, c_int_p]),
    "comex_group_free": (ctypes.c_int, [ctypes.c_int]),
    "comex_group_rank": (ctypes.c_int, [ctypes.c_int, c_int_p]),
    "comex_group_size": (ctypes.c_int, [ctypes.c_int, c_int_p]),
    "comex_group_translate_world": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_int_p]),
    "comex_group_translate_ranks": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_int_p, ctypes.c_int, c_int_p]),
    "comex_rmw": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int]),
    "comex_create_mutexes": (ctypes.c_int, [ctypes.c_int]),
    "comex_destroy_mutexes": (ctypes.c_int, []),
    "comex_lock": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "comex_unlock": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "comex_barrier": (ctypes.c_int, [ctypes.c_int]),
    "comex_put": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "comex_puts": (ctypes.c_int, [ctypes.c_void_p, c_int_p, ctypes.c_void_p, c_int_p, c_int_p,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "comex_putv": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "comex_nbput": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   c_int_p]),
    "comex_nbputs": (ctypes.c_int, [ctypes.c_void_p, c_int_p, ctypes.c_void_p, c_int_p, c_int_p,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, c_int_p]),
    "comex_nbputv": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_int_p]),
    "comex_acc": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int]),
    "comex_accs": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, c_int_p, ctypes.c_void_p,
                                  c_int_p, c_int_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "comex_accv": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int]),
    "comex_nbacc": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, c_int_p]),
    "comex_nbaccs": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, c_int_p, ctypes.c_void_p,
                                    c_int_p, c_int_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_int_p]),
    "comex_nbaccv": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, c_int_p]),
    "comex_get": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "comex_gets": (ctypes.c_int, [ctypes.c_void_p, c_int_p, ctypes.c_void_p, c_int_p, c_int_p,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "comex_getv": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "comex_nbget": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   c_int_p]),
    "comex_nbgets": (ctypes.c_int, [ctypes.c_void_p, c_int_p, ctypes.c_void_p, c_int_p, c_int_p,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, c_int_p]),
    "comex_nbgetv": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_int_p]),
    "comex_malloc": (ctypes.c_int, [c_void_pp, ctypes.c_size_t, ctypes.c_int]),
    "comex_malloc_mem_dev": (ctypes.c_int, [c_void_pp, ctypes.c_size_t, ctypes.c_int, ctypes.c_char_p]),
    "comex_free": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "comex_free_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "comex_malloc_local": (ctypes.c_void_p, [ctypes.c_size_t]),
    "comex_free_local": (ctypes.c_int, [ctypes.c_void_p]),
    "comex_fence_proc": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "comex_fence_all": (ctypes.c_int, [ctypes.c_int]),
    "comex_wait": (ctypes.c_int, [c_int_p]),
    "comex_test": (ctypes.c_int, [c_int_p, c_int_p]),
    "comex_wait_all": (ctypes.c_int, [ctypes.c_int]),
    "comex_wait_proc": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    # armci.h
    "ARMCI_Init": (ctypes.c_int, []),
    "ARMCI_Init_args": (ctypes.c_int, [c_int_p, ctypes.c_void_p]),
    "ARMCI_Initialized": (ctypes.c_int, []),
    "ARMCI_Finalize": (None, []),
    "ARMCI_Barrier": (None, []),
    "ARMCI_Error": (None, [ctypes.c_char_p, ctypes.c_int]),
    "ARMCI_Fence": (None, [ctypes.c_int]),
    "ARMCI_AllFence": (None, []),
    "ARMCI_Put": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "ARMCI_PutS": (ctypes.c_int, [ctypes.c_void_p, c_int_p, ctypes.c_void_p, c_int_p, c_int_p, ctypes.c_int,
                                  ctypes.c_int]),
    "ARMCI_Acc": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.c_int]),
    "ARMCI_AccS": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, c_int_p, ctypes.c_void_p,
                                  c_int_p, c_int_p, ctypes.c_int, ctypes.c_int]),
    "ARMCI_Get": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "ARMCI_GetS": (ctypes.c_int, [ctypes.c_void_p, c_int_p, ctypes.c_void_p, c_int_p, c_int_p, ctypes.c_int,
                                  ctypes.c_int]),
    "ARMCI_PutV": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "ARMCI_GetV": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "ARMCI_AccV": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "ARMCI_NbPut": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, c_int_p]),
    "ARMCI_NbPutS": (ctypes.c_int, [ctypes.c_void_p, c_int_p, ctypes.c_void_p, c_int_p, c_int_p, ctypes.c_int,
                                    ctypes.c_int, c_int_p]),
    "ARMCI_NbAccS": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, c_int_p, ctypes.c_void_p,
                                    c_int_p, c_int_p, ctypes.c_int, ctypes.c_int, c_int_p]),
    "ARMCI_NbGet": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, c_int_p]),
    "ARMCI_NbGetS": (ctypes.c_int, [ctypes.c_void_p, c_int_p, ctypes.c_void_p, c_int_p, c_int_p, ctypes.c_int,
                                    ctypes.c_int, c_int_p]),
    "ARMCI_Wait": (ctypes.c_int, [c_int_p]),
    "ARMCI_Test": (ctypes.c_int, [c_int_p]),
    "ARMCI_WaitAll": (ctypes.c_int, []),
    "ARMCI_WaitProc": (ctypes.c_int, [ctypes.c_int]),
    "ARMCI_Malloc": (ctypes.c_int, [c_void_pp, ctypes.c_long]),
    "ARMCI_Malloc_memdev": (ctypes.c_int, [c_void_pp, ctypes.c_long, ctypes.c_char_p]),
    "ARMCI_Free": (ctypes.c_int, [ctypes.c_void_p]),
    "ARMCI_Free_memdev": (ctypes.c_int, [ctypes.c_void_p]),
    "ARMCI_Malloc_local": (ctypes.c_void_p, [ctypes.c_long]),
    "ARMCI_Free_local": (ctypes.c_int, [ctypes.c_void_p]),
    "armci_check_contiguous": (ctypes.c_int, [c_int_p, c_int_p, c_int_p, ctypes.c_int]),
    "ARMCI_Init_mpi_comm": (ctypes.c_int, [ctypes.c_int]),   # MPI_Comm (MPICH ABI)
    "ARMCI_Cleanup": (None, []),
    "ARMCI_Copy": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "ARMCI_Put_flag": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, c_int_p, ctypes.c_int,
                                      ctypes.c_int]),
    "ARMCI_PutS_flag": (ctypes.c_int, [ctypes.c_void_p, c_int_p, ctypes.c_void_p, c_int_p, c_int_p, ctypes.c_int,
                                       c_int_p, ctypes.c_int, ctypes.c_int]),
    "ARMCI_PutS_flag_dir": (ctypes.c_int, [ctypes.c_void_p, c_int_p, ctypes.c_void_p, c_int_p, c_int_p,
                                           ctypes.c_int, c_int_p, ctypes.c_int, ctypes.c_int]),
    "ARMCI_PutValueInt": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]),
    "ARMCI_PutValueLong": (ctypes.c_int, [ctypes.c_long, ctypes.c_void_p, ctypes.c_int]),
    "ARMCI_PutValueFloat": (ctypes.c_int, [ctypes.c_float, ctypes.c_void_p, ctypes.c_int]),
    "ARMCI_PutValueDouble": (ctypes.c_int, [ctypes.c_double, ctypes.c_void_p, ctypes.c_int]),
    "ARMCI_NbPutValueInt": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, c_int_p]),
    "ARMCI_NbPutValueLong": (ctypes.c_int, [ctypes.c_long, ctypes.c_void_p, ctypes.c_int, c_int_p]),
    "ARMCI_NbPutValueFloat": (ctypes.c_int, [ctypes.c_float, ctypes.c_void_p, ctypes.c_int, c_int_p]),
    "ARMCI_NbPutValueDouble": (ctypes.c_int, [ctypes.c_double, ctypes.c_void_p, ctypes.c_int, c_int_p]),
    "ARMCI_GetValueInt": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "ARMCI_GetValueLong": (ctypes.c_long, [ctypes.c_void_p, ctypes.c_int]),
    "ARMCI_GetValueFloat": (ctypes.c_float, [ctypes.c_void_p, ctypes.c_int]),
    "ARMCI_GetValueDouble": (ctypes.c_double, [ctypes.c_void_p, ctypes.c_int]),
    "ARMCI_NbPutV": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, c_int_p]),
    "ARMCI_NbGetV": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, c_int_p]),
    "ARMCI_NbAccV": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                    c_int_p]),
    "ARMCI_SET_AGGREGATE_HANDLE": (None, [c_int_p]),
    "ARMCI_UNSET_AGGREGATE_HANDLE": (None, [c_int_p]),
    "ARMCI_Rmw": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "ARMCI_Create_mutexes": (ctypes.c_int, [ctypes.c_int]),
    "ARMCI_Destroy_mutexes": (ctypes.c_int, []),
    "ARMCI_Lock": (None, [ctypes.c_int, ctypes.c_int]),
    "ARMCI_Unlock": (None, [ctypes.c_int, ctypes.c_int]),
    "ARMCI_Same_node": (ctypes.c_int, [ctypes.c_int]),
    "ARMCI_Uses_shm": (ctypes.c_int, []),
    "ARMCI_Uses_shm_grp": (ctypes.c_int, [c_int_p]),
    "ARMCI_Set_shm_limit": (None, [ctypes.c_ulong]),
    "armci_notify": (ctypes.c_int, [ctypes.c_int]),
    "armci_notify_wait": (ctypes.c_int, [ctypes.c_int, c_int_p]),
    "parmci_notify": (ctypes.c_int, [ctypes.c_int]),
    "parmci_notify_wait": (ctypes.c_int, [ctypes.c_int, c_int_p]),
    "armci_domain_nprocs": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "armci_domain_id": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "armci_domain_glob_proc_id": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "armci_domain_my_id": (ctypes.c_int, [ctypes.c_int]),
    "armci_domain_count": (ctypes.c_int, [ctypes.c_int]),
    "armci_domain_same_id": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "ARMCI_GroupFence": (None, [c_int_p]),
    "ARMCI_Group_create": (None, [ctypes.c_int, c_int_p, c_int_p]),
    "ARMCI_Group_create_child": (None, [ctypes.c_int, c_int_p, c_int_p, c_int_p]),
    "ARMCI_Group_free": (None, [c_int_p]),
    "ARMCI_Group_rank": (ctypes.c_int, [c_int_p, c_int_p]),
    "ARMCI_Group_size": (None, [c_int_p, c_int_p]),
    "ARMCI_Group_set_default": (None, [c_int_p]),
    "ARMCI_Group_get_default": (None, [c_int_p]),
    "ARMCI_Group_get_world": (None, [c_int_p]),
    "ARMCI_Absolute_id": (ctypes.c_int, [c_int_p, ctypes.c_int]),
    "ARMCI_Malloc_group": (ctypes.c_int, [c_void_pp, ctypes.c_long, c_int_p]),
    "ARMCI_Malloc_group_memdev": (ctypes.c_int, [c_void_pp, ctypes.c_long, c_int_p, ctypes.c_char_p]),
    "ARMCI_Free_group": (ctypes.c_int, [ctypes.c_void_p, c_int_p]),
    "ARMCI_Memget": (None, [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]),
    "ARMCI_Memat": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_long]),
    "ARMCI_Memdt": (None, [ctypes.c_void_p, ctypes.c_long]),
    "ARMCI_Memctl": (None, [ctypes.c_void_p]),
    "armci_write_strided": (None, [ctypes.c_void_p, ctypes.c_int, c_int_p, c_int_p, ctypes.c_void_p]),
    "armci_read_strided": (None, [ctypes.c_void_p, ctypes.c_int, c_int_p, c_int_p, ctypes.c_void_p]),
    # armci_acc.h (legacy ARMCI accumulate loops; pointer arguments as the reference passes them)
    **{f"c_{t}_accumulate_1d_": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_int_p])
       for t in ("d", "f", "c", "z", "i", "l", "ll")},
    **{f"c_{t}_accumulate_2d{u}_": (None, [ctypes.c_void_p, c_int_p, c_int_p, ctypes.c_void_p, c_int_p,
                                           ctypes.c_void_p, c_int_p])
       for t in ("d", "f", "c", "z", "i", "l", "ll") for u in ("", "_u")},
    "armci_acc_2D": (None, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    # message.h
    "armci_msg_snd": (None, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "armci_msg_rcv": (None, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, c_int_p, ctypes.c_int]),
    "armci_msg_rcvany": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, c_int_p]),
    "armci_msg_reduce": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    "armci_msg_reduce_scope": (None, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    "armci_msg_gop_scope": (None, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    "armci_msg_igop": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]),
    "armci_msg_lgop": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]),
    "armci_msg_llgop": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]),
    "armci_msg_fgop": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]),
    "armci_msg_dgop": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]),
    "armci_msg_bcast": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "armci_msg_brdcst": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "armci_msg_bcast_scope": (None, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "armci_msg_sel_scope": (None, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                   ctypes.c_int]),
    "armci_exchange_address": (None, [c_void_pp, ctypes.c_int]),
    "armci_exchange_address_grp": (None, [c_void_pp, ctypes.c_int, c_int_p]),
    "armci_msg_barrier": (None, []),
    "parmci_msg_barrier": (None, []),
    "armci_msg_group_barrier": (None, [c_int_p]),
    "parmci_msg_group_barrier": (None, [c_int_p]),
    "armci_msg_bintree": (None, [ctypes.c_int, c_int_p, c_int_p, c_int_p, c_int_p]),
    "armci_msg_me": (ctypes.c_int, []),
    "armci_msg_nproc": (ctypes.c_int, []),
    "armci_msg_abort": (None, [ctypes.c_int]),
    "armci_msg_init": (None, [c_int_p, ctypes.c_void_p]),
    "armci_msg_finalize": (None, []),
    "armci_timer": (ctypes.c_double, []),
    "armci_msg_clus_brdcst": (None, [ctypes.c_void_p, ctypes.c_int]),
    "armci_msg_clus_igop": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]),
    "armci_msg_clus_fgop": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]),
    "armci_msg_clus_lgop": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]),
    "armci_msg_clus_llgop": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]),
    "armci_msg_clus_dgop": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]),
    "armci_msg_group_gop_scope": (None, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                         c_int_p]),
    "armci_msg_group_igop": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, c_int_p]),
    "armci_msg_group_lgop": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, c_int_p]),
    "armci_msg_group_llgop": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, c_int_p]),
    "armci_msg_group_fgop": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, c_int_p]),
    "armci_msg_group_dgop": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, c_int_p]),
    "armci_msg_group_bcast_scope": (None, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, c_int_p]),
    "armci_grp_clus_brdcst": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_int_p]),
    # ga_amd.h
    "gaamd_set_bootstrap": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p]),
    "gaamd_bootstrap_selftest": (ctypes.c_int, [ctypes.c_int]),
    "gaamd_rank": (ctypes.c_int, []),
    "gaamd_size": (ctypes.c_int, []),
    "gaamd_device": (ctypes.c_int, []),
    "gaamd_device_topology": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)] * 3),
    "gaamd_node_info": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)] * 3),
    "gaamd_wire_selftest": (ctypes.c_int, [ctypes.c_int]),
    "gaamd_strided": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, c_int_p, ctypes.c_void_p,
                                     c_int_p, c_int_p, ctypes.c_int, ctypes.c_void_p]),
    "gaamd_packed_size": (ctypes.c_long, [c_int_p, ctypes.c_int]),
    "gaamd_pack": (ctypes.c_int, [ctypes.c_void_p, c_int_p, c_int_p, ctypes.c_int, ctypes.c_void_p,
                                  ctypes.c_void_p]),
    "gaamd_unpack": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, c_int_p, c_int_p, ctypes.c_int,
                                    ctypes.c_void_p]),
    "gaamd_unpack_acc": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_int_p,
                                        c_int_p, ctypes.c_int, ctypes.c_void_p]),
    "gaamd_last_launch": (ctypes.c_int, [c_int_p, c_int_p, c_int_p, c_int_p,
                                         ctypes.POINTER(ctypes.c_ulonglong)]),
    "gaamd_kernel_counts": (ctypes.c_int, [ctypes.POINTER(ctypes.c_ulonglong)]),
    "gaamd_route_counts": (ctypes.c_int, [ctypes.POINTER(ctypes.c_ulonglong)]),
    "gaamd_toggle_counts": (ctypes.c_int, [ctypes.POINTER(ctypes.c_ulonglong)]),
    "gaamd_iov_path_counts": (ctypes.c_int, [ctypes.POINTER(ctypes.c_ulonglong)]),
    "gaamd_host_parallel": (ctypes.c_int, [ctypes.c_int, ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.c_void_p),
                                           ctypes.c_void_p]),
    "gaamd_one_pass_count": (ctypes.c_ulonglong, []),
    "gaamd_segment_cache_reuse": (ctypes.c_ulonglong, []),
    "gaamd_segment_remaps": (ctypes.c_ulonglong, []),
    "gaamd_segment_cache_trims": (ctypes.c_ulonglong, []),
    "gaamd_segment_kind": (ctypes.c_int, [ctypes.c_void_p]),
    "gaamd_vmm_access_retries": (ctypes.c_ulonglong, []),
    "gaamd_vmm_exchange_selftest": (ctypes.c_int, [ctypes.c_int]),
    "gaamd_owner_counts": (ctypes.c_int, [ctypes.POINTER(ctypes.c_ulonglong)]),
    "gaamd_peers_unmapped": (ctypes.c_int, []),
    "gaamd_plan_strided": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, c_int_p, ctypes.c_void_p, c_int_p, c_int_p,
                                          ctypes.c_int, ctypes.c_ulonglong, ctypes.c_ulonglong,
                                          ctypes.POINTER(ctypes.c_longlong)]),
    "gaamd_set_tuning": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int]),
    "gaamd_get_tuning": (ctypes.c_int, [ctypes.c_char_p]),
    "gaamd_device_count": (ctypes.c_int, []),
    "gaamd_set_device": (ctypes.c_int, [ctypes.c_int]),
    "gaamd_stream": (ctypes.c_void_p, []),
    "gaamd_stream_at": (ctypes.c_void_p, [ctypes.c_int]),
    "gaamd_dev_malloc": (ctypes.c_void_p, [ctypes.c_size_t]),
    "gaamd_dev_free": (ctypes.c_int, [ctypes.c_void_p]),
    "gaamd_host_malloc": (ctypes.c_void_p, [ctypes.c_size_t]),
    "gaamd_host_free": (ctypes.c_int, [ctypes.c_void_p]),
    "gaamd_memcpy": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    "gaamd_memcpy2d": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.c_size_t, ctypes.c_size_t]),
    "gaamd_memset": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]),
    "gaamd_sync": (ctypes.c_int, [ctypes.c_void_p]),
    "gaamd_join": (ctypes.c_int, []),
    "gaamd_num_streams": (ctypes.c_int, []),
    "gaamd_fill_word": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_long, ctypes.c_ulonglong, ctypes.c_void_p]),
    "gaamd_fill": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_ulonglong,
                                  ctypes.c_void_p]),
    "gaamd_stream_create": (ctypes.c_void_p, []),
    "gaamd_stream_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "gaamd_event_create": (ctypes.c_void_p, []),
    "gaamd_event_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "gaamd_event_record": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "gaamd_event_sync": (ctypes.c_int, [ctypes.c_void_p]),
    "gaamd_event_elapsed_ms": (ctypes.c_float, [ctypes.c_void_p, ctypes.c_void_p]),
    "gaamd_version": (ctypes.c_char_p, []),
    "gaamd_hip_runtime": (ctypes.c_char_p, []),
    "gaamd_build_id": (ctypes.c_char_p, []),
    "gaamd_diag": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_longlong, ctypes.POINTER(ctypes.c_ulonglong),
                                  ctypes.c_int]),
}

# ga.h: libga_amd_ga.so
GA_SIGNATURES = {
    "gaamd_ga_proc_grid": (ctypes.c_int, [ctypes.c_int, c_int_p, c_int_p, ctypes.c_int, c_int_p]),
    "GA_Initialize": (ctypes.c_int, []),
    "GA_Terminate": (None, []),
    "GA_Nodeid": (ctypes.c_int, []),
    "GA_Nnodes": (ctypes.c_int, []),
    "GA_Sync": (None, []),
    "GA_Error": (None, [ctypes.c_char_p, ctypes.c_int]),
    "NGA_Create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_int_p, ctypes.c_char_p, c_int_p]),
    "NGA_Create_irreg": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_int_p, ctypes.c_char_p, c_int_p, c_int_p]),
    "GA_Destroy": (None, [ctypes.c_int]),
    "GA_Zero": (None, [ctypes.c_int]),
    "NGA_Distribution": (None, [ctypes.c_int, ctypes.c_int, c_int_p, c_int_p]),
    "NGA_Locate_num_blocks": (ctypes.c_int, [ctypes.c_int, c_int_p, c_int_p]),
    "NGA_Acc": (None, [ctypes.c_int, c_int_p, c_int_p, ctypes.c_void_p, c_int_p, ctypes.c_void_p]),
    "NGA_Put": (None, [ctypes.c_int, c_int_p, c_int_p, ctypes.c_void_p, c_int_p]),
    "NGA_Get": (None, [ctypes.c_int, c_int_p, c_int_p, ctypes.c_void_p, c_int_p]),
    "NGA_Access": (None, [ctypes.c_int, c_int_p, c_int_p, ctypes.c_void_p, c_int_p]),
    "NGA_NbAcc": (None, [ctypes.c_int, c_int_p, c_int_p, ctypes.c_void_p, c_int_p, ctypes.c_void_p,
                         ctypes.POINTER(ctypes.c_long)]),
    "NGA_NbPut": (None, [ctypes.c_int, c_int_p, c_int_p, ctypes.c_void_p, c_int_p, ctypes.POINTER(ctypes.c_long)]),
    "NGA_NbGet": (None, [ctypes.c_int, c_int_p, c_int_p, ctypes.c_void_p, c_int_p, ctypes.POINTER(ctypes.c_long)]),
    "NGA_NbWait": (None, [ctypes.POINTER(ctypes.c_long)]),
    "NGA_Strided_acc": (None, [ctypes.c_int, c_int_p, c_int_p, c_int_p, ctypes.c_void_p, c_int_p, ctypes.c_void_p]),
    "NGA_Strided_put": (None, [ctypes.c_int, c_int_p, c_int_p, c_int_p, ctypes.c_void_p, c_int_p]),
    "NGA_Strided_get": (None, [ctypes.c_int, c_int_p, c_int_p, c_int_p, ctypes.c_void_p, c_int_p]),
    "NGA_Scatter": (None, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "NGA_Scatter_flat": (None, [ctypes.c_int, ctypes.c_void_p, c_int_p, ctypes.c_int]),
    "NGA_Scatter_acc": (None, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "NGA_Scatter_acc_flat": (None, [ctypes.c_int, ctypes.c_void_p, c_int_p, ctypes.c_int, ctypes.c_void_p]),
    "NGA_Gather": (None, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "NGA_Gather_flat": (None, [ctypes.c_int, ctypes.c_void_p, c_int_p, ctypes.c_int]),
    "NGA_Release": (None, [ctypes.c_int, c_int_p, c_int_p]),
    "NGA_Release_update": (None, [ctypes.c_int, c_int_p, c_int_p]),
    "GA_Get_proc_grid": (None, [ctypes.c_int, c_int_p]),
    "GA_Print_stats": (None, []),
}
SIGNATURES.update(GA_SIGNATURES)

# ga_amd_diag.h: libga_amd_diag.so (measurement helpers, not the boundary)
DIAG_SIGNATURES = {
    "gaamd_time_blocking_accs": (ctypes.c_ulonglong, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, c_int_p,
                                                      ctypes.c_void_p, c_int_p, c_int_p, ctypes.c_int, ctypes.c_int,
                                                      ctypes.c_int, ctypes.c_int]),
}
SIGNATURES.update(DIAG_SIGNATURES)

ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)
BARRIER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)

_lib = None


class Libs:
    """The three libraries under one name space: a ga.h function resolves in
    libga_amd_ga.so, a ga_amd_diag.h one in libga_amd_diag.so, everything else in
    libga_amd.so."""

    def __init__(self, core, ga, diag):
        self.core, self.ga, self.diag = core, ga, diag

    def _of(self, name):
        return self.ga if name in GA_SIGNATURES else self.diag if name in DIAG_SIGNATURES else self.core

    def __getattr__(self, name):
        fn = getattr(self._of(name), name)
        setattr(self, name, fn)
        return fn


def load():
    """Load (once) libga_amd.so, libga_amd_ga.so and libga_amd_diag.so; raise if one is absent."""
    global _lib
    if _lib is not None:
        return _lib
    for path in (LIB_PATH, GA_LIB_PATH, DIAG_LIB_PATH):
        if not os.path.exists(path):
            raise ImportError(
                f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "or `make -C ga_amd/csrc` (there is no CPU fallback)")
    libs = Libs(*(ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL) for p in (LIB_PATH, GA_LIB_PATH, DIAG_LIB_PATH)))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(libs._of(name), name)
        fn.restype = res
        fn.argtypes = args
    _lib = libs
    return libs
