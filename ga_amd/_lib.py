"""ctypes binding of libga_amd.so (the C-ABI in include/comex.h, armci.h, ga_amd.h).

The library is built in-tree (``ga_amd/libga_amd.so``) by ``__graft_entry__.build()``
or ``make -C ga_amd/csrc``.  There is no fallback: if the library is missing,
importing this module raises, so a GPU test can never pass on a substitute path.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libga_amd.so")

c_int_p = ctypes.POINTER(ctypes.c_int)
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
    # ga_amd.h
    "gaamd_set_bootstrap": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p]),
    "gaamd_bootstrap_selftest": (ctypes.c_int, [ctypes.c_int]),
    "gaamd_rank": (ctypes.c_int, []),
    "gaamd_size": (ctypes.c_int, []),
    "gaamd_device": (ctypes.c_int, []),
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
    "gaamd_memset": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]),
    "gaamd_sync": (ctypes.c_int, [ctypes.c_void_p]),
    "gaamd_join": (ctypes.c_int, []),
    "gaamd_num_streams": (ctypes.c_int, []),
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
    "gaamd_ga_proc_grid": (ctypes.c_int, [ctypes.c_int, c_int_p, c_int_p, ctypes.c_int, c_int_p]),
    # ga.h
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

ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)
BARRIER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)

_lib = None


def load():
    """Load (once) and return the ctypes handle of libga_amd.so; raise if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C ga_amd/csrc` (there is no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib
