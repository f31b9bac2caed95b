#!/usr/bin/env python3
"""Small-call latency on one rank: blocking comex_accs / puts / gets of 64 B .. 1 MiB
(device and pinned-host sources), the non-blocking form + wait, GA's NGA_Acc / NGA_Get of
small patches and GA_Sync.  Median of 200 calls after 20 untimed.  Looks for host-side
costs that do not belong to the operation (as the io-vector host sort did).
Diagnostic evidence, not the bench."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ga_amd  # noqa: E402

L = ga_amd.lib()


def med(fn, n=200, w=20):
    for _ in range(w):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(ts[len(ts) // 2] * 1e6, 1)


assert L.GA_Initialize() == 0
ME = L.GA_Nodeid()   # the local calls target this rank
dev = ga_amd.DeviceBuffer(4 << 20)
dst = ga_amd.DeviceBuffer(4 << 20)
pin = ga_amd.DeviceBuffer(4 << 20, host=True)
host = np.zeros(1 << 19)
L.gaamd_memset(ctypes.c_void_p(dev.ptr), 0, 4 << 20)
L.gaamd_memset(ctypes.c_void_p(dst.ptr), 0, 4 << 20)
out = {}
BUSY = ME == 0 or not os.environ.get("LAT_ONLY_RANK0")   # LAT_ONLY_RANK0: the other ranks idle
if os.environ.get("LAT_STAMPS") and BUSY:
    # where one small blocking call's time goes: gaamd_diag("stamps") of the last call
    # ([0] entry, [1] route decided, [2] stream picked, [3] kernel launched, [4] return)
    L.gaamd_diag(b"stamps", 1, None, 0)
    for _ in range(50):
        ga_amd.comex_accs(38, 0.5, dev.ptr, [128], dst.ptr, [128], [64, 1], 1, ME)
    st8 = (ctypes.c_ulonglong * 8)()
    L.gaamd_diag(b"stamps", -1, st8, 8)
    out["stamps_us"] = [round((st8[i] - st8[0]) / 1e3, 1) for i in range(5)]
    L.gaamd_diag(b"stamps", 0, None, 0)
for nb in ((64, 4096, 65536, 1 << 20) if BUSY else ()):
    rows = max(1, nb // 4096)
    row = nb // rows
    cnt = [row, rows]
    st = [row * 2]
    out[f"accs_dev_{nb}"] = med(lambda: ga_amd.comex_accs(38, 0.5, dev.ptr, st, dst.ptr, st, cnt, 1, ME))
    out[f"accs_pinned_{nb}"] = med(lambda: ga_amd.comex_accs(38, 0.5, pin.ptr, st, dst.ptr, st, cnt, 1, ME))
    out[f"accs_pageable_{nb}"] = med(lambda: ga_amd.comex_accs(38, 0.5, host.ctypes.data, st, dst.ptr, st, cnt, 1, ME))

    def nbw():
        rc, h = ga_amd.comex_nbaccs(38, 0.5, dev.ptr, st, dst.ptr, st, cnt, 1, ME)
        ga_amd.comex_wait(h)
    out[f"nbaccs_wait_dev_{nb}"] = med(nbw)
    out[f"puts_pageable_{nb}"] = med(lambda: ga_amd.comex_puts(host.ctypes.data, st, dst.ptr, st, cnt, 1, ME))
    out[f"gets_pageable_{nb}"] = med(lambda: ga_amd.comex_gets(dst.ptr, st, host.ctypes.data, st, cnt, 1, ME))
ia = ga_amd.int_array
g = L.NGA_Create(1004, 2, ia([1024, 1024]), b"lat", None)
buf = np.ones(64 * 64)
one = ctypes.c_double(1.0)
for side in ((4, 16, 64) if BUSY else ()):
    out[f"NGA_Acc_{side}x{side}"] = med(lambda: L.NGA_Acc(g, ia([10, 10]), ia([9 + side, 9 + side]),
                                                          buf.ctypes.data_as(ctypes.c_void_p), ia([side]),
                                                          ctypes.byref(one)))
    out[f"NGA_Get_{side}x{side}"] = med(lambda: L.NGA_Get(g, ia([10, 10]), ia([9 + side, 9 + side]),
                                                          buf.ctypes.data_as(ctypes.c_void_p), ia([side])))
out["GA_Sync"] = med(lambda: L.GA_Sync())
if L.GA_Nnodes() > 1:
    # remote owner: rank 0 accumulates into / gets from a patch at the corner of the last
    # rank's block; the others wait at the sync
    me, last = L.GA_Nodeid(), L.GA_Nnodes() - 1
    blo, bhi = (ctypes.c_int * 2)(), (ctypes.c_int * 2)()
    L.NGA_Distribution(g, last, blo, bhi)            # the last rank's block
    for side in (4, 16, 64):
        lo, hi = ia([blo[0], blo[1]]), ia([blo[0] + side - 1, blo[1] + side - 1])
        if me == 0:
            out[f"remote_NGA_Acc_{side}x{side}"] = med(lambda: L.NGA_Acc(g, lo, hi, buf.ctypes.data_as(ctypes.c_void_p),
                                                                         ia([side]), ctypes.byref(one)))
            out[f"remote_NGA_Get_{side}x{side}"] = med(lambda: L.NGA_Get(g, lo, hi, buf.ctypes.data_as(ctypes.c_void_p),
                                                                         ia([side])))
        L.GA_Sync()
if L.GA_Nodeid() != 0:
    out = {}
for k, v in out.items():
    print(json.dumps({"call": k, "median_us": v}))
L.GA_Destroy(g)
L.GA_Terminate()
