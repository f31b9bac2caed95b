#!/usr/bin/env python3
"""Accumulate rate against block size on one box: comex_accs of a contiguous f64 block
(rows of 64 KiB back to back, the launcher's one-run form) from 64 MiB to 8 GiB, in one
process, so box-to-box differences of the 8 GiB case (C5 at N = 1: 0.845 on one box,
0.787 on another with the same kernel and grid) can be told apart from size effects.
Wall clock over `reps` blocking calls after 2 untimed ones; GB/s of 3 x payload.
Diagnostic evidence, not the bench."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ga_amd  # noqa: E402

L = ga_amd.lib()
assert ga_amd.comex_init() == 0
row = 64 << 10
for gib in (1 / 16, 0.5, 1, 2, 4, 8):
    nbytes = int(gib * (1 << 30))
    rows = nbytes // row
    src, dst = ga_amd.DeviceBuffer(nbytes), ga_amd.DeviceBuffer(nbytes)
    L.gaamd_memset(ctypes.c_void_p(src.ptr), 0, nbytes)
    L.gaamd_memset(ctypes.c_void_p(dst.ptr), 0, nbytes)
    ga_amd.sync()
    reps = max(5, int(16 / gib))

    def call():
        assert ga_amd.comex_accs(38, 0.5, src.ptr, [row], dst.ptr, [row], [row, rows], 1, 0) == 0

    for _ in range(2):
        call()
    ga_amd.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        call()
    ga_amd.sync()
    el = (time.perf_counter() - t0) / reps
    print(json.dumps({"block_GiB": gib, "reps": reps, "ms": round(el * 1e3, 3),
                      "GBps": round(3 * nbytes / el / 1e9, 1), "frac_8TBps": round(3 * nbytes / el / 8e12, 4),
                      "kernel": ga_amd.last_launch()}), flush=True)
    src.free()
    dst.free()
ga_amd.comex_finalize()
