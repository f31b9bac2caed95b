"""Column-reduction rate probe: 2048 rows x 64 KiB into one dst run (the shape of
tests/test_gpu_semantics.py::test_ordered_kernel_large_overlapping_rows), three
rotating source copies, 20 launches between events on the library's primary stream;
prints one JSON line per op with GB/s of physical bytes (src once + the dst run read
and written once).  Tuning evidence, not product code.
    python tools/cols_rate.py [ops...]   (comex op codes 37..42; default 42 and 38)
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import ga_amd  # noqa: E402

L = ga_amd._lib.load()


ESZ = {37: 4, 38: 8, 39: 4, 40: 8, 41: 16, 42: 8}


def rate(op, rows=2048, row_bytes=65536, n=20):
    w = row_bytes // 8
    a = -3 if op in (37, 42) else 0.7071067811865476
    srcs = [ga_amd.DeviceBuffer(rows * w * 8) for _ in range(3)]
    dst = ga_amd.DeviceBuffer(w * 8)
    for b in srcs + [dst]:
        L.gaamd_memset(ctypes.c_void_p(b.ptr), 0, b.nbytes)
    keep, sp = ga_amd.scale_buffer(op, a)
    ss, ds, cnt = ga_amd.int_array([w * 8]), ga_amd.int_array([0]), ga_amd.int_array([w * 8, rows])
    old = ga_amd.set_tuning("streams", 1)
    st = L.gaamd_stream()
    ev0, ev1 = L.gaamd_event_create(), L.gaamd_event_create()
    for i in range(3):
        assert L.comex_accs(op, sp, ctypes.c_void_p(srcs[i].ptr), ss, ctypes.c_void_p(dst.ptr), ds, cnt, 1, 0, 0) == 0
    L.comex_wait_all(0)
    L.gaamd_event_record(ev0, st)
    for i in range(n):
        h = ctypes.c_int(-1)
        assert L.comex_nbaccs(op, sp, ctypes.c_void_p(srcs[i % 3].ptr), ss, ctypes.c_void_p(dst.ptr), ds, cnt, 1, 0,
                              0, ctypes.byref(h)) == 0
    L.gaamd_event_record(ev1, st)
    assert L.comex_wait_all(0) == 0
    ms = L.gaamd_event_elapsed_ms(ev0, ev1) / n
    info = ga_amd.last_launch()
    ga_amd.set_tuning("streams", old)
    for b in srcs + [dst]:
        b.free()
    phys = rows * w * 8 + 2 * w * 8
    return {"op": op, "elem_bytes": ESZ[op], "us": round(ms * 1e3, 1), "GBps_physical": round(phys / (ms * 1e-3) / 1e9),
            "blocks": info["blocks"], "variant": info["unroll"]}


if __name__ == "__main__":
    assert ga_amd.comex_init() == 0
    for op in [int(x) for x in sys.argv[1:]] or [42, 38]:
        print(json.dumps(rate(op)), flush=True)
    ga_amd.comex_finalize()
