#!/usr/bin/env python3
"""Accumulate rate across row lengths at a fixed payload: 2-D f64 patches of
`--payload` bytes whose rows are 8 B ... 64 KiB, leading dimension 2 x row
(+16 B when --odd), rotating buffer sets beyond the MALL, one HIP event pair
around `--steps` launches.  Shows which kernel family (flat / rows) serves each
row length and at what fraction of the HBM roofline."""
import argparse
import ctypes
import json
import os
# kernel-timing probe: blocking comex_accs calls only stream-ordered (the documented
# COMEX_AMD_BLOCKING_SYNC=0 opt-out), so back-to-back launches are not host round trips
os.environ.setdefault("COMEX_AMD_BLOCKING_SYNC", "0")
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ga_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--payload", type=int, default=64 << 20)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rows", default="8,16,32,64,128,256,512,1024,2048,4096,8192,16384,65536")
    ap.add_argument("--odd", action="store_true")
    ap.add_argument("--tune", action="append")
    ap.add_argument("--op", type=int, default=38, help="COMEX_ACC_* op (37 int, 38 dbl, 39 flt, 40 cpl, 41 dcp, 42 lng)")
    args = ap.parse_args()
    L = ga_amd.lib()
    assert ga_amd.comex_init() == 0
    for kv in args.tune or []:
        k, v = kv.split("=")
        ga_amd.set_tuning(k, int(v))
    scale = {37: 3, 38: 0.7071067811865476, 39: 0.70710677, 40: 0.6 - 0.8j, 41: 0.6 - 0.8j, 42: -5}[args.op]
    esz = {37: 4, 38: 8, 39: 4, 40: 8, 41: 16, 42: 8}[args.op]
    tcode = {37: 2, 38: 0, 39: 1, 40: 1, 41: 0, 42: 3}[args.op]
    keep, sp = ga_amd.scale_buffer(args.op, scale)
    stream = L.gaamd_stream()
    ev0, ev1 = L.gaamd_event_create(), L.gaamd_event_create()
    for rb in [int(x) for x in args.rows.split(",")]:
        rows = args.payload // rb
        ld = 2 * rb + (16 if args.odd else 0)
        span = ld * (rows - 1) + rb
        nsets = max(2, min(8, (2 << 30) // (2 * span)))
        sets = [(ga_amd.DeviceBuffer(span), ga_amd.DeviceBuffer(span)) for _ in range(nsets)]
        for s, d in sets:
            n = span // (4 if tcode in (1, 2) else 8)
            ga_amd.fill(s.ptr, n, tcode, 1)
            ga_amd.fill(d.ptr, n, tcode, 2)
        ga_amd.sync()
        st, cnt = ga_amd.int_array([ld]), ga_amd.int_array([rb, rows])
        for i in range(4):
            s, d = sets[i % nsets]
            L.comex_accs(args.op, sp, ctypes.c_void_p(s.ptr), st, ctypes.c_void_p(d.ptr), st, cnt, 1, 0, 0)
        ga_amd.sync()
        info = ga_amd.last_launch()
        L.gaamd_event_record(ev0, stream)
        L.gaamd_join()
        for i in range(args.steps):
            s, d = sets[i % nsets]
            L.comex_accs(args.op, sp, ctypes.c_void_p(s.ptr), st, ctypes.c_void_p(d.ptr), st, cnt, 1, 0, 0)
        L.gaamd_join()
        L.gaamd_event_record(ev1, stream)
        ga_amd.sync()
        ms = L.gaamd_event_elapsed_ms(ev0, ev1) / args.steps
        gbs = 3 * args.payload / (ms / 1e3) / 1e9
        print(json.dumps({"op": args.op, "elem_bytes": esz, "row_bytes": rb, "rows": rows, "ld_bytes": ld, "us_per_launch": round(ms * 1e3, 2),
                          "GBps_alg": round(gbs, 1), "frac_8TBps": round(gbs / 8000, 4), "kernel": info}), flush=True)
        for s, d in sets:
            s.free()
            d.free()
    ga_amd.comex_finalize()


if __name__ == "__main__":
    main()
