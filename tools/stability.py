#!/usr/bin/env python3
"""Rate of the headline accumulate over time: `--blocks` blocks of `--per`
launches (rotating buffer sets, as bench.py), one HIP event pair per block,
after a short warm-up.  Shows clock/power ramps and transient slow phases that
a single event pair over the whole run would average away."""
import argparse
import ctypes
import json
import os
# kernel-timing probe: blocking comex_accs calls only stream-ordered (the documented
# COMEX_AMD_BLOCKING_SYNC=0 opt-out), so back-to-back launches are not host round trips
os.environ.setdefault("COMEX_AMD_BLOCKING_SYNC", "0")
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ga_amd  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="H")
    ap.add_argument("--blocks", type=int, default=40)
    ap.add_argument("--per", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--idle", type=float, default=0.0, help="seconds idle before the run")
    args = ap.parse_args()
    L = ga_amd.lib()
    assert ga_amd.comex_init() == 0
    op, count, sstr, dstr, desc = bench.WORKLOADS[args.workload]
    levels = len(count) - 1
    sb, db = bench.span_bytes(count, sstr), bench.span_bytes(count, dstr)
    alg = 3 * bench.patch_bytes(count)
    sets = [(ga_amd.DeviceBuffer(sb), ga_amd.DeviceBuffer(db)) for _ in range(8)]
    for i, (s, d) in enumerate(sets):
        ga_amd.fill(s.ptr, sb // 8, 0, 1 + i)
        ga_amd.fill(d.ptr, db // 8, 0, 100 + i)
    ga_amd.sync()
    keep, sp = ga_amd.scale_buffer(op, bench.SCALE[op])
    ss, ds, cnt = ga_amd.int_array(sstr), ga_amd.int_array(dstr), ga_amd.int_array(count)
    stream = L.gaamd_stream()
    ptrs = [(ctypes.c_void_p(s.ptr), ctypes.c_void_p(d.ptr)) for s, d in sets]
    if args.idle:
        time.sleep(args.idle)
    for i in range(args.warmup):
        L.comex_accs(op, sp, ptrs[i % 8][0], ss, ptrs[i % 8][1], ds, cnt, levels, 0, 0)
    evs = [L.gaamd_event_create() for _ in range(args.blocks + 1)]
    L.gaamd_join()
    L.gaamd_event_record(evs[0], stream)
    k = 0
    for b in range(args.blocks):
        for _ in range(args.per):
            L.comex_accs(op, sp, ptrs[k % 8][0], ss, ptrs[k % 8][1], ds, cnt, levels, 0, 0)
            k += 1
        L.gaamd_join()
        L.gaamd_event_record(evs[b + 1], stream)
    ga_amd.sync()
    rates = []
    for b in range(args.blocks):
        ms = L.gaamd_event_elapsed_ms(evs[b], evs[b + 1])
        rates.append(round(alg * args.per / (ms / 1e3) / 1e9, 1))
    print(json.dumps({"workload": args.workload, "per_block_launches": args.per, "idle_s": args.idle,
                      "GBps_by_block": rates, "min": min(rates), "max": max(rates)}), flush=True)
    ga_amd.comex_finalize()


if __name__ == "__main__":
    main()
