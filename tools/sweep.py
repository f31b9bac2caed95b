#!/usr/bin/env python3
"""Interleaved A/B sweep of kernel tuning knobs on one workload, one process
(cdna_hip_programming.md rule 24): each variant runs `--steps` rotating launches
per round, rounds interleaved, median/min per variant reported as GB/s of
algorithmic traffic from one HIP event pair around the launches (per-launch
event pairs would insert a release between kernels and perturb the result)."""
import argparse
import ctypes
import json
import os
# kernel-timing probe: blocking comex_accs calls only stream-ordered (the documented
# COMEX_AMD_BLOCKING_SYNC=0 opt-out), so back-to-back launches are not host round trips
os.environ.setdefault("COMEX_AMD_BLOCKING_SYNC", "0")
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ga_amd  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="H")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--sets", type=int, default=8)
    ap.add_argument("--ld", type=int, default=0, help="override the leading dimension (elements) of a 2-D workload")
    ap.add_argument("--rows", type=int, default=0, help="override the row count of a 2-D workload")
    ap.add_argument("--row-bytes", type=int, default=0,
                    help="2-D f64 shape with rows of this many bytes, ld = 2 x row, 64 MiB of payload")
    ap.add_argument("--ld-bytes", type=int, default=0, help="with --row-bytes: leading dimension in bytes")
    ap.add_argument("--variants", default="default;block=128;block=64;align=0")
    args = ap.parse_args()
    L = ga_amd.lib()
    assert ga_amd.comex_init() == 0
    op, count, sstr, dstr, desc = bench.WORKLOADS[args.workload]
    if args.ld:
        sstr, dstr = [args.ld * 8], [args.ld * 8]
        desc += f" [ld overridden to {args.ld}]"
    if args.rows:
        count = [count[0], args.rows]
        desc += f" [rows overridden to {args.rows}]"
    if args.row_bytes:
        count = [args.row_bytes, (64 << 20) // args.row_bytes]
        ldb = args.ld_bytes or 2 * args.row_bytes
        sstr, dstr = [ldb], [ldb]
        desc = f"2-D f64, {args.row_bytes} B rows x {count[1]}, ld {ldb} B"
    levels = len(count) - 1
    sb, db = bench.span_bytes(count, sstr), bench.span_bytes(count, dstr)
    alg = 3 * bench.patch_bytes(count)
    sets = []
    for i in range(args.sets):
        s, d = ga_amd.DeviceBuffer(sb), ga_amd.DeviceBuffer(db)
        ga_amd.fill(s.ptr, sb // 8, 0, 1 + i)
        ga_amd.fill(d.ptr, db // 8, 0, 100 + i)
        sets.append((s, d))
    ga_amd.sync()
    keep, sp = ga_amd.scale_buffer(op, bench.SCALE[op])
    ss, ds, cnt = ga_amd.int_array(sstr), ga_amd.int_array(dstr), ga_amd.int_array(count)
    stream = L.gaamd_stream()
    variants = [v for v in args.variants.split(";") if v]
    # every knob is reset to its default before each variant (a variant sets only its own keys)
    defaults = {k: ga_amd.get_tuning(k) for k in ("kind", "flat_max_nvec", "block", "align", "flat_line_min",
                                                   "ordered_cols")}
    defaults["streams"] = L.gaamd_num_streams()
    res = {v: [] for v in variants}
    wall = {v: [] for v in variants}
    enq = {v: [] for v in variants}
    ev = [L.gaamd_event_create() for _ in range(2 * args.steps)]
    # round 0 is a discarded warm-up of every variant: the first variant of a
    # cold process otherwise reads 5-10 % low (clock/ramp), biasing the A/B
    for rnd in range(args.rounds + 1):
        for v in variants:
            for k, val in defaults.items():
                ga_amd.set_tuning(k, val)
            if v != "default":
                for kv in v.split(","):
                    k, val = kv.split("=")
                    ga_amd.set_tuning(k, int(val))
            for i in range(3):   # warm
                s, d = sets[i % len(sets)]
                L.comex_accs(op, sp, ctypes.c_void_p(s.ptr), ss, ctypes.c_void_p(d.ptr), ds, cnt, levels, 0, 0)
            import time
            t0 = time.perf_counter()
            L.gaamd_event_record(ev[0], stream)
            L.gaamd_join()   # every library stream starts after ev[0]
            for i in range(args.steps):
                s, d = sets[i % len(sets)]
                L.comex_accs(op, sp, ctypes.c_void_p(s.ptr), ss, ctypes.c_void_p(d.ptr), ds, cnt, levels, 0, 0)
            L.gaamd_join()   # ev[1] after the launches of every library stream
            L.gaamd_event_record(ev[1], stream)
            t_enq = time.perf_counter() - t0
            ga_amd.sync()
            t_all = time.perf_counter() - t0
            ms = L.gaamd_event_elapsed_ms(ev[0], ev[1]) / args.steps
            if rnd == 0:
                continue
            res[v].append(alg / (ms / 1e3) / 1e9)
            wall[v].append(alg * args.steps / t_all / 1e9)
            enq[v].append(t_enq / args.steps * 1e6)
    out = {"workload": args.workload + (f"@ld{args.ld}" if args.ld else "") + (f"@row{args.row_bytes}B" if args.row_bytes else "") + (f"@ld{args.ld_bytes}B" if args.ld_bytes else "") + (f"@rows{args.rows}" if args.rows else ""),
           "desc": desc, "alg_bytes": alg,
           "GBps": {v: {"median": round(float(np.median(x)), 1), "min": round(float(np.min(x)), 1),
                        "max": round(float(np.max(x)), 1), "wall_median": round(float(np.median(wall[v])), 1),
                        "enqueue_us": round(float(np.median(enq[v])), 2)} for v, x in res.items()}}
    print(json.dumps(out))
    ga_amd.comex_finalize()


if __name__ == "__main__":
    main()
