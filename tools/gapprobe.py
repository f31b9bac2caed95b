#!/usr/bin/env python3
"""Where does wall time go between back-to-back strided-acc launches?
Times K rotating launches of one workload four ways in one process:
  events  : comex_accs with a HIP event pair around every launch
  plain   : comex_accs, no events (wall clock only)
  kernel  : gaamd_strided (kernel-level C ABI, no comex bookkeeping), no events
  region  : comex_accs, one event pair around the whole loop
"""
import argparse
import ctypes
import json
import os
# kernel-timing probe: blocking comex_accs calls only stream-ordered (the documented
# COMEX_AMD_BLOCKING_SYNC=0 opt-out), so back-to-back launches are not host round trips
os.environ.setdefault("COMEX_AMD_BLOCKING_SYNC", "0")
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ga_amd  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="H")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--sets", type=int, default=8)
    ap.add_argument("--tune", action="append")
    args = ap.parse_args()
    L = ga_amd.lib()
    assert ga_amd.comex_init() == 0
    for kv in args.tune or []:
        k, v = kv.split("=")
        ga_amd.set_tuning(k, int(v))
    op, count, sstr, dstr, desc = bench.WORKLOADS[args.workload]
    levels = len(count) - 1
    sb, db = bench.span_bytes(count, sstr), bench.span_bytes(count, dstr)
    alg = 3 * bench.patch_bytes(count)
    sets = []
    for i in range(args.sets):
        s, d = ga_amd.DeviceBuffer(sb), ga_amd.DeviceBuffer(db)
        ga_amd.fill(s.ptr, sb // 8, 0, 1 + i)
        ga_amd.fill(d.ptr, db // 8, 0, 100 + i)
        sets.append((ctypes.c_void_p(s.ptr), ctypes.c_void_p(d.ptr), s, d))
    ga_amd.sync()
    keep, sp = ga_amd.scale_buffer(op, bench.SCALE[op])
    ss, ds, cnt = ga_amd.int_array(sstr), ga_amd.int_array(dstr), ga_amd.int_array(count)
    stream = L.gaamd_stream()
    K = args.steps
    ev = [L.gaamd_event_create() for _ in range(2 * K)]
    res = {m: [] for m in ("events", "plain", "kernel", "region", "two_streams", "four_streams")}
    extra = [L.gaamd_stream_create() for _ in range(3)]
    streams4 = [stream] + extra
    for rnd in range(args.rounds):
        for mode in res:
            for i in range(3):
                s = sets[i % len(sets)]
                L.comex_accs(op, sp, s[0], ss, s[1], ds, cnt, levels, 0, 0)
            ga_amd.sync()
            t0 = time.perf_counter()
            if mode == "region":
                L.gaamd_event_record(ev[0], stream)
            for i in range(K):
                s = sets[i % len(sets)]
                if mode == "events":
                    L.gaamd_event_record(ev[2 * i], stream)
                if mode == "kernel":
                    L.gaamd_strided(op, sp, s[0], ss, s[1], ds, cnt, levels, stream)
                elif mode == "two_streams":
                    L.gaamd_strided(op, sp, s[0], ss, s[1], ds, cnt, levels, streams4[i % 2])
                elif mode == "four_streams":
                    L.gaamd_strided(op, sp, s[0], ss, s[1], ds, cnt, levels, streams4[i % 4])
                else:
                    L.comex_accs(op, sp, s[0], ss, s[1], ds, cnt, levels, 0, 0)
                if mode == "events":
                    L.gaamd_event_record(ev[2 * i + 1], stream)
            if mode == "region":
                L.gaamd_event_record(ev[1], stream)
            t_enq = time.perf_counter() - t0
            for x in streams4:
                ga_amd.sync(x)
            ga_amd.sync()
            t = time.perf_counter() - t0
            r = {"wall_GBps": alg * K / t / 1e9, "enqueue_us": t_enq / K * 1e6}
            if mode == "events":
                ms = [L.gaamd_event_elapsed_ms(ev[2 * i], ev[2 * i + 1]) for i in range(K)]
                r["kernel_GBps"] = alg / (np.mean(ms) / 1e3) / 1e9
            if mode == "region":
                r["region_GBps"] = alg * K / (L.gaamd_event_elapsed_ms(ev[0], ev[1]) / 1e3) / 1e9
            res[mode].append(r)
    out = {"workload": args.workload, "launch": ga_amd.last_launch(), "tune": args.tune,
           "modes": {m: {k: round(float(np.median([x[k] for x in v])), 1) for k in v[0]} for m, v in res.items()}}
    print(json.dumps(out))
    ga_amd.comex_finalize()


if __name__ == "__main__":
    main()
