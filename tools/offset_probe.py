#!/usr/bin/env python3
"""Does the relative placement of src and dst in HBM change the accumulate rate?

Each variant shifts the dst base (and optionally the src base) of every
rotating buffer set by a byte offset inside a larger allocation, then times
`--steps` back-to-back comex_accs launches with one HIP event pair (interleaved
rounds, a discarded warm-up round first, as tools/sweep.py).  Hypothesis under
test: when dst - src is a multiple of a large power of two, the src and dst
vectors one wave loads together fall in the same HBM channel/bank, different
DRAM rows (C4, whose dst rows drift by 128 B per row, runs ~5 % faster than
C2/H)."""
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
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--sets", type=int, default=8)
    ap.add_argument("--offsets", default="0:0;0:256;0:4352;0:65792;0:1048832;0:2097152;4096:0;0:131072")
    args = ap.parse_args()
    L = ga_amd.lib()
    assert ga_amd.comex_init() == 0
    op, count, sstr, dstr, desc = bench.WORKLOADS[args.workload]
    levels = len(count) - 1
    sb, db = bench.span_bytes(count, sstr), bench.span_bytes(count, dstr)
    alg = 3 * bench.patch_bytes(count)
    # a variant is "src_off:dst_off" or "src_off:dst_off:knob=val,knob=val" (knobs set for it only)
    variants = [v for v in args.offsets.split(";") if v]

    def parse(v):
        f = v.split(":")
        knobs = dict(kv.split("=") for kv in f[2].split(",")) if len(f) > 2 and f[2] else {}
        return int(f[0]), int(f[1]), {k: int(x) for k, x in knobs.items()}
    pad = max(max(parse(v)[0], parse(v)[1]) for v in variants) + 4096
    sets = []
    for i in range(args.sets):
        s, d = ga_amd.DeviceBuffer(sb + pad), ga_amd.DeviceBuffer(db + pad)
        ga_amd.fill(s.ptr, (sb + pad) // 8, 0, 1 + i)
        ga_amd.fill(d.ptr, (db + pad) // 8, 0, 100 + i)
        sets.append((s, d))
    ga_amd.sync()
    keep, sp = ga_amd.scale_buffer(op, bench.SCALE[op])
    ss, ds, cnt = ga_amd.int_array(sstr), ga_amd.int_array(dstr), ga_amd.int_array(count)
    stream = L.gaamd_stream()
    ev = [L.gaamd_event_create() for _ in range(2)]
    res = {v: [] for v in variants}
    for rnd in range(args.rounds + 1):
        for v in variants:
            so, do, knobs = parse(v)
            old = {k: ga_amd.set_tuning(k, x) for k, x in knobs.items()}
            ptrs = [(ctypes.c_void_p(s.ptr + so), ctypes.c_void_p(d.ptr + do)) for s, d in sets]
            for i in range(3):
                L.comex_accs(op, sp, ptrs[i % len(ptrs)][0], ss, ptrs[i % len(ptrs)][1], ds, cnt, levels, 0, 0)
            L.gaamd_event_record(ev[0], stream)
            L.gaamd_join()   # every library stream starts after ev[0]
            for i in range(args.steps):
                L.comex_accs(op, sp, ptrs[i % len(ptrs)][0], ss, ptrs[i % len(ptrs)][1], ds, cnt, levels, 0, 0)
            L.gaamd_join()   # ev[1] after the launches of every library stream
            L.gaamd_event_record(ev[1], stream)
            ga_amd.sync()
            ms = L.gaamd_event_elapsed_ms(ev[0], ev[1]) / args.steps
            for k, x in old.items():
                ga_amd.set_tuning(k, x)
            if rnd:
                res[v].append(alg / (ms / 1e3) / 1e9)
    addrs = [(hex(s.ptr), hex(d.ptr)) for s, d in sets[:2]]
    out = {"workload": args.workload, "desc": desc, "alg_bytes": alg, "bases": addrs,
           "GBps": {"src+{}:dst+{}{}".format(*v.split(":")[:2], (":" + v.split(":")[2]) if v.count(":") > 1 else ""):
                    {"median": round(float(np.median(x)), 1), "min": round(float(np.min(x)), 1),
                     "max": round(float(np.max(x)), 1)} for v, x in res.items()}}
    print(json.dumps(out), flush=True)
    ga_amd.comex_finalize()


if __name__ == "__main__":
    main()
