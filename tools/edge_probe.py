#!/usr/bin/env python3
"""Where do the edges of a short timed region go?  The driver times 20 headline
steps (~0.66 ms): a fixed cost at the region's edges (first dispatch after an
idle GPU, the timing events, the final synchronisation) is a few % of it.

One process, interleaved rounds of --steps headline steps (workload H, 8
rotating sets) under several region shapes:
  join      ev0 + join ... join + ev1 (round-1 bench.py), comex_wait_all
  perstream one start/end event per library stream, no joins, comex_wait_all
  noevents  no events at all, comex_wait_all
  blocking  comex_accs (blocking: one host round trip per step)
Reports the median wall time per step and event time per step of each shape.
COMEX_AMD_WAIT (spin / yield / blocking) is read once at comex_init: run the
probe once per setting to compare host wait modes.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ga_amd  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="H")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--sets", type=int, default=8)
    ap.add_argument("--shapes", default="join,perstream,noevents,blocking")
    args = ap.parse_args()
    L = ga_amd.lib()
    assert ga_amd.comex_init() == 0
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
    nstreams = L.gaamd_num_streams()
    streams = [L.gaamd_stream_at(i) for i in range(nstreams)]
    ev0 = [L.gaamd_event_create() for _ in streams]
    ev1 = [L.gaamd_event_create() for _ in streams]
    hd = bench.Handles(L)
    k = [0]

    def nb_step():
        s, d = sets[k[0] % len(sets)][:2]
        k[0] += 1
        assert L.comex_nbaccs(op, sp, s, ss, d, ds, cnt, levels, 0, 0, hd.new()) == 0

    def blocking_step():
        s, d = sets[k[0] % len(sets)][:2]
        k[0] += 1
        assert L.comex_accs(op, sp, s, ss, d, ds, cnt, levels, 0, 0) == 0

    t_w = time.perf_counter()
    while time.perf_counter() - t_w < 0.5:
        nb_step()
    hd.drain()

    def region(shape):
        L.comex_barrier(0)
        ga_amd.sync()
        t0 = time.perf_counter()
        if shape == "join":
            L.gaamd_event_record(ev0[0], streams[0])
            L.gaamd_join()
        elif shape == "perstream":
            for e, st in zip(ev0, streams):
                L.gaamd_event_record(e, st)
        t_first = None
        for _ in range(args.steps):
            (blocking_step if shape == "blocking" else nb_step)()
            if t_first is None:
                t_first = time.perf_counter()
        t_enq = time.perf_counter()
        if shape == "join":
            L.gaamd_join()
            L.gaamd_event_record(ev1[0], streams[0])
        elif shape == "perstream":
            for e, st in zip(ev1, streams):
                L.gaamd_event_record(e, st)
        hd.drain()
        t1 = time.perf_counter()
        ev_ms = None
        if shape == "join":
            ev_ms = L.gaamd_event_elapsed_ms(ev0[0], ev1[0])
        elif shape == "perstream":
            ev_ms = max(L.gaamd_event_elapsed_ms(a, b) for a in ev0 for b in ev1)
        res[shape]["first_call_us"].append((t_first - t0) * 1e6)
        res[shape]["enqueue_us"].append((t_enq - t0) * 1e6)
        return (t1 - t0) * 1e3, ev_ms

    shapes = args.shapes.split(",")
    res = {s: {"wall_ms": [], "ev_ms": [], "first_call_us": [], "enqueue_us": []} for s in shapes}
    for _ in range(args.rounds):
        for shp in shapes:
            w, e = region(shp)
            res[shp]["wall_ms"].append(w)
            if e is not None:
                res[shp]["ev_ms"].append(e)
    out = {"workload": args.workload, "steps": args.steps, "rounds": args.rounds, "streams": nstreams,
           "wait": os.environ.get("COMEX_AMD_WAIT", "default"), "shapes": {}}
    for shp, r in res.items():
        w = statistics.median(r["wall_ms"]) / args.steps
        d = {"wall_us_per_step": round(w * 1e3, 2), "wall_frac": round(alg / (w * 1e-3) / 8e12, 4),
             "wall_us_per_step_min": round(min(r["wall_ms"]) / args.steps * 1e3, 2),
             "first_call_us": round(statistics.median(r["first_call_us"]), 2),
             "enqueue_all_us": round(statistics.median(r["enqueue_us"]), 2)}
        if r["ev_ms"]:
            e = statistics.median(r["ev_ms"]) / args.steps
            d.update({"event_us_per_step": round(e * 1e3, 2), "event_frac": round(alg / (e * 1e-3) / 8e12, 4)})
        out["shapes"][shp] = d
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
