#!/usr/bin/env python3
"""Place the bench's value region on the kernel trace.

bench.py records the region's two ends on CLOCK_BOOTTIME (value_region.boottime_ns),
the clock rocprofv3 stamps kernels with.  This prints, for the K kernels inside the
region: the gap from the region's start to the first kernel's start, the GPU span
of the K kernels and their merged busy time (two streams overlap), the idle gaps
between consecutive kernels, and the gap from the last kernel's end to the region's
end.  usage: region_edges.py run_results.db bench.json"""
import json
import sqlite3
import sys


def main():
    db, bench = sys.argv[1], sys.argv[2]
    line = json.load(open(bench))
    b0, b1 = line["value_region"]["boottime_ns"]
    k = line["steps"]
    c = sqlite3.connect(db)
    rows = sorted((int(s), int(e), n) for n, s, e in c.execute("select name, start, end from kernels")
                  if "k_rows2d" in n or "k_rows" in n)
    inside = [r for r in rows if r[0] >= b0 and r[1] <= b1 + 200000]
    inside = inside[:k]
    if len(inside) < k:
        print(json.dumps({"error": f"found {len(inside)} kernels inside the region, expected {k}"}))
        return
    first_start, last_end = inside[0][0], max(e for _, e, _ in inside)
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, _ in sorted(inside):
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    alg = line["config"]["algorithmic_bytes_per_step"]
    out = {
        "region_us": round((b1 - b0) / 1e3, 2),
        "start_to_first_kernel_us": round((first_start - b0) / 1e3, 2),
        "kernels_span_us": round((last_end - first_start) / 1e3, 2),
        "merged_busy_us": round(busy / 1e3, 2),
        "idle_gaps_between_kernels_us": [round(g / 1e3, 2) for g in gaps],
        "last_kernel_end_to_region_end_us": round((b1 - last_end) / 1e3, 2),
        "kernel_durations_us": [round((e - s) / 1e3, 2) for s, e, _ in inside],
        "value_frac": round(alg * k / ((b1 - b0) / 1e9) / 8e12, 4),
        "span_frac": round(alg * k / ((last_end - first_start) / 1e9) / 8e12, 4),
        "first_call_us": line["value_region"]["first_call_us"],
        "enqueue_all_us": line["value_region"]["enqueue_all_us"],
    }
    st = line["value_region"].get("stamps_ns")
    if st:
        # BENCH_STAMPS=1: the library's own host stamps on the same clock
        f, w = st["first_call"], st["wait"]
        us = lambda a, b: round((b - a) / 1e3, 2)
        out["first_call_breakdown_us"] = {
            "python_to_library_entry": us(b0, f[0]),
            "entry_to_route_decided": us(f[0], f[1]),
            "stream_pick": us(f[1], f[2]),
            "plan_and_hip_launch": us(f[2], f[3]),
            "launch_to_call_return": us(f[3], f[4]),
            "launch_return_to_first_kernel_start": us(f[3], first_start),
        }
        out["close_breakdown_us"] = {
            "python_wait_call_to_library_wait_entry": us(st["wait_call_py"], w[0]),
            "wait_entry_to_stream_sync": us(w[0], w[1]),
            "stream_sync_begin_after_last_kernel_end": us(last_end, w[1]),
            "last_kernel_end_to_sync_return": us(last_end, w[2]),
            "sync_return_to_region_end": us(w[2], b1),
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
