#!/usr/bin/env python3
"""Per-launch time of the dominant kernel from a rocprofv3 --kernel-trace CSV,
valid when launches overlap.

With the default two library streams (ga_amd/csrc/sched.cpp) independent
accumulates run concurrently at their edges, so rocprofv3's per-dispatch
AverageNs (end - start of each dispatch) counts the shared time twice and no
longer equals the time one launch costs.  This tool merges the dispatch
intervals of the dominant kernel into busy periods and reports
    busy_union_ns / dispatches
= the GPU time each launch adds, the figure bench.py's event pair measures
(region / steps).  AverageNs is reported beside it.

usage: kernel_union.py <kernel_trace.csv> [--match SUBSTR] [--json OUT]
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="k_rows")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    iv = []
    name = None
    with open(args.trace) as f:
        for row in csv.DictReader(f):
            k = row.get("Kernel_Name", "")
            if args.match not in k:
                continue
            name = k
            iv.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    if not iv:
        raise SystemExit(f"no dispatch matching {args.match!r} in {args.trace}")
    iv.sort()
    busy, cur_s, cur_e, periods = 0, iv[0][0], iv[0][1], 1
    for s, e in iv[1:]:
        if s <= cur_e:
            cur_e = max(cur_e, e)
        else:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
            periods += 1
    busy += cur_e - cur_s
    n = len(iv)
    avg = sum(e - s for s, e in iv) / n
    out = {"kernel": name, "dispatches": n, "avg_dispatch_ns": round(avg, 1),
           "busy_union_ns": busy, "busy_periods": periods, "union_ns_per_dispatch": round(busy / n, 1),
           "note": "union_ns_per_dispatch = merged busy time of all dispatches / dispatches "
                   "(the per-launch cost when launches overlap on two streams)"}
    print(json.dumps(out))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
