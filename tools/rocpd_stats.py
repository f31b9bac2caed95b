#!/usr/bin/env python3
"""rocprofv3 rocpd database (run_results.db) -> the `--stats` kernel summary CSV
(Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev) plus
the merged busy time per dispatch of each kernel (consecutive launches on two
library streams overlap, so AverageNs counts their shared time twice; the
merged figure is what the bench's event pair measures).

usage: rocpd_stats.py run_results.db out_stats.csv [out_union.json]"""
import csv
import json
import math
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end from kernels"))
    by = {}
    for name, s, e in rows:
        by.setdefault(name, []).append((int(s), int(e)))
    total_all = sum(e - s for v in by.values() for s, e in v)
    stats, union = [], {}
    for name, iv in by.items():
        d = [e - s for s, e in iv]
        n, tot = len(d), sum(d)
        mean = tot / n
        sd = math.sqrt(sum((x - mean) ** 2 for x in d) / n)
        stats.append([name, n, tot, round(mean, 3), round(100.0 * tot / total_all, 4), min(d), max(d), round(sd, 3)])
        iv.sort()
        busy, cs, ce = 0, None, None
        for s, e in iv:
            if cs is None or s > ce:
                if cs is not None:
                    busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        union[name] = {"dispatches": n, "merged_busy_ns_per_dispatch": round(busy / n, 1),
                       "average_ns": round(mean, 1)}
    stats.sort(key=lambda r: -r[2])
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        w.writerows(stats)
    if len(sys.argv) > 3:
        json.dump(union, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
