#!/usr/bin/env python3
"""Which dispatches of the headline kernel are slow (rocprofv3
AverageNs 32.1 us over MinNs 30.8 / MaxNs 37.4 us on one stream).

Reads a rocprofv3 kernel trace (rocpd run_results.db) of a ONE-stream bench run
(COMEX_AMD_STREAMS=1, so dispatch durations do not overlap) and groups the
durations of `k_rows2d` dispatches by:
  * what preceded them: the GPU idle for more than 2 us (the first launch after a
    host synchronisation: region starts, warm-up boundaries) or back to back;
  * the step's buffer set (steps rotate over `sets` buffer sets: i % sets);
  * their position in the run (warm-up vs the rest).
and lists the slowest dispatches with their context.
usage: dispatch_tail.py run_results.db [sets=8]"""
import json
import sqlite3
import statistics
import sys


def stats(xs):
    if not xs:
        return None
    xs = sorted(xs)
    q = lambda p: xs[min(len(xs) - 1, int(p * len(xs)))]
    return {"n": len(xs), "min": round(xs[0], 2), "median": round(q(0.5), 2), "mean": round(statistics.fmean(xs), 2),
            "p99": round(q(0.99), 2), "max": round(xs[-1], 2)}


def main():
    db = sys.argv[1]
    sets = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    c = sqlite3.connect(db)
    ks = sorted((int(s), int(e)) for n, s, e in c.execute("select name, start, end from kernels") if "k_rows2d" in n)
    if not ks:
        print(json.dumps({"error": "no k_rows2d dispatches"}))
        return
    rows = []
    prev_end = None
    for i, (s, e) in enumerate(ks):
        gap = None if prev_end is None else (s - prev_end) / 1e3
        rows.append({"i": i, "us": (e - s) / 1e3, "gap_before_us": gap})
        prev_end = e if prev_end is None else max(prev_end, e)
    overlapping = sum(1 for r in rows if r["gap_before_us"] is not None and r["gap_before_us"] < -0.5)
    after_idle = [r["us"] for r in rows if r["gap_before_us"] is not None and r["gap_before_us"] > 2.0]
    b2b = [r["us"] for r in rows if r["gap_before_us"] is not None and r["gap_before_us"] <= 2.0]
    by_set = {k: stats([r["us"] for r in rows if r["i"] % sets == k]) for k in range(sets)}
    # the dispatch right after an idle one, and the second after it (does a burst settle?)
    idle_idx = [r["i"] for r in rows if r["gap_before_us"] is not None and r["gap_before_us"] > 2.0]
    second = [rows[i + 1]["us"] for i in idle_idx if i + 1 < len(rows) and rows[i + 1]["gap_before_us"] <= 2.0]
    slow = sorted(rows, key=lambda r: -r["us"])[:15]
    out = {
        "dispatches": len(rows),
        "overlapping_dispatches": overlapping,
        "all_us": stats([r["us"] for r in rows]),
        "after_gpu_idle_gt_2us": stats(after_idle),
        "second_after_idle": stats(second),
        "back_to_back": stats(b2b),
        "by_buffer_set": by_set,
        "slowest": [{"i": r["i"], "us": round(r["us"], 2),
                     "gap_before_us": None if r["gap_before_us"] is None else round(r["gap_before_us"], 2),
                     "prev_us": round(rows[r["i"] - 1]["us"], 2) if r["i"] else None} for r in slow],
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
