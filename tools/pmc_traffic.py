#!/usr/bin/env python3
"""HBM traffic per launch of the strided-acc kernel from rocprofv3 PMC counters.

Runs (as child processes, the profiled program directly after `--`):
    rocprofv3 --pmc FETCH_SIZE  -- python3 tools/sweep.py --workload W ...
    rocprofv3 --pmc WRITE_SIZE  -- python3 tools/sweep.py --workload W ...
one counter per pass (TCC slots: FETCH_SIZE costs 3 of 4, WRITE_SIZE 2), then
applies the gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE counts
exactly half the bytes of a 16-B/lane coalesced streaming read, so it is
doubled; WRITE_SIZE is exact for 16-B/lane streaming stores.  Both are in KiB.
Writes profiles/pmc_<tag>.json and profiles/pmc_latest.json (read by bench.py).
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_pass(counter, workload, outdir, steps):
    d = os.path.join(outdir, counter)
    # each counter pass under its own hard time limit (a pass asked for more counters than
    # the hardware holds hangs after printing error 38)
    cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
           sys.executable, os.path.join(ROOT, "tools", "sweep.py"), "--workload", workload, "--rounds", "1",
           "--steps", str(steps), "--sets", "8", "--variants", "default"]
    env = dict(os.environ, TMPDIR="/tmp")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        print(r.stdout[-2000:], r.stderr[-2000:], file=sys.stderr)
        raise SystemExit(f"rocprofv3 pass {counter} failed ({r.returncode})")
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {d}")
    vals = []
    with open(files[0]) as f:
        for row in csv.DictReader(f):
            if "k_rows" not in row.get("Kernel_Name", ""):
                continue
            if row.get("Counter_Name") != counter:
                continue
            vals.append(float(row["Counter_Value"]))
    return vals, files[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="H")
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--outdir", default=os.path.join(ROOT, "gpurun_out", "pmc"))
    args = ap.parse_args()
    sys.path.insert(0, ROOT)
    import bench
    op, count, sstr, dstr, desc = bench.WORKLOADS[args.workload]
    alg = 3 * bench.patch_bytes(count)
    fetch, ff = run_pass("FETCH_SIZE", args.workload, args.outdir, args.steps)
    write, wf = run_pass("WRITE_SIZE", args.workload, args.outdir, args.steps)
    # drop the 3 warm-up launches of sweep.py
    fetch_kb = sum(fetch[3:]) / max(1, len(fetch[3:]))
    write_kb = sum(write[3:]) / max(1, len(write[3:]))
    hbm = (2.0 * fetch_kb + write_kb) * 1024.0
    out = {"workload": args.workload, "desc": desc, "launches": len(fetch),
           "FETCH_SIZE_KiB_per_launch": round(fetch_kb, 1), "WRITE_SIZE_KiB_per_launch": round(write_kb, 1),
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950: FETCH_SIZE = half of a 16-B/lane read)",
           "hbm_bytes_per_launch": int(hbm), "algorithmic_bytes_per_launch": alg,
           "hbm_over_algorithmic": round(hbm / alg, 4), "csv": [os.path.relpath(ff, ROOT), os.path.relpath(wf, ROOT)]}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    for name in (f"pmc_{args.tag}_{args.workload}.json", "pmc_latest.json"):
        with open(os.path.join(ROOT, "profiles", name), "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
