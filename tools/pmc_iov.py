#!/usr/bin/env python3
"""HBM traffic of the io-vector accumulate (a roofline for the 1 Mi-pair
apply), from rocprofv3 PMC counters, one counter per pass:

    rocprofv3 --pmc FETCH_SIZE -- python3 tools/scatter_bench.py --pairs N --no-cpu --steps S
    rocprofv3 --pmc WRITE_SIZE -- (the same)

Per call, summed over the call's kernels (the io-vector ones: k_iov*, k_iovh_*, k_rs_*, and
the list-upload copy), in bytes per pair: FETCH_SIZE raw and x2 (MI355X_MICROARCH.md: on
gfx950 FETCH_SIZE tallies each 128-byte request as 64 bytes), WRITE_SIZE.  Against them:
the algorithmic 24 B per pair (src read, dst read, dst write of one f64), and the
line-granular bound of a random single-f64 destination -- a whole 128-byte line read per
pair (MI355X reads whole lines: profiles/r05/s3/granule_probe.jsonl), a 64-byte partial
write, the source and the uploaded destination list (8 + 8 read, 8 written).
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("k_iov", "k_rs_", "k_copy", "k_strided", "k_flat", "k_rows")


def run_pass(counter, pairs, steps, outdir):
    d = os.path.join(outdir, counter)
    cmd = ["timeout", "-s", "KILL", "150", "rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o",
           "pmc", "--", sys.executable, os.path.join(ROOT, "tools", "scatter_bench.py"), "--pairs", str(pairs),
           "--no-cpu", "--steps", str(steps)]
    r = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ, TMPDIR="/tmp"), capture_output=True, text=True,
                       timeout=600)
    if r.returncode != 0:
        print(r.stdout[-2000:], r.stderr[-2000:], file=sys.stderr)
        raise SystemExit(f"rocprofv3 pass {counter} failed ({r.returncode})")
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    per_kernel = {}
    with open(files[0]) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            name = row.get("Kernel_Name", "")
            short = name.split("(")[0].split("<")[0].replace("void ", "").replace("gaamd::", "")
            per_kernel.setdefault(short, []).append(float(row["Counter_Value"]) * 1024.0)   # KiB -> B
    return per_kernel


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--outdir", default=os.path.join(ROOT, "gpurun_out", "pmc_iov"))
    args = ap.parse_args()
    calls = args.steps + 1           # scatter_bench: one untimed call, then --steps
    fetch = run_pass("FETCH_SIZE", args.pairs, args.steps, args.outdir)
    write = run_pass("WRITE_SIZE", args.pairs, args.steps, args.outdir)
    out = {"tool": "pmc_iov", "pairs": args.pairs, "calls": calls, "kernels": {}}
    tot_f = tot_w = 0.0
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith(KERNELS):
            continue
        f = sum(fetch.get(k, [])) / calls
        w = sum(write.get(k, [])) / calls
        tot_f += f
        tot_w += w
        out["kernels"][k] = {"launches_per_call": len(fetch.get(k, [])) / calls,
                             "fetch_raw_B_per_pair": round(f / args.pairs, 2),
                             "write_B_per_pair": round(w / args.pairs, 2)}
    out["fetch_raw_B_per_pair"] = round(tot_f / args.pairs, 2)
    out["fetch_x2_B_per_pair"] = round(2 * tot_f / args.pairs, 2)
    out["write_B_per_pair"] = round(tot_w / args.pairs, 2)
    out["algorithmic_B_per_pair"] = 24
    out["line_granular_bound_B_per_pair"] = {"dst line read": 128, "dst partial write": 64, "src read": 8,
                                             "dst list read": 8, "dst list write (upload)": 8, "total": 216}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
