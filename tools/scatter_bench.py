#!/usr/bin/env python3
"""Vector accumulate (comex_accv / ARMCI_AccV feeding
NGA_Scatter_acc) on one GPU, next to the reference's per-pair _acc on the host.

Workload: one io-vector descriptor of n (src, dst) pairs of one f64 each, as GA's
scatter-accumulate hands to ARMCI_AccV (onesided.c:2747 gai_gatscat ->
ARMCI_AccV per owner); destinations uniform at random in a 1 GiB array (so a
few repeat, which must be applied in order), sources one contiguous vector
(GA's `v`) in HBM (--src dev) or in pageable host memory (--src host, the MA
case).  Algorithmic bytes: 24 per pair.  One JSON line per configuration:
whole-call rate (host work + kernel, wall clock over --steps calls) and the
CPU reference (oracle/_ref ref_accv: comex.c:7327-7400 -> _acc per pair) on
one host thread over host copies of the same lists.
Tuning/measurement evidence, not the headline bench."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ga_amd  # noqa: E402

DBL = 38
ALPHA = 0.7071067811865476


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", default="65536,1048576,4194304")
    ap.add_argument("--src", default="dev", choices=["dev", "host"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--slots", type=int, default=0,
                    help="destinations drawn from this many f64 slots (repeats) instead of the whole 1 GiB")
    ap.add_argument("--ab", action="store_true",
                    help="interleaved A/B of the LDS ordering paths (tuning iov_lds=1: one workgroup below 1 Ki "
                         "pairs, hash partitions up to 1 Mi) against the hashed / radix paths (iov_lds=0): "
                         "5 alternations of --steps calls each")
    ap.add_argument("--ab-key", default="iov_lds",
                    help="the tuning key --ab alternates between 1 and 0 (iov_lds; iov_flag was a round-6 experiment, since removed)")
    ap.add_argument("--nb", action="store_true",
                    help="also time --steps non-blocking calls back to back (comex_nbaccv, one wait at the end)")
    ap.add_argument("--ga", action="store_true",
                    help="NGA_Scatter_acc_flat / NGA_Gather_flat of n elements of a 16384^2 f64 GA (host v)")
    args = ap.parse_args()
    L = ga_amd.lib()
    if args.ga:
        return ga_main(L, args)
    assert ga_amd.comex_init() == 0
    region = 1 << 30
    dstb = ga_amd.DeviceBuffer(region)
    L.gaamd_memset(ctypes.c_void_p(dstb.ptr), 0, region)
    rng = np.random.default_rng(7)
    keep_s, sp = ga_amd.scale_buffer(DBL, ALPHA)
    for n in [int(x) for x in args.pairs.split(",")]:
        idx = rng.integers(0, args.slots or region // 8, n).astype(np.uint64)
        dups = n - len(np.unique(idx))
        v = rng.random(n)
        if args.src == "dev":
            vb = ga_amd.DeviceBuffer(8 * n)
            vb.upload(v)
            sbase = vb.ptr
        else:
            vb = None
            sbase = v.ctypes.data
        src_list = (np.uint64(sbase) + 8 * np.arange(n, dtype=np.uint64)).astype(np.uint64)
        dst_list = (np.uint64(dstb.ptr) + 8 * idx).astype(np.uint64)
        g = ga_amd.GIOV()
        g.src = ctypes.cast(ctypes.c_void_p(src_list.ctypes.data), ctypes.POINTER(ctypes.c_void_p))
        g.dst = ctypes.cast(ctypes.c_void_p(dst_list.ctypes.data), ctypes.POINTER(ctypes.c_void_p))
        g.count, g.bytes = n, 8

        def call():
            rc = L.comex_accv(DBL, sp, ctypes.byref(g), 1, 0, 0)
            assert rc == 0, rc

        def timed():
            call()
            ga_amd.sync()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                call()
            ga_amd.sync()
            return (time.perf_counter() - t0) / args.steps

        paths0 = ga_amd.iov_path_counts()
        el = timed()
        paths1 = ga_amd.iov_path_counts()
        line = {"tool": "scatter_bench", "pairs": n, "bytes_per_pair": 8, "repeated_destinations": int(dups),
                "src": args.src, "steps": args.steps, "ms_per_call": round(el * 1e3, 3),
                "Mpairs_per_s": round(n / el / 1e6, 2), "GBps_alg": round(24 * n / el / 1e9, 2),
                "kernel": ga_amd.last_launch(),
                "iov_path": [k for k in paths1 if paths1[k] > paths0[k]]}
        if args.ab:
            runs = {1: [], 0: []}
            for _ in range(5):
                for val in (1, 0):
                    old = ga_amd.set_tuning(args.ab_key, val)
                    runs[val].append(timed())
                    ga_amd.set_tuning(args.ab_key, old)
            # (files written before the partitioned path named these "lds_one_launch" /
            # "hashed_three_launches")
            names = {"iov_lds": ("lds_paths", "hashed_radix_paths")}.get(args.ab_key, ("on", "off"))
            line["ab_key"] = args.ab_key
            line["ab_ms_per_call"] = {names[0]: [round(x * 1e3, 4) for x in runs[1]],
                                      names[1]: [round(x * 1e3, 4) for x in runs[0]]}
        if args.nb:
            hs = [ctypes.c_int(-1) for _ in range(args.steps)]
            call()
            ga_amd.sync()
            t0 = time.perf_counter()
            for h in hs:
                assert L.comex_nbaccv(DBL, sp, ctypes.byref(g), 1, 0, 0, ctypes.byref(h)) == 0
            assert L.comex_wait_all(0) == 0
            line["nb_ms_per_call"] = round((time.perf_counter() - t0) / args.steps * 1e3, 4)
        if not args.no_cpu:
            from oracle import Ref, ref_available
            if ref_available():
                hd = np.zeros(region // 8)
                hs = v.copy()
                s_list = (np.uint64(hs.ctypes.data) + 8 * np.arange(n, dtype=np.uint64)).astype(np.uint64)
                d_list = (np.uint64(hd.ctypes.data) + 8 * idx).astype(np.uint64)
                ref = Ref()
                ref.accv(DBL, ALPHA, s_list, d_list, 8)   # page-in
                reps, t0 = 0, time.perf_counter()
                while True:
                    ref.accv(DBL, ALPHA, s_list, d_list, 8)
                    reps += 1
                    if time.perf_counter() - t0 > 1.0 and reps >= 2:
                        break
                ce = (time.perf_counter() - t0) / reps
                line["cpu_reference"] = {"cores": 1, "ms_per_call": round(ce * 1e3, 3),
                                         "Mpairs_per_s": round(n / ce / 1e6, 2),
                                         "kind": "reference acc.h _acc per pair (oracle/_ref ref_accv)"}
                del hd
        print(json.dumps(line), flush=True)
        if vb is not None:
            vb.free()
    ga_amd.comex_finalize()


def ga_main(L, args):
    """GA caller layer: gai_gatscat owner grouping (onesided.c:2747) -> one ARMCI_AccV /
    ARMCI_GetV per owner (one owner here), subscripts and `v` in host memory."""
    assert L.GA_Initialize() == 0
    side = 16384
    g = L.NGA_Create(1004, 2, ga_amd.int_array([side, side]), b"scat", None)
    assert g > 0
    L.GA_Zero(g)
    rng = np.random.default_rng(3)
    alpha = ctypes.c_double(ALPHA)
    for n in [int(x) for x in args.pairs.split(",")]:
        subs = rng.integers(0, side, 2 * n).astype(np.int32)
        v = rng.random(n)
        out = np.zeros(n)
        sp = subs.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
        for name, fn in (("NGA_Scatter_acc_flat",
                          lambda: L.NGA_Scatter_acc_flat(g, ctypes.c_void_p(v.ctypes.data), sp, n, ctypes.byref(alpha))),
                         ("NGA_Gather_flat", lambda: L.NGA_Gather_flat(g, ctypes.c_void_p(out.ctypes.data), sp, n))):
            fn()
            ga_amd.sync()

            def timed():
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    fn()
                ga_amd.sync()
                return (time.perf_counter() - t0) / args.steps
            el = timed()
            line = {"tool": "scatter_bench", "api": name, "elements": n, "ga": f"{side}^2 f64, 1 rank",
                    "steps": args.steps, "ms_per_call": round(el * 1e3, 3), "Melems_per_s": round(n / el / 1e6, 2)}
            if args.ab:   # interleaved: --ab-key at 1, then 0, five times
                runs = {1: [], 0: []}
                for _ in range(5):
                    for val in (1, 0):
                        old = ga_amd.set_tuning(args.ab_key, val)
                        runs[val].append(timed())
                        ga_amd.set_tuning(args.ab_key, old)
                line["ab_key"] = args.ab_key
                line["ab_ms_per_call"] = {"on": [round(x * 1e3, 3) for x in runs[1]],
                                          "off": [round(x * 1e3, 3) for x in runs[0]]}
            print(json.dumps(line), flush=True)
    L.GA_Terminate()


if __name__ == "__main__":
    main()
