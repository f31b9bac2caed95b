#!/usr/bin/env python3
"""GA_Dgemm / GA_Sgemm throughput on one GPU (tuning evidence, not the headline).

C = alpha*A*B + beta*C on n x n GAs (include/ga.h GA_Dgemm; reference capi.c:3518
-> pnga_matmul, matmul.c:1290): every rank gets its op(A) row panel and op(B)
column panel by NGA_Get into HBM, chunked along k, and runs one rocBLAS gemm per
chunk on its own block.  Reports TFLOP/s (2 n^3 per call) of the whole call,
panel gets included, one JSON line per (type, n)."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ga_amd  # noqa: E402

TYPES = {"d": (1004, 8, "GA_Dgemm", ctypes.c_double), "s": (1003, 4, "GA_Sgemm", ctypes.c_float)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="8192,16384")
    ap.add_argument("--types", default="d,s")
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    L = ga_amd.lib()
    assert ga_amd.comex_init() == 0
    assert L.GA_Initialize() == 0
    ia = ga_amd.int_array
    for t in args.types.split(","):
        ctype, esz, fname, scal = TYPES[t]
        fn = getattr(L, fname)
        for n in (int(x) for x in args.n.split(",")):
            g = [L.NGA_Create(ctype, 2, ia([n, n]), b"gm", None) for _ in range(3)]
            for h in g:   # fill each rank's block (fill draws f64 or f32 from the type code)
                lo, hi = (ctypes.c_int * 2)(), (ctypes.c_int * 2)()
                L.NGA_Distribution(h, L.gaamd_rank(), lo, hi)
                ptr, ld = ctypes.c_void_p(), (ctypes.c_int * 1)()
                L.NGA_Access(h, lo, hi, ctypes.byref(ptr), ld)
                cnt = (hi[0] - lo[0] + 1) * (hi[1] - lo[1] + 1)
                ga_amd.fill(ptr.value, cnt, 0 if esz == 8 else 1, 1234 + h)
            ga_amd.sync()
            L.GA_Sync()
            fn(b"N", b"N", n, n, n, scal(1.0), g[0], g[1], scal(0.0), g[2])   # warm: rocBLAS load + first call
            ts = []
            for _ in range(args.iters):
                t0 = time.perf_counter()
                fn(b"N", b"N", n, n, n, scal(1.0), g[0], g[1], scal(0.5), g[2])
                ts.append(time.perf_counter() - t0)
            best = min(ts)
            print(json.dumps({"tool": "gemm_bench", "call": fname, "n": n, "ranks": L.gaamd_size(),
                              "s_per_call_best": round(best, 5), "s_per_call": [round(x, 5) for x in ts],
                              "TFLOPs": round(2.0 * n ** 3 / best / 1e12, 2)}), flush=True)
            for h in g:
                L.GA_Destroy(h)
    L.GA_Terminate()


if __name__ == "__main__":
    main()
