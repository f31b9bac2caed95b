#!/usr/bin/env python3
"""Repro probe: strided gets from HBM into a fresh pageable numpy array, four
sub-patches per trial whose page ranges overlap (the pattern NGA_Get produces
when a patch spans four owners), checked after every trial.  Single rank."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ga_amd  # noqa: E402


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    assert ga_amd.comex_init() == 0
    rows, cols = 300, 200
    a = (np.arange(rows * cols, dtype=np.float64) + 1.0).reshape(rows, cols)
    d = ga_amd.DeviceBuffer(a.nbytes)
    d.upload(a)
    bad = 0
    for t in range(trials):
        r0, c0 = 145, 60
        q = np.zeros((40, 50))
        # four pieces split at row 150 and column 100, like four owners
        for (ra, rb), (ca, cb) in [((145, 150), (60, 100)), ((150, 185), (60, 100)), ((150, 185), (100, 110)),
                                   ((145, 150), (100, 110))]:
            src = d.ptr + (ra * cols + ca) * 8
            dst = q.ctypes.data + ((ra - r0) * 50 + (ca - c0)) * 8
            rc = ga_amd.comex_gets(src, [cols * 8], dst, [50 * 8], [(cb - ca) * 8, rb - ra], 1, 0)
            assert rc == 0
        want = a[r0:r0 + 40, c0:c0 + 50]
        if not np.array_equal(q, want):
            bad += 1
            w = np.argwhere(q != want)
            print(f"trial {t}: {len(w)} differ, rows {sorted(set(w[:, 0].tolist()))[:6]} cols "
                  f"{sorted(set(w[:, 1].tolist()))[:6]}", flush=True)
    print(f"hostreg_probe: {bad} of {trials} trials wrong", flush=True)
    ga_amd.comex_finalize()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
