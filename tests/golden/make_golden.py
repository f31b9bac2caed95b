"""Generate tests/golden/golden.npz + manifest.json from the REFERENCE's own _acc.

Run in the survey container (where /root/reference exists):

    make -C oracle            # builds oracle/_ref/libref_acc.so from acc.h
    python tests/golden/make_golden.py

For every case of cases.py the inputs (src, dst before) and the expected dst
after one comex_accs-equivalent call are stored.  The expected dst comes from
oracle/_ref: the reference's _acc (comex/src-common/acc.h:106-154, HAVE_BLAS=0)
applied row by row in the nb_accs odometer order (comex.c:6936-6961).  For the
full-size configurations (C2, H, C3, C4 of SURVEY.md §8(d)) only the sha256 of
the whole dst buffer after the call is kept, since the buffers are 256+ MiB.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import cases as C  # noqa: E402
from oracle import Ref, Oracle  # noqa: E402


def full_size_configs():
    """SURVEY.md §8(d) shapes (bytes, strides in bytes)."""
    return [
        dict(name="C2_1d_f64_64MiB", op=C.DBL, count=[64 << 20], levels=0, src_stride=[], dst_stride=[],
             src_off=0, dst_off=0, src_bytes=64 << 20, dst_bytes=64 << 20),
        dict(name="H_2d_f64_2048x4096_ld8192", op=C.DBL, count=[2048 * 8, 4096], levels=1,
             src_stride=[8192 * 8], dst_stride=[8192 * 8], src_off=0, dst_off=0,
             src_bytes=8192 * 8 * 4095 + 2048 * 8, dst_bytes=8192 * 8 * 4095 + 2048 * 8),
        dict(name="H_2d_f64_2048x4096_ld8200", op=C.DBL, count=[2048 * 8, 4096], levels=1,
             src_stride=[8200 * 8], dst_stride=[8200 * 8], src_off=0, dst_off=0,
             src_bytes=8200 * 8 * 4095 + 2048 * 8, dst_bytes=8200 * 8 * 4095 + 2048 * 8),
        dict(name="C3_2d_f64_4096x4096_ld8192", op=C.DBL, count=[4096 * 8, 4096], levels=1,
             src_stride=[8192 * 8], dst_stride=[8192 * 8], src_off=0, dst_off=0,
             src_bytes=8192 * 8 * 4095 + 4096 * 8, dst_bytes=8192 * 8 * 4095 + 4096 * 8),
        dict(name="C4_3d_dcpl_256cubed", op=C.DCP, count=[4096, 256, 256], levels=2,
             src_stride=[4096, 1048576], dst_stride=[4224, 1115136], src_off=0, dst_off=0,
             src_bytes=4096 * 256 * 256, dst_bytes=1115136 * 255 + 4224 * 255 + 4096),
    ]


def run_ref(ref, case, src, dst):
    if case.get("alias"):
        src = dst   # src = dst buffer + src_off: the reference's _acc on aliased memory
    ref.accs(case["op"], C.SCALE[case["op"]], src, case["src_off"], case["src_stride"], dst, case["dst_off"],
             case["dst_stride"], case["count"], case["levels"])


def main():
    ref = Ref()
    ora = Oracle()
    arrays = {}
    manifest = {"generator": "tests/golden/make_golden.py", "expected_by": "oracle/_ref (reference acc.h _acc)",
                "seed": C.SEED, "cases": [], "full_size": []}
    for case in C.cases():
        src, dst = C.make_inputs(case)
        out = dst.copy()
        run_ref(ref, case, src, out)
        # the restatement must agree bit for bit before anything is committed
        chk = dst.copy()
        ora.accs(case["op"], C.SCALE[case["op"]], chk if case.get("alias") else src, case["src_off"],
                 case["src_stride"], chk, case["dst_off"], case["dst_stride"], case["count"], case["levels"])
        assert np.array_equal(chk, out), case["name"]
        n = case["name"]
        arrays[f"{n}/src"] = src
        arrays[f"{n}/dst_in"] = dst
        arrays[f"{n}/dst_out"] = out
        m = {k: v for k, v in case.items()}
        m["scale"] = repr(C.SCALE[case["op"]])
        manifest["cases"].append(m)
    np.savez_compressed(os.path.join(HERE, "golden.npz"), **arrays)

    for cfg in full_size_configs():
        src = C.fill_bytes(cfg["op"], cfg["src_bytes"], C.SEED)
        dst = C.fill_bytes(cfg["op"], cfg["dst_bytes"], C.SEED + 1)
        run_ref(ref, cfg, src, dst)
        cfg = dict(cfg)
        cfg["dst_sha256"] = hashlib.sha256(dst.tobytes()).hexdigest()
        cfg["src_sha256"] = hashlib.sha256(src.tobytes()).hexdigest()
        manifest["full_size"].append(cfg)
        print(cfg["name"], cfg["dst_sha256"][:16])
        del src, dst
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"{len(manifest['cases'])} cases, {os.path.getsize(os.path.join(HERE, 'golden.npz')) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
