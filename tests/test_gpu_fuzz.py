"""Seeded random strided descriptors through the C ABI, bit-exact against the oracle
(the CPU restatement of comex.c's odometer + acc.h's `_acc`, itself pinned against the
reference's compiled acc.h / iterator.c: tests/test_oracle*.py).

The golden cases (tests/golden/) cover the shapes the reference's tests and SURVEY §8(d)
name; this file draws the rest of the descriptor space at random, so that the launcher's
choice among its kernel families (flat, rows, 2-D rows, column-ordered, ordered rows,
serial) is exercised on geometries nobody wrote down:
  * every op (comex.h COMEX_ACC_*), stride levels 0..7 (comex.c:1273's int[7] odometer);
  * row lengths log-uniform from one element to 8 Ki elements (either side of the
    flat/rows thresholds and the 64-lane wave);
  * strides padded past the row, smaller than it (rows overlap: the reference's row order
    decides the bytes), or zero (every row onto one run);
  * offsets at the element's alignment or below it (4 bytes for 8/16-byte types: a
    Fortran complex*16 array is only 8-byte aligned);
  * src inside the dst buffer (a patch of one array into another patch of it);
  * random alpha, including negative and complex values.
Each case also runs pack -> unpack-acc (comex.c:1267-1328, 4238-4268) and, for puts,
a byte-granular row length. Sizes stay below 2 MiB a case so the whole file runs in
seconds."""
import ctypes
import os

import numpy as np
import pytest

import cases as C
import ga_amd
from helpers import first_mismatch, same_bits_nan_aware

pytestmark = pytest.mark.gpu

OPS = (C.INT, C.DBL, C.FLT, C.CPL, C.DCP, C.LNG)
# GAAMD_FUZZ_SEED shifts every seed (soak runs: tools/sessions/r05_soak.sh); 0 is the suite's
SEED = int(os.environ.get("GAAMD_FUZZ_SEED", "0")) * 100003


def random_alpha(rng, op):
    if op in (C.INT, C.LNG):
        return int(rng.integers(-5, 6))
    if op in (C.FLT, C.DBL):
        return float(rng.uniform(-2, 2))
    return complex(rng.uniform(-2, 2), rng.uniform(-2, 2))


def random_side(rng, count, levels, esz, allow_overlap):
    """strides of one side: past the row (padded), inside it (overlap) or zero"""
    strides, span = [], count[0]
    for j in range(levels):
        r = rng.random()
        if allow_overlap and r < 0.06:
            s = 0
        elif allow_overlap and r < 0.16:
            s = esz * int(rng.integers(1, max(2, span // esz)))
        else:
            s = span + esz * int(rng.integers(0, 5))
        strides.append(s)
        span = s * (count[j + 1] - 1) + span
    return strides


def random_case(rng, op):
    esz = C.ESZ[op]
    levels = int(rng.choice([0, 1, 1, 1, 2, 2, 3, 4, 5, 6, 7]))
    row_el = max(1, int(np.exp(rng.uniform(0, np.log(8192)))))
    count = [row_el * esz]
    rows = max(1, (2 << 20) // count[0])
    for _ in range(levels):
        c = int(rng.integers(1, min(9, rows) + 1))
        rows = max(1, rows // c)
        count.append(c)
    ss = random_side(rng, count, levels, esz, allow_overlap=True)
    ds = random_side(rng, count, levels, esz, allow_overlap=True)
    sub = min(esz, 4) if (esz >= 8 and rng.random() < 0.2) else esz   # below natural alignment
    so = sub * int(rng.integers(0, 16))
    do = sub * int(rng.integers(0, 16))
    alias = rng.random() < 0.15
    if alias:   # both sides' elements at one phase of the shared buffer's fill
        so += (do - so) % esz
    return dict(op=op, count=count, levels=levels, ss=ss, ds=ds, so=so, do=do, alias=alias,
                alpha=random_alpha(rng, op))


def phased_fill(op, nbytes, off, seed):
    """fill values laid out from byte `off % esz` on, so that the elements a side
    reads at an offset below the natural alignment are the generator's values, not
    bit patterns straddling two of them (which include NaNs: the sign and payload of
    a NaN that arithmetic produces are not pinned, so they would differ in the bytes)"""
    ph = off % C.ESZ[op]
    out = np.zeros(nbytes, dtype=np.uint8)
    out[ph:] = C.fill_bytes(op, nbytes - ph, seed)
    return out


def run_case(L, oracle, k, case):
    op, count, levels = case["op"], case["count"], case["levels"]
    ss, ds, so, do = case["ss"], case["ds"], case["so"], case["do"]
    s_hi = so + C.span(ss, count, levels)[1]
    d_hi = do + C.span(ds, count, levels)[1]
    if case["alias"]:
        d_hi = max(d_hi, s_hi)
    src = phased_fill(op, max(16, s_hi), so, 1000 + k)
    dst = phased_fill(op, max(16, d_hi), do, 2000 + k)
    sb, db = ga_amd.DeviceBuffer(src.size), ga_amd.DeviceBuffer(dst.size)
    try:
        sb.upload(src)
        db.upload(dst)
        keep, sp = ga_amd.scale_buffer(op, case["alpha"])
        sptr = (db.ptr if case["alias"] else sb.ptr) + so
        rc = L.comex_accs(op, sp, ctypes.c_void_p(sptr), ga_amd.int_array(ss), ctypes.c_void_p(db.ptr + do),
                          ga_amd.int_array(ds), ga_amd.int_array(count), levels, 0, 0)
        assert rc == 0
        assert L.comex_fence_all(0) == 0
        got = db.download(np.uint8, dst.size)
        want = dst.copy()
        if case["alias"]:
            oracle.accs(op, case["alpha"], want, so, ss, want, do, ds, count, levels)
        else:
            oracle.accs(op, case["alpha"], src, so, ss, want, do, ds, count, levels)
        # compare from the dst elements' phase, so a NaN (whose sign and payload are not
        # pinned; an overflowing recurrence of an aliased patch makes them) is seen whole
        ph = do % np.dtype(C.REAL[op]).itemsize
        if not (np.array_equal(got[:ph], want[:ph]) and same_bits_nan_aware(got[ph:], want[ph:], op)):
            return f"accs {case}: {first_mismatch(got[ph:], want[ph:], op)}"
        return None
    finally:
        sb.free()
        db.free()


@pytest.mark.parametrize("op", OPS, ids=lambda o: C.NAMES[o])
def test_random_strided_accumulates(gpu_lib, oracle, op):
    """200 random descriptors per op through comex_accs, bit-exact against the oracle."""
    rng = np.random.default_rng(9000 + op + SEED)
    bad = []
    for k in range(200):
        err = run_case(gpu_lib, oracle, k, random_case(rng, op))
        if err:
            bad.append(err)
    assert not bad, "\n".join(bad[:5]) + f"\n({len(bad)} of 200 cases differ)"


@pytest.mark.parametrize("knob", [("kind", 1), ("kind", 2), ("kind", 4), ("block", 64), ("block", 128), ("align", 0),
                                  ("flat_line_min", 0), ("ordered_cols", 0), ("ordered_cols", 1)],
                         ids=lambda k: f"{k[0]}={k[1]}")
def test_random_strided_accumulates_every_kernel_family(gpu_lib, oracle, knob):
    """The same random descriptors with the launcher's choices forced one way (kernel
    family, block size, chunk alignment, the flat/rows line rule, the column kernels):
    every variant it ships gives the reference's bytes, not only the one it picks."""
    key, val = knob
    old = ga_amd.set_tuning(key, val)
    try:
        rng = np.random.default_rng(5000 + sum(map(ord, key)) + val + SEED)
        bad = []
        for k in range(60):
            op = OPS[k % len(OPS)]
            err = run_case(gpu_lib, oracle, k, random_case(rng, op))
            if err:
                bad.append(err)
        assert not bad, "\n".join(bad[:5]) + f"\n({len(bad)} of 60 cases differ)"
    finally:
        ga_amd.set_tuning(key, old)


@pytest.mark.parametrize("seed", range(4))
def test_random_pack_unpack_acc_and_puts(gpu_lib, oracle, seed):
    """Random descriptors through pack -> unpack-acc and unpack (the remote path's two
    kernels) and through comex_puts / comex_gets with byte-granular rows, against the
    oracle's pack / unpack / unpack_acc / puts (pinned against iterator.c)."""
    rng = np.random.default_rng(7000 + seed + SEED)
    for k in range(60):
        op = OPS[int(rng.integers(0, len(OPS)))]
        case = random_case(rng, op)
        count, levels = case["count"], case["levels"]
        # the packed path reads src without overlap concerns; dst rows must not overlap
        # for unpack (a put into overlapping rows is order-dependent in the same way)
        ss = case["ss"]
        ds = random_side(rng, count, levels, C.ESZ[op], allow_overlap=False)
        src = C.fill_bytes(op, C.span(ss, count, levels)[1], 300 + k)
        dst = C.fill_bytes(op, C.span(ds, count, levels)[1], 400 + k)
        P = oracle.packed_size(count, levels)
        sb, db, pb = ga_amd.DeviceBuffer(src.size), ga_amd.DeviceBuffer(dst.size), ga_amd.DeviceBuffer(max(16, P))
        try:
            sb.upload(src)
            db.upload(dst)
            ga_amd.pack(sb.ptr, ss, count, levels, pb.ptr)
            ga_amd.sync()
            packed = pb.download(np.uint8, P)
            assert np.array_equal(packed, oracle.pack(src, 0, ss, count, levels)), case
            ga_amd.unpack_acc(op, case["alpha"], pb.ptr, db.ptr, ds, count, levels)
            ga_amd.sync()
            want = dst.copy()
            oracle.unpack_acc(op, case["alpha"], packed, want, 0, ds, count, levels)
            got = db.download(np.uint8, dst.size)
            assert same_bits_nan_aware(got, want, op), (case, first_mismatch(got, want, op))
            ga_amd.unpack(pb.ptr, db.ptr, ds, count, levels)
            ga_amd.sync()
            oracle.unpack(packed, want, 0, ds, count, levels)
            assert np.array_equal(db.download(np.uint8, dst.size), want), case
        finally:
            sb.free()
            db.free()
            pb.free()
        # puts / gets: rows of any byte length, offsets of any byte
        bcount = [count[0] + int(rng.integers(0, 8))] + count[1:]
        bss = random_side(rng, bcount, levels, 1, allow_overlap=False)
        bds = random_side(rng, bcount, levels, 1, allow_overlap=False)
        bso, bdo = int(rng.integers(0, 16)), int(rng.integers(0, 16))
        s8 = rng.integers(0, 256, bso + C.span(bss, bcount, levels)[1], dtype=np.uint8)
        d8 = rng.integers(0, 256, bdo + C.span(bds, bcount, levels)[1], dtype=np.uint8)
        sb, db = ga_amd.DeviceBuffer(s8.size), ga_amd.DeviceBuffer(d8.size)
        try:
            sb.upload(s8)
            db.upload(d8)
            assert ga_amd.comex_puts(sb.ptr + bso, bss, db.ptr + bdo, bds, bcount, levels, 0) == 0
            ga_amd.comex_fence_all()
            want = d8.copy()
            oracle.puts(s8, bso, bss, want, bdo, bds, bcount, levels)
            assert np.array_equal(db.download(np.uint8, d8.size), want), (bcount, bss, bds)
            back = np.zeros_like(s8)
            sb.upload(back)
            assert ga_amd.comex_gets(db.ptr + bdo, bds, sb.ptr + bso, bss, bcount, levels, 0) == 0
            ga_amd.comex_fence_all()
            want_back = back.copy()
            oracle.puts(want, bdo, bds, want_back, bso, bss, bcount, levels)
            assert np.array_equal(sb.download(np.uint8, s8.size), want_back), (bcount, bss, bds)
        finally:
            sb.free()
            db.free()


def _giov(src_addrs, dst_addrs, nbytes):
    src_addrs = np.ascontiguousarray(src_addrs, dtype=np.uint64)
    dst_addrs = np.ascontiguousarray(dst_addrs, dtype=np.uint64)
    g = ga_amd.GIOV()
    g._keep = (src_addrs, dst_addrs)
    g.src = ctypes.cast(ctypes.c_void_p(src_addrs.ctypes.data), ctypes.POINTER(ctypes.c_void_p))
    g.dst = ctypes.cast(ctypes.c_void_p(dst_addrs.ctypes.data), ctypes.POINTER(ctypes.c_void_p))
    g.count, g.bytes = len(src_addrs), nbytes
    return g


def random_pairs(rng, n, nbytes, esz):
    """(src offsets, dst offsets, dst region bytes): sources one vector in pair order
    (GA's `v`), a permutation or random repeats; destinations one vector (cannot
    repeat), sparse random (a few repeats, the hashed path), dense random (many repeats,
    conflicts beyond the LDS list: the radix fallback) or a small hot set"""
    k = int(rng.integers(0, 3))
    if k == 0:
        so = np.arange(n, dtype=np.uint64) * np.uint64(nbytes)
    elif k == 1:
        so = rng.permutation(n).astype(np.uint64) * np.uint64(nbytes)
    else:
        so = rng.integers(0, n, n).astype(np.uint64) * np.uint64(nbytes)
    mode = int(rng.integers(0, 4))
    if mode == 0:
        do, slots = np.arange(n, dtype=np.uint64) * np.uint64(nbytes), n
        return so, do, n * nbytes
    slots = {1: 8 * n + 16, 2: max(1, n // 4), 3: int(rng.integers(1, 64))}[mode]
    # destinations on a grid of whole pairs, or (when a pair holds several elements)
    # of single elements, so that pairs overlap partially
    step = nbytes if rng.random() < 0.7 else esz
    do = rng.integers(0, slots, n).astype(np.uint64) * np.uint64(step)
    return so, do, slots * step + nbytes


@pytest.mark.parametrize("seed", range(6))
def test_random_io_vectors(gpu_lib, oracle, seed):
    """comex_accv / comex_putv / comex_getv (comex.c:7327-7400) on random pair lists
    through every ordering path the io-vector code has (contiguous sides, hashed
    repeats, radix fallback, per-pair serial), sources in HBM or pageable host memory,
    1 to 150 000 pairs: bit-exact against the oracle's pair-by-pair loop (ora_accv /
    ora_copyv, pinned against the reference's _acc per pair)."""
    rng = np.random.default_rng(6000 + seed + SEED)
    for k in range(12):
        kind = ("acc", "acc", "put", "get")[k % 4]
        op = OPS[int(rng.integers(0, len(OPS)))] if kind == "acc" else C.DBL
        esz = C.ESZ[op]
        nel = int(rng.choice([1, 1, 1, 2, 3, 8]))
        nbytes = esz * nel if kind == "acc" else int(rng.choice([esz * nel, 1 + int(rng.integers(0, 40))]))
        n = max(1, int(np.exp(rng.uniform(0, np.log(150000)))))
        so, do, d_bytes = random_pairs(rng, n, nbytes, esz if kind == "acc" else 1)
        s_bytes = int(so.max()) + nbytes
        src_h = C.fill_bytes(op, s_bytes, 50 + k)
        dst_h = C.fill_bytes(op, d_bytes, 60 + k)
        host_src = kind != "get" and rng.random() < 0.3
        host_dst = kind == "get" and rng.random() < 0.5
        sb = None if host_src else ga_amd.DeviceBuffer(s_bytes)
        db = None if host_dst else ga_amd.DeviceBuffer(d_bytes)
        src_g = src_h.copy()                      # what the library reads when host_src
        dst_g = dst_h.copy()                      # what the library writes when host_dst
        try:
            if sb:
                sb.upload(src_h)
            if db:
                db.upload(dst_h)
            s_base = src_g.ctypes.data if host_src else sb.ptr
            d_base = dst_g.ctypes.data if host_dst else db.ptr
            g = _giov(so + np.uint64(s_base), do + np.uint64(d_base), nbytes)
            if kind == "acc":
                alpha = random_alpha(rng, op)
                keep, sp = ga_amd.scale_buffer(op, alpha)
                assert gpu_lib.comex_accv(op, sp, ctypes.byref(g), 1, 0, 0) == 0
            elif kind == "put":
                assert gpu_lib.comex_putv(ctypes.byref(g), 1, 0, 0) == 0
            else:
                assert gpu_lib.comex_getv(ctypes.byref(g), 1, 0, 0) == 0
            ga_amd.comex_fence_all()
            got = dst_g if host_dst else db.download(np.uint8, d_bytes)
            want = dst_h.copy()
            sa, da = so + np.uint64(src_h.ctypes.data), do + np.uint64(want.ctypes.data)
            if kind == "acc":
                oracle.accv(op, alpha, sa, da, nbytes)
            else:
                oracle.copyv(sa, da, nbytes)
            what = dict(kind=kind, op=C.NAMES[op], n=n, nbytes=nbytes, host_src=host_src, host_dst=host_dst)
            assert same_bits_nan_aware(got, want, op), (what, first_mismatch(got, want, op))
        finally:
            if sb:
                sb.free()
            if db:
                db.free()
