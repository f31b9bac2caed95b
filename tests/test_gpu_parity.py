"""GPU parity: the HIP path through the C ABI against the reference's golden
vectors (bit-exact; NaN payloads excepted) and the oracle.  Runs on the MI355X."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

import cases as C
import ga_amd
from helpers import same_bits_nan_aware, first_mismatch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_case_device(L, case, src, dst_in, api="comex", kind=None):
    """One golden case through the C ABI; an `alias` case reads src from the dst
    buffer (a patch of one array accumulated into another patch of it)."""
    sbuf = ga_amd.DeviceBuffer(max(16, src.size))
    dbuf = ga_amd.DeviceBuffer(max(16, dst_in.size))
    sbuf.upload(src)
    dbuf.upload(dst_in)
    op = case["op"]
    keep, sp = ga_amd.scale_buffer(op, C.SCALE[op])
    ss, ds, cnt = ga_amd.int_array(case["src_stride"]), ga_amd.int_array(case["dst_stride"]), ga_amd.int_array(case["count"])
    sptr = ctypes.c_void_p((dbuf.ptr if case.get("alias") else sbuf.ptr) + case["src_off"])
    dptr = ctypes.c_void_p(dbuf.ptr + case["dst_off"])
    if api == "comex":
        rc = L.comex_accs(op, sp, sptr, ss, dptr, ds, cnt, case["levels"], 0, 0)
    elif api == "armci":
        rc = L.ARMCI_AccS(op, sp, sptr, ss, dptr, ds, cnt, case["levels"], 0)
    elif api == "nb":
        h = ctypes.c_int(-1)
        rc = L.comex_nbaccs(op, sp, sptr, ss, dptr, ds, cnt, case["levels"], 0, 0, ctypes.byref(h))
        assert rc == 0
        rc = L.comex_wait(ctypes.byref(h))
    elif api == "kernel":
        rc = L.gaamd_strided(op, sp, sptr, ss, dptr, ds, cnt, case["levels"], None)
    assert rc == 0
    assert L.comex_fence_all(0) == 0
    out = dbuf.download(np.uint8, dst_in.size)
    sbuf.free()
    dbuf.free()
    return out


def test_golden_cases_comex_accs(gpu_lib, manifest, golden):
    bad = []
    for case in manifest["cases"]:
        n = case["name"]
        out = run_case_device(gpu_lib, case, golden[f"{n}/src"], golden[f"{n}/dst_in"])
        if not same_bits_nan_aware(out, golden[f"{n}/dst_out"], case["op"]):
            bad.append(f"{n}: {first_mismatch(out, golden[f'{n}/dst_out'], case['op'])}")
    assert not bad, "\n".join(bad)


def test_golden_cases_armci_and_nb(gpu_lib, manifest, golden):
    bad = []
    for case in manifest["cases"][::3]:
        n = case["name"]
        for api in ("armci", "nb"):
            out = run_case_device(gpu_lib, case, golden[f"{n}/src"], golden[f"{n}/dst_in"], api=api)
            if not same_bits_nan_aware(out, golden[f"{n}/dst_out"], case["op"]):
                bad.append(f"{api} {n}")
    assert not bad, bad


@pytest.mark.parametrize("knob", [("kind", 1), ("kind", 2), ("kind", 3), ("kind", 4), ("block", 128), ("block", 64),
                                  ("align", 0), ("align", 1), ("flat_line_min", 0), ("ordered_cols", 0)])
def test_kernel_variants_identical(gpu_lib, manifest, golden, knob):
    """Every shipped kernel family / tuning gives the same bits as the reference
    (ordered_cols 0: the coinciding-row golden cases on the one-workgroup kernel)."""
    key, val = knob
    old = ga_amd.set_tuning(key, val)
    try:
        bad = []
        for case in manifest["cases"]:
            n = case["name"]
            if key == "kind" and val in (3, 4) and case["count"][0] * np.prod(case["count"][1:]) > 200000:
                continue
            out = run_case_device(gpu_lib, case, golden[f"{n}/src"], golden[f"{n}/dst_in"], api="kernel")
            if not same_bits_nan_aware(out, golden[f"{n}/dst_out"], case["op"]):
                bad.append(n)
        assert not bad, bad
    finally:
        ga_amd.set_tuning(key, old)


def _random_patch(rng, levels, esz):
    count = [int(rng.integers(1, 40)) * esz] + [int(rng.integers(1, 6)) for _ in range(levels)]
    ss, ds, a, b = [], [], count[0] + esz * int(rng.integers(0, 3)), count[0] + esz * int(rng.integers(0, 3))
    for j in range(levels):
        ss.append(a)
        ds.append(b)
        a = a * count[j + 1] + esz * int(rng.integers(0, 2))
        b = b * count[j + 1] + esz * int(rng.integers(0, 2))
    return count, ss, ds


@pytest.mark.parametrize("levels", [0, 1, 2, 3, 5, 7])
def test_pack_unpack_unpack_acc(gpu_lib, oracle, levels):
    rng = np.random.default_rng(100 + levels)
    for op in (C.DBL, C.DCP, C.INT):
        esz = C.ESZ[op]
        count, ss, ds = _random_patch(rng, levels, esz)
        src = C.fill_bytes(op, C.span(ss, count, levels)[1], 5)
        dst = C.fill_bytes(op, C.span(ds, count, levels)[1], 6)
        P = oracle.packed_size(count, levels)
        sb, db, pb = ga_amd.DeviceBuffer(src.size), ga_amd.DeviceBuffer(dst.size), ga_amd.DeviceBuffer(P)
        sb.upload(src)
        db.upload(dst)
        ga_amd.pack(sb.ptr, ss, count, levels, pb.ptr)
        ga_amd.sync()
        packed = pb.download(np.uint8, P)
        assert np.array_equal(packed, oracle.pack(src, 0, ss, count, levels))
        ga_amd.unpack_acc(op, C.SCALE[op], pb.ptr, db.ptr, ds, count, levels)
        ga_amd.sync()
        want = dst.copy()
        oracle.unpack_acc(op, C.SCALE[op], packed, want, 0, ds, count, levels)
        assert np.array_equal(db.download(np.uint8, dst.size), want)
        ga_amd.unpack(pb.ptr, db.ptr, ds, count, levels)
        ga_amd.sync()
        oracle.unpack(packed, want, 0, ds, count, levels)
        assert np.array_equal(db.download(np.uint8, dst.size), want)


@pytest.mark.parametrize("levels", [0, 1, 2, 4, 6])
def test_puts_gets_local(gpu_lib, oracle, levels):
    rng = np.random.default_rng(200 + levels)
    count, ss, ds = _random_patch(rng, levels, 1)
    count[0] += 3   # odd byte rows exercise the byte-wide copy
    src = rng.integers(0, 256, C.span(ss, count, levels)[1] + 8, dtype=np.uint8)
    dst = rng.integers(0, 256, C.span(ds, count, levels)[1] + 8, dtype=np.uint8)
    sb, db = ga_amd.DeviceBuffer(src.size), ga_amd.DeviceBuffer(dst.size)
    sb.upload(src)
    db.upload(dst)
    assert ga_amd.comex_puts(sb.ptr + 1, ss, db.ptr + 2, ds, count, levels, 0) == 0
    ga_amd.comex_fence_all()
    want = dst.copy()
    oracle.puts(src, 1, ss, want, 2, ds, count, levels)
    assert np.array_equal(db.download(np.uint8, dst.size), want)
    back = np.zeros_like(src)
    bb = ga_amd.DeviceBuffer(back.size)
    bb.upload(back)
    assert ga_amd.comex_gets(db.ptr + 2, ds, bb.ptr + 1, ss, count, levels, 0) == 0
    ga_amd.comex_fence_all()
    want_back = back.copy()
    oracle.puts(want, 2, ds, want_back, 1, ss, count, levels)
    assert np.array_equal(bb.download(np.uint8, back.size), want_back)


def test_host_memory_operands(gpu_lib, manifest, golden):
    """MA-style host buffers: pageable src + device dst, device src + pinned dst,
    pageable both (test.c:1028-1128 accumulates from a malloc'd local buffer)."""
    L = gpu_lib
    for case in [c for c in manifest["cases"] if not c.get("alias")][::5]:
        n, op = case["name"], case["op"]
        src, dst_in, want = golden[f"{n}/src"], golden[f"{n}/dst_in"], golden[f"{n}/dst_out"]
        keep, sp = ga_amd.scale_buffer(op, C.SCALE[op])
        ss, ds, cnt = (ga_amd.int_array(case["src_stride"]), ga_amd.int_array(case["dst_stride"]),
                       ga_amd.int_array(case["count"]))
        # pageable host src, device dst
        hsrc = src.copy()
        dbuf = ga_amd.DeviceBuffer(max(16, dst_in.size))
        dbuf.upload(dst_in)
        rc = L.comex_accs(op, sp, ctypes.c_void_p(hsrc.ctypes.data + case["src_off"]), ss,
                          ctypes.c_void_p(dbuf.ptr + case["dst_off"]), ds, cnt, case["levels"], 0, 0)
        assert rc == 0
        L.comex_fence_all(0)
        assert same_bits_nan_aware(dbuf.download(np.uint8, dst_in.size), want, op), ("host src", n)
        # pageable host src and pageable host dst
        hdst = dst_in.copy()
        rc = L.comex_accs(op, sp, ctypes.c_void_p(hsrc.ctypes.data + case["src_off"]), ss,
                          ctypes.c_void_p(hdst.ctypes.data + case["dst_off"]), ds, cnt, case["levels"], 0, 0)
        assert rc == 0
        L.comex_fence_all(0)
        assert same_bits_nan_aware(hdst, want, op), ("host both", n)
        # pinned (comex_malloc_local) dst, device src
        pin = L.comex_malloc_local(max(16, dst_in.size))
        ctypes.memmove(pin, dst_in.ctypes.data, dst_in.size)
        sbuf = ga_amd.DeviceBuffer(max(16, src.size))
        sbuf.upload(src)
        rc = L.comex_accs(op, sp, ctypes.c_void_p(sbuf.ptr + case["src_off"]), ss,
                          ctypes.c_void_p(pin + case["dst_off"]), ds, cnt, case["levels"], 0, 0)
        assert rc == 0
        L.comex_fence_all(0)
        got = np.ctypeslib.as_array((ctypes.c_uint8 * dst_in.size).from_address(pin)).copy()
        L.comex_free_local(ctypes.c_void_p(pin))
        assert same_bits_nan_aware(got, want, op), ("pinned dst", n)


@pytest.mark.parametrize("rows,row_el", [(7, 5), (40, 33), (300, 100)])
def test_pageable_sides_on_shared_pages(gpu_lib, oracle, rows, row_el):
    """Source and destination patches interleaved in ONE pageable buffer (their pages
    overlap): small spans go through the thread's pinned bounce buffer as one union, and
    only the destination's rows are written back -- every byte outside them, including
    the source rows and the gaps, is left as it was; above the bounce limit (the 300-row
    case, 240 KiB) the union is registered instead.  Also a put and a get between the
    two patches.  Exact against the oracle."""
    op, esz = C.DBL, 8
    row = row_el * esz
    ld = 2 * row + 24                      # src row, gap, dst row, gap
    buf = C.fill_bytes(op, rows * ld + 64, 77)
    so, do = 0, row + 8                    # dst rows start 8 bytes after each src row ends
    keep, sp = ga_amd.scale_buffer(op, C.SCALE[op])
    want = buf.copy()
    oracle.accs(op, C.SCALE[op], want, so, [ld], want, do, [ld], [row, rows], 1)
    got = buf.copy()
    assert gpu_lib.comex_accs(op, sp, ctypes.c_void_p(got.ctypes.data + so), ga_amd.int_array([ld]),
                              ctypes.c_void_p(got.ctypes.data + do), ga_amd.int_array([ld]),
                              ga_amd.int_array([row, rows]), 1, 0, 0) == 0
    ga_amd.comex_fence_all()
    assert np.array_equal(got, want), first_mismatch(got, want, op)
    # put: src rows -> dst rows (byte copy), then get them back into the src rows' place
    got2 = buf.copy()
    want2 = buf.copy()
    oracle.puts(want2, so, [ld], want2, do, [ld], [row - 3, rows], 1)
    assert ga_amd.comex_puts(got2.ctypes.data + so, [ld], got2.ctypes.data + do, [ld], [row - 3, rows], 1, 0) == 0
    ga_amd.comex_fence_all()
    assert np.array_equal(got2, want2)
    oracle.puts(want2, do + 5, [ld], want2, so + 1, [ld], [row - 9, rows], 1)
    assert ga_amd.comex_gets(got2.ctypes.data + do + 5, [ld], got2.ctypes.data + so + 1, [ld], [row - 9, rows], 1,
                             0) == 0
    ga_amd.comex_fence_all()
    assert np.array_equal(got2, want2)


def test_nb_pageable_sources_through_ring(gpu_lib, oracle):
    """Non-blocking accumulates and puts from ONE pageable buffer, refilled right after
    every call: a small source is copied into the thread's pinned ring and the call
    returns with its kernel queued (views.cpp ring_view), so each kernel must read the
    bytes of its own call.  About 10 MiB of sources in 4 MiB of ring (several laps and
    wrap gaps), destinations overlapping earlier calls (issue order), handles waited at
    random, sources above the ring's 64 KiB limit on the synchronous route.  Exact
    against the oracle applied in issue order."""
    op, esz = C.DBL, 8
    rng = np.random.default_rng(C.SEED + 901)
    D = 6 << 20
    dst0 = C.fill_bytes(op, D, 91)
    db = ga_amd.DeviceBuffer(D)
    db.upload(dst0)
    want = dst0.copy()
    src = np.zeros(200 << 10, dtype=np.uint8)          # pageable, reused by every call
    handles = []
    for k in range(320):
        big = k % 37 == 5
        row = int(rng.integers(1, 40 if not big else 200)) * esz
        rows = int(rng.integers(1, 24))
        ld = row + int(rng.integers(0, 6)) * esz
        span = (rows - 1) * ld + row
        if not big:
            while span > (64 << 10) - 512:
                rows = max(1, rows // 2)
                span = (rows - 1) * ld + row
        so = int(rng.integers(0, 32)) * esz
        src[:] = 0
        src[so:so + span] = C.fill_bytes(op, span, 1000 + k)
        dld = row + int(rng.integers(0, 9)) * esz
        dspan = (rows - 1) * dld + row
        do = int(rng.integers(0, (D - dspan) // esz)) * esz
        if k % 5 == 4:
            do = int(rng.integers(0, 4096)) * esz                        # a region many calls hit
        put = k % 7 == 3
        if put:
            oracle.puts(src, so, [ld], want, do, [dld], [row, rows], 1)
            h = ctypes.c_int(-1)
            rc = gpu_lib.comex_nbputs(ctypes.c_void_p(src.ctypes.data + so), ga_amd.int_array([ld]),
                                      ctypes.c_void_p(db.ptr + do), ga_amd.int_array([dld]),
                                      ga_amd.int_array([row, rows]), 1, 0, 0, ctypes.byref(h))
        else:
            oracle.accs(op, C.SCALE[op], src, so, [ld], want, do, [dld], [row, rows], 1)
            rc, h = ga_amd.comex_nbaccs(op, C.SCALE[op], src.ctypes.data + so, [ld], db.ptr + do, [dld],
                                        [row, rows], 1, 0)
        assert rc == 0
        src[:] = 0xAB                                     # the call's bytes are gone from the source
        handles.append(h)
        if rng.random() < 0.1 and handles:
            assert ga_amd.comex_wait(handles.pop(int(rng.integers(0, len(handles))))) == 0
    assert gpu_lib.comex_wait_all(0) == 0
    got = db.download(np.uint8, D)
    db.free()
    assert np.array_equal(got, want), first_mismatch(got, want, op)


@pytest.mark.parametrize("type_code,dtype", [(0, np.float64), (1, np.float32), (2, np.int32), (3, np.int64)])
def test_device_generator_matches_host(gpu_lib, type_code, dtype):
    n = 100003
    b = ga_amd.DeviceBuffer(n * np.dtype(dtype).itemsize)
    ga_amd.fill(b.ptr, n, type_code, C.SEED + 7)
    ga_amd.sync()
    assert np.array_equal(b.download(dtype, n), C.fill_real(dtype, n, C.SEED + 7))


def _fill_device(buf, op, nbytes, seed):
    rt = np.dtype(C.REAL[op])
    code = {np.dtype(np.float64): 0, np.dtype(np.float32): 1, np.dtype(np.int32): 2, np.dtype(np.int64): 3}[rt]
    ga_amd.fill(buf.ptr, nbytes // rt.itemsize, code, seed)
    tail = nbytes % rt.itemsize
    if tail:
        ga_amd.lib().gaamd_memset(ctypes.c_void_p(buf.ptr + nbytes - tail), 0, tail)


@pytest.mark.parametrize("idx", range(5))
def test_full_size_digest(gpu_lib, manifest, idx):
    """Full BASELINE sizes (C2, H ld 8192/8200, C3, C4): sha256 of the whole dst
    after one comex_accs equals the reference _acc's (oracle/_ref, manifest)."""
    cfg = manifest["full_size"][idx]
    op = cfg["op"]
    sb, db = ga_amd.DeviceBuffer(cfg["src_bytes"]), ga_amd.DeviceBuffer(cfg["dst_bytes"])
    _fill_device(sb, op, cfg["src_bytes"], C.SEED)
    _fill_device(db, op, cfg["dst_bytes"], C.SEED + 1)
    ga_amd.sync()
    assert hashlib.sha256(sb.download(np.uint8, cfg["src_bytes"]).tobytes()).hexdigest() == cfg["src_sha256"]
    rc = ga_amd.comex_accs(op, C.SCALE[op], sb.ptr, cfg["src_stride"], db.ptr, cfg["dst_stride"], cfg["count"],
                           cfg["levels"], 0)
    assert rc == 0
    ga_amd.comex_fence_all()
    got = hashlib.sha256(db.download(np.uint8, cfg["dst_bytes"]).tobytes()).hexdigest()
    assert got == cfg["dst_sha256"], cfg["name"]


def test_full_size_integer_roundtrip(gpu_lib):
    """Linearity at the headline shape in int64: acc(+a) then acc(-a) restores dst
    exactly (size-independent property; bit-exact integer path)."""
    count, stride = [2048 * 8, 4096], [8192 * 8]
    nbytes = stride[0] * 4095 + count[0]
    sb, db = ga_amd.DeviceBuffer(nbytes), ga_amd.DeviceBuffer(nbytes)
    _fill_device(sb, C.LNG, nbytes, 1)
    _fill_device(db, C.LNG, nbytes, 2)
    ga_amd.sync()
    before = hashlib.sha256(db.download(np.uint8, nbytes).tobytes()).hexdigest()
    assert ga_amd.comex_accs(C.LNG, 12345, sb.ptr, stride, db.ptr, stride, count, 1, 0) == 0
    mid = hashlib.sha256(db.download(np.uint8, nbytes).tobytes()).hexdigest()
    assert ga_amd.comex_accs(C.LNG, -12345, sb.ptr, stride, db.ptr, stride, count, 1, 0) == 0
    ga_amd.comex_fence_all()
    after = hashlib.sha256(db.download(np.uint8, nbytes).tobytes()).hexdigest()
    assert mid != before and after == before


def test_armci_contiguous_patch_over_2GiB(gpu_lib):
    """ARMCI_AccS on a contiguous patch of 2 GiB + 8 KiB: the reference's
    collapse to one comex_acc of (int)prod(count) bytes would wrap (armci.c:231-233,
    SURVEY appendix A.8); the library keeps the strided path.  int64 data, checked
    exactly on the first, middle and last rows against the oracle."""
    L = gpu_lib
    rows, row = 8193, 262144                  # 8193 * 256 KiB = 2 GiB + 256 KiB
    nbytes = rows * row
    sb, db = ga_amd.DeviceBuffer(nbytes), ga_amd.DeviceBuffer(nbytes)
    try:
        _fill_device(sb, C.LNG, nbytes, 3)
        _fill_device(db, C.LNG, nbytes, 4)
        ga_amd.sync()
        probe = [0, rows // 2, rows - 1]
        s_rows = {r: sb.download(np.int64, row // 8, r * row) for r in probe}
        d_rows = {r: db.download(np.int64, row // 8, r * row) for r in probe}
        keep, sp = ga_amd.scale_buffer(C.LNG, -5)
        rc = L.ARMCI_AccS(C.LNG, sp, ctypes.c_void_p(sb.ptr), ga_amd.int_array([row]), ctypes.c_void_p(db.ptr),
                          ga_amd.int_array([row]), ga_amd.int_array([row, rows]), 1, 0)
        assert rc == 0
        ga_amd.comex_fence_all()
        for r in probe:
            want = (d_rows[r].astype(np.uint64) + s_rows[r].astype(np.uint64) * np.uint64(2 ** 64 - 5)).view(np.int64)
            assert np.array_equal(db.download(np.int64, row // 8, r * row), want), r
    finally:
        sb.free()
        db.free()


def test_empty_patches_are_noops(gpu_lib):
    """count[j]=0 (j>=1) -> n1dim = 0 -> the reference loop runs zero times."""
    b = ga_amd.DeviceBuffer(64)
    b.upload(np.arange(8, dtype=np.float64))
    assert ga_amd.comex_accs(C.DBL, 2.0, b.ptr, [16], b.ptr + 32, [16], [16, 0], 1, 0) == 0
    ga_amd.comex_fence_all()
    assert np.array_equal(b.download(np.float64, 8), np.arange(8, dtype=np.float64))


@pytest.mark.parametrize("knobs", [{}, {"align": 0}, {"align": 1, "block": 128}, {"block": 64},
                                   {"streams": 1}, {"kind": 4}])
def test_wide_rows_odd_strides_all_knobs(gpu_lib, oracle, knobs):
    """Rows of 8-40 KiB (several chunks per row) at odd leading dimensions and
    offsets, so chunk splitting, the aligned-chunk grid and row tails are all
    exercised on the 2-D kernel; f64 and double complex, bit-exact vs oracle."""
    old = {k: ga_amd.set_tuning(k, v) for k, v in knobs.items()}
    try:
        rng = np.random.default_rng(42)
        for op in (C.DBL, C.DCP, C.FLT):
            esz = C.ESZ[op]
            for _ in range(3):
                w = int(rng.integers(1024, 5000)) * 8 // esz
                rows = int(rng.integers(3, 40))
                lds, ldd = w + int(rng.integers(0, 70)), w + int(rng.integers(0, 70))
                so, do = esz * int(rng.integers(0, 9)), esz * int(rng.integers(0, 9))
                count = [w * esz, rows]
                src = C.fill_bytes(op, so + lds * esz * rows, 11)
                dst = C.fill_bytes(op, do + ldd * esz * rows, 12)
                sb, db = ga_amd.DeviceBuffer(src.size), ga_amd.DeviceBuffer(dst.size)
                sb.upload(src)
                db.upload(dst)
                assert ga_amd.comex_accs(op, C.SCALE[op], sb.ptr + so, [lds * esz], db.ptr + do, [ldd * esz],
                                         count, 1, 0) == 0
                ga_amd.comex_fence_all()
                want = dst.copy()
                oracle.accs(op, C.SCALE[op], src, so, [lds * esz], want, do, [ldd * esz], count, 1)
                got = db.download(np.uint8, dst.size)
                assert np.array_equal(got, want), (op, w, rows, lds, ldd, so, do, knobs)
    finally:
        for k, v in old.items():
            ga_amd.set_tuning(k, v)


def test_whole_chunk_rows_every_op(gpu_lib, oracle):
    """Rows that are whole 4 KiB chunks (the loop-free kernels k_rows2d / k_rowsnd;
    4-D rows take k_rows), 1-D to 4-D, every op, odd leading dimensions and
    offsets (16-byte aligned), bit-exact vs the oracle."""
    rng = np.random.default_rng(7)
    for op in (C.INT, C.DBL, C.FLT, C.CPL, C.DCP, C.LNG):
        for levels in (0, 1, 2, 3):
            wbytes = 4096 * int(rng.integers(1, 4))
            count = [wbytes] + [int(rng.integers(2, 6)) for _ in range(levels)]
            st, dt = [], []
            sx, dx = wbytes, wbytes
            for j in range(levels):
                sx += 16 * int(rng.integers(0, 40))
                dx += 16 * int(rng.integers(0, 40))
                st.append(sx)
                dt.append(dx)
                sx *= count[j + 1]
                dx *= count[j + 1]
            so, do = 16 * int(rng.integers(0, 5)), 16 * int(rng.integers(0, 5))
            src = C.fill_bytes(op, so + C.span(st, count, levels)[1], 21)
            dst = C.fill_bytes(op, do + C.span(dt, count, levels)[1], 22)
            sb, db = ga_amd.DeviceBuffer(src.size), ga_amd.DeviceBuffer(dst.size)
            sb.upload(src)
            db.upload(dst)
            assert ga_amd.comex_accs(op, C.SCALE[op], sb.ptr + so, st, db.ptr + do, dt, count, levels, 0) == 0
            ga_amd.comex_fence_all()
            info = ga_amd.last_launch()
            assert info["kind"] == "rows" and info["width"] == 16, info
            want = dst.copy()
            oracle.accs(op, C.SCALE[op], src, so, st, want, do, dt, count, levels)
            got = db.download(np.uint8, dst.size)
            assert np.array_equal(got, want), (op, levels, count, st, dt, so, do)


@pytest.mark.parametrize("op,off", [(C.DCP, 8), (C.CPL, 4), (C.DBL, 4), (C.LNG, 4)])
def test_sub_natural_alignment(gpu_lib, oracle, op, off):
    """Elements below their natural alignment (a Fortran complex*16 array is only
    8-byte aligned): one element per dword-aligned vector, 1-D and 2-D, both sides
    misaligned, bit-exact vs the oracle."""
    esz = C.ESZ[op]
    for count, st in (([esz * 777], []), ([esz * 301, 9], [esz * 333 + 8])):
        levels = len(st)
        src = C.fill_bytes(op, 64 + C.span(st, count, levels)[1], 31)
        dst = C.fill_bytes(op, 64 + C.span(st, count, levels)[1], 32)
        sb, db = ga_amd.DeviceBuffer(src.size), ga_amd.DeviceBuffer(dst.size)
        sb.upload(src)
        db.upload(dst)
        assert ga_amd.comex_accs(op, C.SCALE[op], sb.ptr + off, st, db.ptr + 16 + off, st, count, levels, 0) == 0
        ga_amd.comex_fence_all()
        info = ga_amd.last_launch()
        assert info["width"] == esz, info
        want = dst.copy()
        oracle.accs(op, C.SCALE[op], src, off, st, want, 16 + off, st, count, levels)
        assert np.array_equal(db.download(np.uint8, dst.size), want), (op, off, count)


def test_stream_scheduler_random_dependencies(gpu_lib, oracle):
    """Random chains of accumulates and puts over a few buffers, with overlapping
    and disjoint ranges, issued back to back: independent ops may run on
    different streams (sched.cpp), dependent ones must keep program order.  The
    final buffers equal the oracle applying the same ops one by one (int64 data,
    exact)."""
    old_streams = ga_amd.set_tuning("streams", 3)
    assert gpu_lib.gaamd_num_streams() == 3
    try:
        _random_dependency_chain(oracle)
    finally:
        ga_amd.set_tuning("streams", old_streams)


def _random_dependency_chain(oracle):
    rng = np.random.default_rng(2024)
    nbuf, nbytes = 4, 8 << 20
    host = [C.fill_bytes(C.LNG, nbytes, 100 + i) for i in range(nbuf)]
    dev = [ga_amd.DeviceBuffer(nbytes) for _ in range(nbuf)]
    for h, d in zip(host, dev):
        d.upload(h)
    for it in range(160):
        op = C.LNG if rng.random() < 0.7 else 0
        w = int(rng.integers(1, 2048)) * 8
        rows = int(rng.integers(1, 64))
        ld_s = w + 8 * int(rng.integers(0, 64))
        ld_d = w + 8 * int(rng.integers(0, 64))
        bs, bd = int(rng.integers(0, nbuf)), int(rng.integers(0, nbuf))
        so = 8 * int(rng.integers(0, (nbytes - ld_s * rows) // 8))
        do = 8 * int(rng.integers(0, (nbytes - ld_d * rows) // 8))
        if bs == bd and rng.random() < 0.5:
            do = so   # same patch: in-place self-accumulate / copy
            ld_d = ld_s
        count = [w, rows]
        if op:
            a = int(rng.integers(-3, 4))
            assert ga_amd.comex_accs(op, a, dev[bs].ptr + so, [ld_s], dev[bd].ptr + do, [ld_d], count, 1, 0) == 0
            oracle.accs(op, a, host[bs], so, [ld_s], host[bd], do, [ld_d], count, 1)
        else:
            assert ga_amd.comex_puts(dev[bs].ptr + so, [ld_s], dev[bd].ptr + do, [ld_d], count, 1, 0) == 0
            if bs == bd:
                tmp = host[bs].copy()
                oracle.puts(tmp, so, [ld_s], host[bd], do, [ld_d], count, 1)
            else:
                oracle.puts(host[bs], so, [ld_s], host[bd], do, [ld_d], count, 1)
    ga_amd.comex_fence_all()
    for i in range(nbuf):
        assert np.array_equal(dev[i].download(np.uint8, nbytes), host[i]), f"buffer {i} diverged"


def _oracle_acc_pairs(oracle, op, scale, host_src, host_dst, pairs, nbytes):
    s = np.array([scale], dtype=C.REAL[op] if op not in (C.CPL, C.DCP) else
                 (np.complex64 if op == C.CPL else np.complex128))
    for so, do in pairs:
        oracle.L.ora_acc(op, nbytes, ctypes.c_void_p(host_dst.ctypes.data + do),
                         ctypes.c_void_p(host_src.ctypes.data + so), s.ctypes.data_as(ctypes.c_void_p))


@pytest.mark.parametrize("op,nbytes,dups", [(C.DBL, 8, False), (C.DBL, 8, True), (C.DCP, 16 * 5, False),
                                            (C.INT, 4 * 7, True), (C.FLT, 4 * 33, False), (C.LNG, 8 * 3, True)])
def test_accv_local(gpu_lib, oracle, op, nbytes, dups):
    """comex_accv (comex.c:7327-7400): n (src, dst) pairs in one descriptor through one
    io-vector kernel; duplicate destinations (GA scatter-acc) must apply in order."""
    rng = np.random.default_rng(nbytes + dups)
    esz = C.ESZ[op]
    nslots = 4000
    src = C.fill_bytes(op, nslots * nbytes, 1)
    dst = C.fill_bytes(op, nslots * nbytes, 2)
    sb, db = ga_amd.DeviceBuffer(src.size), ga_amd.DeviceBuffer(dst.size)
    sb.upload(src)
    db.upload(dst)
    n = 1500
    so = [int(x) * nbytes for x in rng.integers(0, nslots, n)]
    if dups:
        do = [int(x) * nbytes for x in rng.integers(0, 40, n)]      # many duplicates
    else:
        do = [int(x) * nbytes for x in rng.permutation(nslots)[:n]]
    descs = [([sb.ptr + a for a in so[:700]], [db.ptr + b for b in do[:700]], nbytes),
             ([sb.ptr + a for a in so[700:]], [db.ptr + b for b in do[700:]], nbytes)]
    assert ga_amd.comex_accv(op, C.SCALE[op], descs, 0) == 0
    ga_amd.comex_fence_all()
    want = dst.copy()
    _oracle_acc_pairs(oracle, op, C.SCALE[op], src, want, list(zip(so, do)), nbytes)
    got = db.download(np.uint8, dst.size)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("layout,n", [("src_seq", 6000), ("src_seq", 700), ("dst_seq", 6000), ("both_seq", 6000),
                                      ("chain", 3000), ("both_seq", 1)])
def test_accv_contiguous_sides(gpu_lib, oracle, layout, n):
    """A side that is one contiguous vector in pair order (pair i at base + i*bytes:
    GA's `v` of a scatter into one owner) is read as a packed side and its list is
    not uploaded; a contiguous destination side needs no repeat ordering. Same bits
    as the reference's per-pair loop (comex.c:7327-7400): src_seq with random,
    repeating destinations (6000 pairs: the GPU-ordered path), dst_seq with random
    sources, both, and a chain inside one buffer (pair i's source is pair i-1's
    destination: the in-order kernel must see each update)."""
    op, nbytes, nslots = C.DBL, 16, 8000
    rng = np.random.default_rng(31 + n + len(layout))
    src = C.fill_bytes(op, nslots * nbytes, 41)
    dst = C.fill_bytes(op, nslots * nbytes, 42)
    sb, db = ga_amd.DeviceBuffer(src.size), ga_amd.DeviceBuffer(dst.size)
    sb.upload(src)
    db.upload(dst)
    if layout == "chain":
        so = [i * nbytes for i in range(n)]
        do = [(i + 1) * nbytes for i in range(n)]
        descs = [([db.ptr + a for a in so], [db.ptr + b for b in do], nbytes)]
    else:
        so = ([int(x) * nbytes for x in rng.integers(0, nslots, n)] if layout == "dst_seq" else
              [(i + 7) * nbytes for i in range(n)])
        do = ([int(x) * nbytes for x in rng.integers(0, 60, n)] if layout == "src_seq" else
              [(i + 3) * nbytes for i in range(n)])
        descs = [([sb.ptr + a for a in so], [db.ptr + b for b in do], nbytes)]
    assert ga_amd.comex_accv(op, C.SCALE[op], descs, 0) == 0
    ga_amd.comex_fence_all()
    want = dst.copy()
    if layout == "chain":
        _oracle_acc_pairs(oracle, op, C.SCALE[op], want, want, list(zip(so, do)), nbytes)
    else:
        _oracle_acc_pairs(oracle, op, C.SCALE[op], src, want, list(zip(so, do)), nbytes)
    assert np.array_equal(db.download(np.uint8, dst.size), want)


@pytest.mark.parametrize("split", ["src", "dst", "both"])
def test_accv_sides_in_two_allocations(gpu_lib, oracle, split):
    """A descriptor of >= 1024 pairs whose sources (or destinations) lie in two
    separate HBM allocations: the one-allocation fast path (bounds of the first
    pair's allocations checked in the translate pass) must step aside for the
    per-address classification; same bits as the reference's loop."""
    op, nbytes, n, nslots = C.DBL, 8, 5000, 6000
    rng = np.random.default_rng(5 + len(split))
    src = [C.fill_bytes(op, nslots * nbytes, 11 + i) for i in range(2)]
    dst = [C.fill_bytes(op, nslots * nbytes, 21 + i) for i in range(2)]
    sb = [ga_amd.DeviceBuffer(x.size) for x in src]
    db = [ga_amd.DeviceBuffer(x.size) for x in dst]
    for b, x in zip(sb + db, src + dst):
        b.upload(x)
    # pair i: source slot in buffer sbuf[i], destination slot (distinct) in buffer dbuf[i]
    sbuf = (rng.random(n) < 0.5).astype(int) if split in ("src", "both") else np.zeros(n, int)
    dbuf = (rng.random(n) < 0.5).astype(int) if split in ("dst", "both") else np.zeros(n, int)
    sbuf[0] = dbuf[0] = 0                           # the first pair in buffer 0: the fast path tries first
    sbuf[-1] = 1 if split in ("src", "both") else 0
    dbuf[-1] = 1 if split in ("dst", "both") else 0
    so = rng.integers(0, nslots, n)
    do = np.concatenate([rng.permutation(nslots)[:n]])
    descs = [([sb[int(b)].ptr + int(a) * nbytes for a, b in zip(so, sbuf)],
              [db[int(b)].ptr + int(a) * nbytes for a, b in zip(do, dbuf)], nbytes)]
    assert ga_amd.comex_accv(op, C.SCALE[op], descs, 0) == 0
    ga_amd.comex_fence_all()
    want = [x.copy() for x in dst]
    for i in range(n):   # the reference's per-pair _acc, in order
        one_s = src[int(sbuf[i])][int(so[i]) * nbytes:(int(so[i]) + 1) * nbytes].copy()
        w = want[int(dbuf[i])]
        seg = w[int(do[i]) * nbytes:(int(do[i]) + 1) * nbytes].copy()
        _oracle_acc_pairs(oracle, op, C.SCALE[op], one_s, seg, [(0, 0)], nbytes)
        w[int(do[i]) * nbytes:(int(do[i]) + 1) * nbytes] = seg
    for b, w in zip(db, want):
        assert np.array_equal(b.download(np.uint8, w.size), w)


def test_putv_getv_local(gpu_lib):
    rng = np.random.default_rng(9)
    nbytes, n = 24, 900
    src = rng.integers(0, 256, 4000 * nbytes, dtype=np.uint8)
    sb, db = ga_amd.DeviceBuffer(src.size), ga_amd.DeviceBuffer(src.size)
    sb.upload(src)
    db.upload(np.zeros_like(src))
    perm = rng.permutation(4000)[:n]
    descs = [([sb.ptr + i * nbytes for i in range(n)], [db.ptr + int(p) * nbytes for p in perm], nbytes)]
    assert ga_amd.comex_putv(descs, 0) == 0
    ga_amd.comex_fence_all()
    got = db.download(np.uint8, src.size).reshape(4000, nbytes)
    assert np.array_equal(got[perm], src.reshape(4000, nbytes)[:n])
    back = ga_amd.DeviceBuffer(n * nbytes)
    descs = [([db.ptr + int(p) * nbytes for p in perm], [back.ptr + i * nbytes for i in range(n)], nbytes)]
    assert ga_amd.comex_getv(descs, 0) == 0
    ga_amd.comex_fence_all()
    assert np.array_equal(back.download(np.uint8, n * nbytes), src[: n * nbytes])


def test_accv_host_source_pairs(gpu_lib, oracle):
    """Pageable host sources (MA buffers) fall back to per-pair transfers; same bits."""
    op, nbytes, n = C.DBL, 16, 50
    src = C.fill_bytes(op, n * nbytes, 3)
    dst = C.fill_bytes(op, n * nbytes, 4)
    db = ga_amd.DeviceBuffer(dst.size)
    db.upload(dst)
    descs = [([src.ctypes.data + i * nbytes for i in range(n)], [db.ptr + (n - 1 - i) * nbytes for i in range(n)],
              nbytes)]
    assert ga_amd.comex_accv(op, C.SCALE[op], descs, 0) == 0
    ga_amd.comex_fence_all()
    want = dst.copy()
    _oracle_acc_pairs(oracle, op, C.SCALE[op], src, want, [(i * nbytes, (n - 1 - i) * nbytes) for i in range(n)],
                      nbytes)
    assert np.array_equal(db.download(np.uint8, dst.size), want)


def _giov_np(src_addrs, dst_addrs, nbytes):
    """one comex_giov_t over numpy uint64 address arrays (large n without Python lists);
    the arrays stay referenced by the returned descriptor."""
    src_addrs = np.ascontiguousarray(src_addrs, dtype=np.uint64)
    dst_addrs = np.ascontiguousarray(dst_addrs, dtype=np.uint64)
    g = ga_amd.GIOV()
    g._keep = (src_addrs, dst_addrs)
    g.src = ctypes.cast(ctypes.c_void_p(src_addrs.ctypes.data), ctypes.POINTER(ctypes.c_void_p))
    g.dst = ctypes.cast(ctypes.c_void_p(dst_addrs.ctypes.data), ctypes.POINTER(ctypes.c_void_p))
    g.count, g.bytes = len(src_addrs), nbytes
    return g


@pytest.mark.parametrize("op,nbytes,slots,shift", [(C.DBL, 8, 3000, 0), (C.DBL, 8, 10 ** 6, 0), (C.FLT, 4, 500, 0),
                                                   (C.DCP, 16, 2000, 0), (C.INT, 12, 700, 0), (C.LNG, 8, 100, 0),
                                                   (C.CPL, 8 * 3, 5000, 0), (C.DBL, 48, 4000, 0),
                                                   (C.DBL, 320, 300, 0), (C.DBL, 16, 3000, 8)])
def test_accv_large_repeated_destinations(gpu_lib, oracle, op, nbytes, slots, shift):
    """GA scatter-acc sizes: 40 000 pairs in one descriptor, destinations drawn from
    `slots` (many repeats), bit-exact against the pairs applied one by one in order.
    The GPU orders repeated destinations and applies each destination's pairs in input
    order: the partitioned LDS path (round 6), and the hashed path (+ the radix path
    for heavy repeats) with tuning iov_lds=0; 320-byte pairs and destinations not
    congruent modulo the pair size (`shift`: some start half a pair later) take the
    host-checked path instead."""
    rng = np.random.default_rng(nbytes * 7 + slots)
    n = 40000
    src = C.fill_bytes(op, n * nbytes, 5)
    dst = C.fill_bytes(op, slots * nbytes + 64, 6)
    sb, db = ga_amd.DeviceBuffer(src.size), ga_amd.DeviceBuffer(dst.size)
    sb.upload(src)
    db.upload(dst)
    so = np.arange(n, dtype=np.uint64) * nbytes
    do = rng.integers(0, slots, n).astype(np.uint64) * nbytes
    if shift:
        do[rng.random(n) < 0.01] += shift
    g = _giov_np(so + np.uint64(sb.ptr), do + np.uint64(db.ptr), nbytes)
    keep, sp = ga_amd.scale_buffer(op, C.SCALE[op])
    paths0 = ga_amd.iov_path_counts()
    assert gpu_lib.comex_accv(op, sp, ctypes.byref(g), 1, 0, 0) == 0
    ga_amd.comex_fence_all()
    paths1 = ga_amd.iov_path_counts()
    want = dst.copy()
    _oracle_acc_pairs(oracle, op, C.SCALE[op], src, want, list(zip(so.tolist(), do.tolist())), nbytes)
    got = db.download(np.uint8, dst.size)
    assert same_bits_nan_aware(got, want, op)
    if nbytes <= 256 and not shift:
        # up to 64 Ki pairs the partitioned LDS path orders them (round 6); the hashed
        # path (and the radix path for what it leaves) with iov_lds=0, below
        assert paths1["lds"] == paths0["lds"] + 1, (paths0, paths1)
        old = ga_amd.set_tuning("iov_lds", 0)
        try:
            db.upload(dst)
            assert gpu_lib.comex_accv(op, sp, ctypes.byref(g), 1, 0, 0) == 0
            ga_amd.comex_fence_all()
        finally:
            ga_amd.set_tuning("iov_lds", old)
        assert same_bits_nan_aware(db.download(np.uint8, dst.size), want, op)
        paths2 = ga_amd.iov_path_counts()
        conflicting = n - int(np.sum(np.unique(do, return_counts=True)[1] == 1))
        key = "hashed" if conflicting <= 8192 else "hashed_then_radix"
        assert paths2[key] == paths1[key] + 1, (conflicting, paths1, paths2)


PART_MAX = 1 << 22   # kIovPartMax (gaamd_kernels.h): the partitioned LDS path's largest call


@pytest.mark.parametrize("op,nbytes,slots,n", [(C.DBL, 8, 150000, 600037), (C.FLT, 4, 900, 530001),
                                               (C.LNG, 8, 70000, 4 * 2 ** 18 + 5)])
def test_accv_radix_path(gpu_lib, oracle, op, nbytes, slots, n):
    """Above 2^19 pairs the hashed path is skipped: with tuning iov_lds=0 (and by default
    above PART_MAX pairs, where the partitioned LDS path stops) every destination is sorted on
    the GPU by the library's own stable LSD radix sort (k_rs_*; 8-bit digits, 2 passes at
    900 slots, 3 at 70 000 and 150 000; ragged last tile) and each destination's pairs
    applied in input order -- bit-exact against the pairs applied one by one; by default,
    up to PART_MAX pairs, the partitioned path gives the same bytes."""
    rng = np.random.default_rng(n)
    src = C.fill_bytes(op, n * nbytes, 11)
    dst = C.fill_bytes(op, slots * nbytes, 12)
    sb, db = ga_amd.DeviceBuffer(src.size), ga_amd.DeviceBuffer(dst.size)
    sb.upload(src)
    so = np.arange(n, dtype=np.uint64) * nbytes
    do = rng.integers(0, slots, n).astype(np.uint64) * nbytes
    g = _giov_np(so + np.uint64(sb.ptr), do + np.uint64(db.ptr), nbytes)
    keep, sp = ga_amd.scale_buffer(op, C.SCALE[op])
    want = dst.copy()
    _oracle_acc_pairs(oracle, op, C.SCALE[op], src, want, zip(so.tolist(), do.tolist()), nbytes)
    for lds in (0, 1):
        db.upload(dst)
        old = ga_amd.set_tuning("iov_lds", lds)
        try:
            paths0 = ga_amd.iov_path_counts()
            assert gpu_lib.comex_accv(op, sp, ctypes.byref(g), 1, 0, 0) == 0
            ga_amd.comex_fence_all()
            paths1 = ga_amd.iov_path_counts()
        finally:
            ga_amd.set_tuning("iov_lds", old)
        key = "lds" if lds and n <= PART_MAX else "radix"
        assert paths1[key] == paths0[key] + 1, (lds, paths0, paths1)
        got = db.download(np.uint8, dst.size)
        assert same_bits_nan_aware(got, want, op), f"iov_lds={lds}"


@pytest.mark.parametrize("n", [50, 20000, 200000])
def test_accv_host_sources_packed(gpu_lib, oracle, n):
    """Pageable host sources (GA's MA buffer `v` of NGA_Scatter_acc) are gathered on the
    host and uploaded packed (one kernel, not one transfer per pair); repeated
    destinations still apply in order. From 65 536 pairs a source side lying in one
    host mapping is recognised with one /proc/self/maps lookup (host_cpu_range)."""
    op, nbytes = C.DBL, 8
    rng = np.random.default_rng(n)
    src = C.fill_bytes(op, n * nbytes, 3)
    dst = C.fill_bytes(op, 1000 * nbytes, 4)
    db = ga_amd.DeviceBuffer(dst.size)
    db.upload(dst)
    so = np.arange(n, dtype=np.uint64) * nbytes
    do = rng.integers(0, 1000, n).astype(np.uint64) * nbytes
    g = _giov_np(so + np.uint64(src.ctypes.data), do + np.uint64(db.ptr), nbytes)
    keep, sp = ga_amd.scale_buffer(op, C.SCALE[op])
    assert gpu_lib.comex_accv(op, sp, ctypes.byref(g), 1, 0, 0) == 0
    ga_amd.comex_fence_all()
    want = dst.copy()
    _oracle_acc_pairs(oracle, op, C.SCALE[op], src, want, list(zip(so.tolist(), do.tolist())), nbytes)
    assert np.array_equal(db.download(np.uint8, dst.size), want)


@pytest.mark.parametrize("n", [30000, 100000])
def test_getv_putv_host_side_packed(gpu_lib, n):
    """comex_getv into pageable host memory (results packed on the GPU, scattered on
    the host in pair order: a repeated destination keeps the last pair's bytes) and
    comex_putv from pageable host memory, n pairs of 24 bytes (100 000: the whole-side
    host test of the local fast path)."""
    rng = np.random.default_rng(11)
    nbytes, slots = 24, 5000
    dev = rng.integers(0, 256, slots * nbytes, dtype=np.uint8)
    db = ga_amd.DeviceBuffer(dev.size)
    db.upload(dev)
    so = rng.integers(0, slots, n).astype(np.uint64) * nbytes
    host = np.zeros(2000 * nbytes, dtype=np.uint8)
    do = rng.integers(0, 2000, n).astype(np.uint64) * nbytes
    g = _giov_np(so + np.uint64(db.ptr), do + np.uint64(host.ctypes.data), nbytes)
    assert gpu_lib.comex_getv(ctypes.byref(g), 1, 0, 0) == 0
    want = np.zeros_like(host)
    for a, b in zip(so.tolist(), do.tolist()):
        want[b:b + nbytes] = dev[a:a + nbytes]
    assert np.array_equal(host, want)
    # putv from host: repeated destinations, last pair wins
    src = rng.integers(0, 256, n * nbytes, dtype=np.uint8)
    s_off = np.arange(n, dtype=np.uint64) * nbytes
    d_off = rng.integers(0, slots, n).astype(np.uint64) * nbytes
    g = _giov_np(s_off + np.uint64(src.ctypes.data), d_off + np.uint64(db.ptr), nbytes)
    assert gpu_lib.comex_putv(ctypes.byref(g), 1, 0, 0) == 0
    ga_amd.comex_fence_all()
    want = dev.copy()
    for a, b in zip(s_off.tolist(), d_off.tolist()):
        want[b:b + nbytes] = src[a:a + nbytes]
    assert np.array_equal(db.download(np.uint8, dev.size), want)


def test_accv_host_sources_in_two_buffers(gpu_lib, oracle):
    """Host sources alternating between two separate pageable buffers: the span of the
    source side is not one mapping (or is, if the allocator placed them adjacently);
    either way the result equals the pairs applied in order."""
    op, nbytes, n = C.DBL, 8, 70000
    rng = np.random.default_rng(5)
    a = C.fill_bytes(op, n * nbytes, 7)
    b = C.fill_bytes(op, n * nbytes, 8)
    dst = C.fill_bytes(op, 3000 * nbytes, 9)
    db = ga_amd.DeviceBuffer(dst.size)
    db.upload(dst)
    idx = np.arange(n, dtype=np.uint64) * nbytes
    pick = rng.random(n) < 0.5
    sa = np.where(pick, idx + np.uint64(a.ctypes.data), idx + np.uint64(b.ctypes.data)).astype(np.uint64)
    do = rng.integers(0, 3000, n).astype(np.uint64) * nbytes
    g = _giov_np(sa, do + np.uint64(db.ptr), nbytes)
    keep, sp = ga_amd.scale_buffer(op, C.SCALE[op])
    assert gpu_lib.comex_accv(op, sp, ctypes.byref(g), 1, 0, 0) == 0
    ga_amd.comex_fence_all()
    both = np.concatenate([a, b])
    so = np.where(pick, idx, idx + np.uint64(a.size)).astype(np.uint64)
    want = dst.copy()
    _oracle_acc_pairs(oracle, op, C.SCALE[op], both, want, list(zip(so.tolist(), do.tolist())), nbytes)
    assert np.array_equal(db.download(np.uint8, dst.size), want)


def _maps_lines_covering(lo, hi):
    """the /proc/self/maps lines that overlap [lo, hi)"""
    out = []
    with open("/proc/self/maps") as f:
        for line in f:
            a, b = (int(x, 16) for x in line.split()[0].split("-"))
            if a < hi and b > lo:
                out.append(line.strip())
    return out


def test_accv_host_source_over_split_mappings(gpu_lib, oracle):
    """A pageable source buffer the kernel keeps as several adjacent mappings (numpy
    advises huge pages on the 2 MiB-aligned part of arrays from 4 MiB up; here
    madvise(MADV_DONTFORK) on the middle splits one anonymous mapping in three) is
    still recognised as one host side by the /proc/self/maps pass (one lookup, not a
    device-view query per page: the 1 Mi-element scatter went 10 ms -> 1.5 ms,
    profiles/r05/scatter), and the result equals the pairs applied in order."""
    op, nbytes, n = C.DBL, 8, 200000
    size = 4 << 20
    libc = ctypes.CDLL(None, use_errno=True)
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
    libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    base = libc.mmap(None, size, 3, 0x22, -1, 0)   # PROT_READ|PROT_WRITE, MAP_PRIVATE|MAP_ANONYMOUS
    assert base not in (None, ctypes.c_void_p(-1).value)
    assert libc.madvise(ctypes.c_void_p(base + (1 << 20)), 1 << 20, 10) == 0, ctypes.get_errno()   # MADV_DONTFORK
    assert len(_maps_lines_covering(base, base + n * nbytes)) >= 2
    src = C.fill_bytes(op, n * nbytes, 12)
    ctypes.memmove(base, src.ctypes.data, src.size)
    rng = np.random.default_rng(12)
    dst = C.fill_bytes(op, 4000 * nbytes, 13)
    db = ga_amd.DeviceBuffer(dst.size)
    db.upload(dst)
    so = np.arange(n, dtype=np.uint64) * nbytes
    do = rng.integers(0, 4000, n).astype(np.uint64) * nbytes
    g = _giov_np(so + np.uint64(base), do + np.uint64(db.ptr), nbytes)
    keep, sp = ga_amd.scale_buffer(op, C.SCALE[op])
    c0 = (ctypes.c_ulonglong * 1)()
    assert gpu_lib.gaamd_diag(b"iov_host_sides", 0, c0, 1) == 0
    assert gpu_lib.comex_accv(op, sp, ctypes.byref(g), 1, 0, 0) == 0
    ga_amd.comex_fence_all()
    c1 = (ctypes.c_ulonglong * 1)()
    assert gpu_lib.gaamd_diag(b"iov_host_sides", 0, c1, 1) == 0
    assert c1[0] == c0[0] + 1, (c0[0], c1[0])
    want = dst.copy()
    _oracle_acc_pairs(oracle, op, C.SCALE[op], src, want, list(zip(so.tolist(), do.tolist())), nbytes)
    assert np.array_equal(db.download(np.uint8, dst.size), want)
    del g
    assert libc.munmap(ctypes.c_void_p(base), size) == 0


@pytest.mark.parametrize("op,nbytes,slots,n,src", [
    (C.DBL, 8, 10 ** 6, 16384, "seq"), (C.DBL, 8, 3000, 16384, "perm"), (C.FLT, 4, 100, 16384, "seq"),
    (C.DCP, 16, 2000, 8192, "perm"), (C.INT, 12, 700, 4096, "seq"), (C.LNG, 8, 50, 2048, "perm"),
    (C.CPL, 24, 5000, 12000, "seq"), (C.DBL, 256, 300, 3000, "perm"), (C.DBL, 8, 1, 4095, "seq"),
    (C.DBL, 8, 1, 4096, "seq"), (C.DBL, 8, 200, 1000, "host"), (C.FLT, 4, 1 << 20, 16384, "host"),
    (C.LNG, 8, 3, 64, "perm"), (C.INT, 4, 1 << 20, 3000, "perm"), (C.DCP, 16, 1 << 20, 9000, "perm"),
    (C.DBL, 8, 10 ** 6, 65536, "seq"), (C.FLT, 4, 7, 30000, "perm"), (C.CPL, 8, 40000, 50000, "host")])
def test_accv_one_workgroup_path(gpu_lib, oracle, op, nbytes, slots, n, src):
    """io-vectors of up to 64 Ki pairs whose destinations may repeat are
    ordered in LDS: below 1 Ki pairs ONE launch of one 1024-thread workgroup (k_iov_lds:
    keys and a hash table in LDS, repeated pairs sorted by (destination, index), applied
    in input order); from 1 Ki pairs the keys into hash-partition buckets, then one
    workgroup per partition finds its repeated keys in an LDS table, sorts only those and
    applies them (k_iov_keyof + k_iov_part; a skewed partition -- 7 destinations for
    30 000 pairs -- in windows of the input).  Sources contiguous (GA's
    `v`), permuted, or gathered from pageable host memory; from one destination for
    every pair to nearly all distinct; bit-exact against the pairs applied one by one,
    and the same bytes as the hashed three-launch path (tuning iov_lds=0)."""
    rng = np.random.default_rng(n * 31 + slots)
    srcb = C.fill_bytes(op, n * nbytes, 21)
    dst = C.fill_bytes(op, slots * nbytes, 22)
    db = ga_amd.DeviceBuffer(dst.size)
    if src == "host":
        sbase, sb = srcb.ctypes.data, None
    else:
        sb = ga_amd.DeviceBuffer(srcb.size)
        sb.upload(srcb)
        sbase = sb.ptr
    so = (rng.permutation(n) if src == "perm" else np.arange(n)).astype(np.uint64) * nbytes
    do = rng.integers(0, slots, n).astype(np.uint64) * nbytes
    g = _giov_np(so + np.uint64(sbase), do + np.uint64(db.ptr), nbytes)
    keep, sp = ga_amd.scale_buffer(op, C.SCALE[op])
    want = dst.copy()
    _oracle_acc_pairs(oracle, op, C.SCALE[op], srcb, want, list(zip(so.tolist(), do.tolist())), nbytes)
    outs = []
    for lds in (1, 0):
        old = ga_amd.set_tuning("iov_lds", lds)
        try:
            db.upload(dst)
            paths0 = ga_amd.iov_path_counts()
            assert gpu_lib.comex_accv(op, sp, ctypes.byref(g), 1, 0, 0) == 0
            ga_amd.comex_fence_all()
            paths1 = ga_amd.iov_path_counts()
        finally:
            ga_amd.set_tuning("iov_lds", old)
        assert (paths1["lds"] - paths0["lds"]) == lds, (lds, n, paths0, paths1)
        got = db.download(np.uint8, dst.size)
        assert same_bits_nan_aware(got, want, op), f"iov_lds={lds}"
        outs.append(got)
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.parametrize("op,nbytes,slots,n,deferred", [
    (C.DBL, 8, 200, 300000, True), (C.DBL, 8, 10 ** 7, 300000, False), (C.DCP, 16, 50, 150000, True),
    (C.FLT, 4, 3000, 1 << 20, None), (C.INT, 12, 2, 70000, True)])
def test_accv_partitions_large(gpu_lib, oracle, op, nbytes, slots, n, deferred):
    """The partitioned path above kIovPartWindowMax (64 Ki) pairs: a partition holding more
    pairs than its bucket (heavy repeats -- 200 destinations for 300 000 pairs) is left to
    the radix path, masked, once the stream has completed (path counters "lds" and
    "radix" both advance); random destinations never defer.  Bit-exact against the pairs
    applied one by one in input order (comex.c:7342-7351)."""
    rng = np.random.default_rng(n + slots)
    srcb = C.fill_bytes(op, n * nbytes, 31)
    dst = C.fill_bytes(op, slots * nbytes, 32) if slots <= 10 ** 6 else None
    span = slots if dst is not None else n * 4
    if dst is None:
        dst = C.fill_bytes(op, span * nbytes, 32)
    sb = ga_amd.DeviceBuffer(srcb.size)
    sb.upload(srcb)
    db = ga_amd.DeviceBuffer(dst.size)
    db.upload(dst)
    so = np.arange(n, dtype=np.uint64) * nbytes
    do = rng.integers(0, span, n).astype(np.uint64) * nbytes
    g = _giov_np(so + np.uint64(sb.ptr), do + np.uint64(db.ptr), nbytes)
    keep, sp = ga_amd.scale_buffer(op, C.SCALE[op])
    want = dst.copy()
    _oracle_acc_pairs(oracle, op, C.SCALE[op], srcb, want, list(zip(so.tolist(), do.tolist())), nbytes)
    p0 = ga_amd.iov_path_counts()
    assert gpu_lib.comex_accv(op, sp, ctypes.byref(g), 1, 0, 0) == 0
    ga_amd.comex_fence_all()
    p1 = ga_amd.iov_path_counts()
    assert p1["lds"] == p0["lds"] + 1, (p0, p1)
    if deferred is not None:
        assert p1["radix"] == p0["radix"] + int(deferred), (p0, p1)
    assert same_bits_nan_aware(db.download(np.uint8, dst.size), want, op)
    # the counters are zero again: a second call on the same destinations
    want2 = want.copy()
    _oracle_acc_pairs(oracle, op, C.SCALE[op], srcb, want2, list(zip(so.tolist(), do.tolist())), nbytes)
    assert gpu_lib.comex_accv(op, sp, ctypes.byref(g), 1, 0, 0) == 0
    ga_amd.comex_fence_all()
    assert same_bits_nan_aware(db.download(np.uint8, dst.size), want2, op)
