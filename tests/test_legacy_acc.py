"""The legacy ARMCI accumulate path: armci/src/xfer/
caccumulate.c's c_?_accumulate_{1d,2d,2d_u}_ loops and armci_acc_2D
(armci/src/xfer/strided.c:257-328).

CPU: the oracle's restatement (oracle/comex_oracle.c ora_legacy_acc_2d) is
pinned bit for bit against the reference's own loops compiled from
/root/reference (oracle/_ref/libref_legacy_acc.so), and shown equal to comex's
_acc on the same patch (the complex products commute).
GPU: the library's entry points (include/armci_acc.h) on HBM and on host
memory, bit-exact against the reference's loops (or the pinned restatement
where _ref is absent)."""
import ctypes

import numpy as np
import pytest

from oracle import LegacyRef, Oracle, legacy_ref_available

INT, DBL, FLT, CPL, DCP, LNG = 37, 38, 39, 40, 41, 42
DT = {INT: np.int32, DBL: np.float64, FLT: np.float32, CPL: np.complex64, DCP: np.complex128, LNG: np.int64}
ALPHA = {INT: 3, DBL: 1.5, FLT: -0.75, CPL: 0.5 - 1.25j, DCP: -2.0 + 0.375j, LNG: -7}


def rand(op, n, rng):
    dt = np.dtype(DT[op])
    if dt.kind == "i":
        return rng.integers(-2 ** 20, 2 ** 20, n).astype(dt)
    if dt.kind == "c":
        return (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(dt)
    return rng.standard_normal(n).astype(dt)


def shapes(rng, k=12):
    out = [(1, 1, 1, 1), (5, 3, 5, 7), (4, 4, 9, 4), (17, 1, 20, 17), (0, 5, 3, 3), (6, 0, 6, 6)]
    for _ in range(k):
        rows, cols = int(rng.integers(1, 40)), int(rng.integers(1, 12))
        out.append((rows, cols, rows + int(rng.integers(0, 9)), rows + int(rng.integers(0, 9))))
    return out


@pytest.mark.skipif(not legacy_ref_available(), reason="oracle/_ref/libref_legacy_acc.so not built")
@pytest.mark.parametrize("op", [INT, DBL, FLT, CPL, DCP, LNG])
def test_restatement_matches_reference_loops(op):
    ora, ref = Oracle(), LegacyRef()
    rng = np.random.default_rng(op)
    for rows, cols, ald, bld in shapes(rng):
        A0 = rand(op, max(1, ald * cols), rng)
        B = rand(op, max(1, bld * cols), rng)
        want = A0.copy()
        ref.acc_2d(op, ALPHA[op], rows, cols, want, ald, B, bld)
        got = A0.copy()
        ora.legacy_acc_2d(op, ALPHA[op], rows, cols, got, ald, B, bld)
        assert got.tobytes() == want.tobytes(), (rows, cols, ald, bld)
        unrolled = A0.copy()
        ref.acc_2d(op, ALPHA[op], rows, cols, unrolled, ald, B, bld, unrolled=True)
        assert unrolled.tobytes() == want.tobytes(), ("_u", rows, cols, ald, bld)
    if op == LNG:   # c_ll_ (long long) is the same loop on 8-byte integers
        A0, B = rand(op, 60, rng), rand(op, 60, rng)
        a, b = A0.copy(), A0.copy()
        ref.acc_2d(op, ALPHA[op], 5, 6, a, 10, B, 10, name="ll")
        ora.legacy_acc_2d(op, ALPHA[op], 5, 6, b, 10, B, 10)
        assert a.tobytes() == b.tobytes()


@pytest.mark.parametrize("op", [INT, DBL, FLT, CPL, DCP, LNG])
def test_legacy_equals_comex_acc(op):
    """caccumulate.c's complex form alpha.i*B.r + alpha.r*B.i is comex acc.h's
    B.r*alpha.i + B.i*alpha.r with the products commuted: one kernel serves both."""
    ora = Oracle()
    rng = np.random.default_rng(100 + op)
    esz = np.dtype(DT[op]).itemsize
    for rows, cols, ald, bld in shapes(rng):
        if rows == 0 or cols == 0:
            continue
        A0, B = rand(op, ald * cols, rng), rand(op, bld * cols, rng)
        a = A0.copy()
        ora.legacy_acc_2d(op, ALPHA[op], rows, cols, a, ald, B, bld)
        c = A0.copy()
        ora.accs(op, ALPHA[op], B.view(np.uint8), 0, [bld * esz], c.view(np.uint8), 0, [ald * esz],
                 [rows * esz, cols], 1)
        assert a.tobytes() == c.tobytes()


def test_acc_2D_truncates_byte_strides():
    """strided.c:262-298: bytes and strides become elements by integer division."""
    ora = Oracle()
    rng = np.random.default_rng(7)
    A0, B = rand(DBL, 400, rng), rand(DBL, 400, rng)
    got = A0.copy()
    ora.legacy_acc_2D(DBL, 2.0, B, got, 8 * 5 + 3, 6, 8 * 9 + 7, 8 * 11 + 1)   # 5 rows, lds 9, ldd 11
    want = A0.copy()
    ora.legacy_acc_2d(DBL, 2.0, 5, 6, want, 11, B, 9)
    assert got.tobytes() == want.tobytes()


# ---------------------------------------------------------------- GPU
def _lib():
    import ga_amd
    L = ga_amd.lib()
    assert L.comex_init() == 0
    return ga_amd, L


def _call_2d(L, op, alpha, rows, cols, A_ptr, ald, B_ptr, bld, unrolled=False, name=None):
    import ga_amd
    a, ap = ga_amd.scale_buffer(op, alpha)
    t = name or {DBL: "d", FLT: "f", CPL: "c", DCP: "z", INT: "i", LNG: "l"}[op]
    fn = getattr(L, f"c_{t}_accumulate_2d{'_u' if unrolled else ''}_")
    ip = lambda v: ctypes.byref(ctypes.c_int(v))   # noqa: E731
    fn(ap, ip(rows), ip(cols), ctypes.c_void_p(A_ptr), ip(ald), ctypes.c_void_p(B_ptr), ip(bld))


def _expected(op, alpha, rows, cols, A0, ald, B, bld, name=None):
    want = A0.copy()
    if legacy_ref_available():
        LegacyRef().acc_2d(op, alpha, rows, cols, want, ald, B, bld, name=name)
    else:
        Oracle().legacy_acc_2d(op, alpha, rows, cols, want, ald, B, bld)
    return want


@pytest.mark.gpu
@pytest.mark.parametrize("op", [INT, DBL, FLT, CPL, DCP, LNG])
@pytest.mark.parametrize("where", ["hbm", "host"])
def test_gpu_legacy_acc_2d(op, where):
    ga_amd, L = _lib()
    rng = np.random.default_rng(1000 + op)
    esz = np.dtype(DT[op]).itemsize
    cases = shapes(rng, 8) + [(2048, 512, 2056, 2048)]
    for k, (rows, cols, ald, bld) in enumerate(cases):
        A0, B = rand(op, max(1, ald * cols), rng), rand(op, max(1, bld * cols), rng)
        want = _expected(op, ALPHA[op], rows, cols, A0, ald, B, bld)
        if where == "hbm":
            da, db = ga_amd.DeviceBuffer(A0.nbytes), ga_amd.DeviceBuffer(B.nbytes)
            da.upload(A0)
            db.upload(B)
            _call_2d(L, op, ALPHA[op], rows, cols, da.ptr, ald, db.ptr, bld, unrolled=bool(k % 2))
            got = da.download(DT[op], A0.size)
            da.free()
            db.free()
        else:
            got = A0.copy()
            _call_2d(L, op, ALPHA[op], rows, cols, got.ctypes.data, ald, B.ctypes.data, bld, unrolled=bool(k % 2))
        assert got.tobytes() == want.tobytes(), (where, rows, cols, ald, bld)
    assert esz > 0


@pytest.mark.gpu
def test_gpu_legacy_1d_ll_and_acc_2D():
    ga_amd, L = _lib()
    rng = np.random.default_rng(3)
    # 1-D forms on host memory
    for op, t in ((DBL, "d"), (FLT, "f"), (CPL, "c"), (DCP, "z"), (INT, "i"), (LNG, "l"), (LNG, "ll")):
        A0, B = rand(op, 1000, rng), rand(op, 1000, rng)
        got = A0.copy()
        a, ap = ga_amd.scale_buffer(op, ALPHA[op])
        getattr(L, f"c_{t}_accumulate_1d_")(ap, ctypes.c_void_p(got.ctypes.data), ctypes.c_void_p(B.ctypes.data),
                                            ctypes.byref(ctypes.c_int(999)))
        want = _expected(op, ALPHA[op], 999, 1, A0, 999, B, 999, name=t)
        assert got.tobytes() == want.tobytes(), t
    # c_ll_accumulate_2d_ and armci_acc_2D with strides that are not element multiples
    A0, B = rand(LNG, 600, rng), rand(LNG, 600, rng)
    got = A0.copy()
    _call_2d(L, LNG, -7, 9, 20, got.ctypes.data, 25, B.ctypes.data, 30, name="ll")
    assert got.tobytes() == _expected(LNG, -7, 9, 20, A0, 25, B, 30, name="ll").tobytes()
    A0, B = rand(DBL, 400, rng), rand(DBL, 400, rng)
    da, db = ga_amd.DeviceBuffer(A0.nbytes), ga_amd.DeviceBuffer(B.nbytes)
    da.upload(A0)
    db.upload(B)
    a, ap = ga_amd.scale_buffer(DBL, 2.0)
    me = ctypes.c_int()
    L.comex_group_rank(0, ctypes.byref(me))
    L.armci_acc_2D(DBL, ap, me.value, ctypes.c_void_p(db.ptr), ctypes.c_void_p(da.ptr), 8 * 5 + 3, 6, 8 * 9 + 7,
                   8 * 11 + 1, 1)
    got = da.download(np.float64, 400)
    want = A0.copy()
    Oracle().legacy_acc_2D(DBL, 2.0, B, want, 8 * 5 + 3, 6, 8 * 9 + 7, 8 * 11 + 1)
    assert got.tobytes() == want.tobytes()
