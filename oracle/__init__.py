"""oracle -- CPU parity checker for the ga_amd HIP path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
package; the product library (ga_amd/libga_amd.so) never links or calls it.

* ``Oracle``: ctypes wrapper of liboracle.so, the C restatement of the reference
  path (comex_oracle.c: _acc acc.h:106-154, pack/unpack comex.c:1267-1384,
  nb_accs comex.c:6890-6962, unpack-acc comex.c:4238-4268,
  armci_check_contiguous armci.c:114-170).
* ``Ref``: ctypes wrapper of _ref/libref_acc.so, the REFERENCE's own _acc
  compiled from /root/reference/comex/src-common/acc.h (built only where the
  reference tree exists; the .so travels to the GPU box).
* ``LegacyRef``: _ref/libref_legacy_acc.so, the legacy ARMCI accumulate loops
  (armci/src/xfer/caccumulate.c) compiled as they lie.
* ``IterRef``: _ref/libref_iterator.so, ComEx-ARMCI's stride iterator
  (comex/src-armci/iterator.c) compiled as it lies: armci_write_strided (strided
  -> contiguous, the reference's pack in odometer order) and armci_read_strided
  (its unpack).
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref_acc.so")
LEGACY_SO = os.path.join(HERE, "_ref", "libref_legacy_acc.so")
ITER_SO = os.path.join(HERE, "_ref", "libref_iterator.so")

_ip = ctypes.POINTER(ctypes.c_int)
_vp = ctypes.c_void_p


def _ints(vals):
    vals = list(vals) if vals is not None else []
    return (ctypes.c_int * max(1, len(vals)))(*vals)


def _ptr(a):
    return a.ctypes.data_as(_vp)


class Oracle:
    def __init__(self, path=ORACLE_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        sig = {
            "ora_acc": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _vp, _vp, _vp]),
            "ora_elem_size": (ctypes.c_int, [ctypes.c_int]),
            "ora_packed_size": (ctypes.c_long, [_ip, ctypes.c_int]),
            "ora_pack": (ctypes.c_long, [_vp, _ip, _ip, ctypes.c_int, _vp]),
            "ora_unpack": (ctypes.c_long, [_vp, _vp, _ip, _ip, ctypes.c_int]),
            "ora_unpack_acc": (ctypes.c_long, [ctypes.c_int, _vp, _vp, _vp, _ip, _ip, ctypes.c_int]),
            "ora_accs": (ctypes.c_int, [ctypes.c_int, _vp, _vp, _ip, _vp, _ip, _ip, ctypes.c_int]),
            "ora_accv": (ctypes.c_int, [ctypes.c_int, _vp, _vp, _vp, ctypes.c_long, ctypes.c_int]),
            "ora_copyv": (None, [_vp, _vp, ctypes.c_long, ctypes.c_int]),
            "ora_accs_mt": (ctypes.c_int, [ctypes.c_int, _vp, _vp, _ip, _vp, _ip, _ip, ctypes.c_int, ctypes.c_int]),
            "ora_accs_packed": (ctypes.c_int, [ctypes.c_int, _vp, _vp, _ip, _vp, _ip, _ip, ctypes.c_int]),
            "ora_puts": (ctypes.c_int, [_vp, _ip, _vp, _ip, _ip, ctypes.c_int]),
            "ora_gets": (ctypes.c_int, [_vp, _ip, _vp, _ip, _ip, ctypes.c_int]),
            "ora_check_contiguous": (ctypes.c_int, [_ip, _ip, _ip, ctypes.c_int]),
            "ora_legacy_acc_2d": (ctypes.c_int, [ctypes.c_int, _vp, ctypes.c_int, ctypes.c_int, _vp, ctypes.c_int,
                                                 _vp, ctypes.c_int]),
            "ora_legacy_acc_2D": (ctypes.c_int, [ctypes.c_int, _vp, _vp, _vp, ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_int, ctypes.c_int]),
            "ora_fill_f64": (None, [_vp, ctypes.c_long, ctypes.c_uint64]),
            "ora_fill_f32": (None, [_vp, ctypes.c_long, ctypes.c_uint64]),
            "ora_fill_i32": (None, [_vp, ctypes.c_long, ctypes.c_uint64]),
            "ora_fill_i64": (None, [_vp, ctypes.c_long, ctypes.c_uint64]),
            "ora_splitmix64": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64]),
        }
        for n, (r, a) in sig.items():
            f = getattr(L, n)
            f.restype = r
            f.argtypes = a
        self.L = L

    # all byte buffers are numpy arrays; offsets in bytes
    def accs(self, op, scale, src, src_off, src_stride, dst, dst_off, dst_stride, count, levels):
        s = np.array([scale], dtype=_scale_dtype(op))
        rc = self.L.ora_accs(op, _ptr(s), _vp(src.ctypes.data + src_off), _ints(src_stride),
                             _vp(dst.ctypes.data + dst_off), _ints(dst_stride), _ints(count), levels)
        assert rc == 0

    def accs_mt(self, op, scale, src, src_off, src_stride, dst, dst_off, dst_stride, count, levels, nthreads):
        s = np.array([scale], dtype=_scale_dtype(op))
        rc = self.L.ora_accs_mt(op, _ptr(s), _vp(src.ctypes.data + src_off), _ints(src_stride),
                                _vp(dst.ctypes.data + dst_off), _ints(dst_stride), _ints(count), levels, nthreads)
        assert rc == 0

    def accs_packed(self, op, scale, src, src_off, src_stride, dst, dst_off, dst_stride, count, levels):
        s = np.array([scale], dtype=_scale_dtype(op))
        rc = self.L.ora_accs_packed(op, _ptr(s), _vp(src.ctypes.data + src_off), _ints(src_stride),
                                    _vp(dst.ctypes.data + dst_off), _ints(dst_stride), _ints(count), levels)
        assert rc == 0

    def accv(self, op, scale, src_addrs, dst_addrs, nbytes):
        """one _acc per (src, dst) pair in order; uint64 arrays of host addresses"""
        s = np.array([scale], dtype=_scale_dtype(op))
        assert self.L.ora_accv(op, _ptr(s), _vp(src_addrs.ctypes.data), _vp(dst_addrs.ctypes.data),
                               len(src_addrs), nbytes) == 0

    def copyv(self, src_addrs, dst_addrs, nbytes):
        """one memcpy per (src, dst) pair in order (putv / getv)"""
        self.L.ora_copyv(_vp(src_addrs.ctypes.data), _vp(dst_addrs.ctypes.data), len(src_addrs), nbytes)

    def puts(self, src, src_off, src_stride, dst, dst_off, dst_stride, count, levels):
        self.L.ora_puts(_vp(src.ctypes.data + src_off), _ints(src_stride), _vp(dst.ctypes.data + dst_off),
                        _ints(dst_stride), _ints(count), levels)

    def packed_size(self, count, levels):
        return self.L.ora_packed_size(_ints(count), levels)

    def pack(self, src, src_off, src_stride, count, levels):
        out = np.zeros(max(1, self.packed_size(count, levels)), dtype=np.uint8)
        self.L.ora_pack(_vp(src.ctypes.data + src_off), _ints(src_stride), _ints(count), levels, _ptr(out))
        return out[: self.packed_size(count, levels)]

    def unpack(self, packed, dst, dst_off, dst_stride, count, levels):
        self.L.ora_unpack(_ptr(packed), _vp(dst.ctypes.data + dst_off), _ints(dst_stride), _ints(count), levels)

    def unpack_acc(self, op, scale, packed, dst, dst_off, dst_stride, count, levels):
        s = np.array([scale], dtype=_scale_dtype(op))
        self.L.ora_unpack_acc(op, _ptr(s), _ptr(packed), _vp(dst.ctypes.data + dst_off), _ints(dst_stride),
                              _ints(count), levels)

    def legacy_acc_2d(self, op, alpha, rows, cols, A, ald, B, bld):
        """caccumulate.c: A (numpy, column-major with leading dim ald elements) += alpha * B"""
        s = np.array([alpha], dtype=_scale_dtype(op))
        assert self.L.ora_legacy_acc_2d(op, _ptr(s), rows, cols, _ptr(A), ald, _ptr(B), bld) == 0

    def legacy_acc_2D(self, op, alpha, src, dst, nbytes, cols, src_stride, dst_stride):
        """strided.c armci_acc_2D on numpy buffers (byte strides, truncated to elements)"""
        s = np.array([alpha], dtype=_scale_dtype(op))
        assert self.L.ora_legacy_acc_2D(op, _ptr(s), _ptr(src), _ptr(dst), nbytes, cols, src_stride,
                                        dst_stride) == 0

    def check_contiguous(self, src_stride, dst_stride, count, n_stride):
        return self.L.ora_check_contiguous(_ints(src_stride), _ints(dst_stride), _ints(count), n_stride)

    def fill(self, arr, seed):
        n = arr.size
        fn = {np.dtype(np.float64): self.L.ora_fill_f64, np.dtype(np.float32): self.L.ora_fill_f32,
              np.dtype(np.int32): self.L.ora_fill_i32, np.dtype(np.int64): self.L.ora_fill_i64}[arr.dtype]
        fn(_ptr(arr), n, seed)
        return arr


class Ref:
    """The reference's own _acc (acc.h) driven per row; None-able if not built."""

    def __init__(self, path=REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        L = ctypes.CDLL(path)
        L.ref_acc.restype = ctypes.c_int
        L.ref_acc.argtypes = [ctypes.c_int, ctypes.c_int, _vp, _vp, _vp]
        L.ref_accs.restype = ctypes.c_int
        L.ref_accs.argtypes = [ctypes.c_int, _vp, _vp, _ip, _vp, _ip, _ip, ctypes.c_int]
        L.ref_accs_mt.restype = ctypes.c_int
        L.ref_accs_mt.argtypes = [ctypes.c_int, _vp, _vp, _ip, _vp, _ip, _ip, ctypes.c_int, ctypes.c_int]
        L.ref_accv.restype = ctypes.c_int
        L.ref_accv.argtypes = [ctypes.c_int, _vp, _vp, _vp, ctypes.c_long, ctypes.c_int]
        self.L = L

    def accs(self, op, scale, src, src_off, src_stride, dst, dst_off, dst_stride, count, levels):
        s = np.array([scale], dtype=_scale_dtype(op))
        self.L.ref_accs(op, _ptr(s), _vp(src.ctypes.data + src_off), _ints(src_stride),
                        _vp(dst.ctypes.data + dst_off), _ints(dst_stride), _ints(count), levels)

    def accs_mt(self, op, scale, src, src_off, src_stride, dst, dst_off, dst_stride, count, levels, nthreads):
        s = np.array([scale], dtype=_scale_dtype(op))
        rc = self.L.ref_accs_mt(op, _ptr(s), _vp(src.ctypes.data + src_off), _ints(src_stride),
                                _vp(dst.ctypes.data + dst_off), _ints(dst_stride), _ints(count), levels, nthreads)
        assert rc == 0

    def accv(self, op, scale, src_addrs, dst_addrs, nbytes):
        """one _acc per (src, dst) pair; src_addrs/dst_addrs: uint64 arrays of host addresses."""
        s = np.array([scale], dtype=_scale_dtype(op))
        assert self.L.ref_accv(op, _ptr(s), _vp(src_addrs.ctypes.data), _vp(dst_addrs.ctypes.data),
                               len(src_addrs), nbytes) == 0


LEGACY_NAME = {38: "d", 39: "f", 40: "c", 41: "z", 37: "i", 42: "l"}


class LegacyRef:
    """The reference's legacy c_?_accumulate_2d_ loops, called as GA's legacy
    ARMCI calls them (pointers to scalars, column-major)."""

    def __init__(self, path=LEGACY_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.L = ctypes.CDLL(path)

    def acc_2d(self, op, alpha, rows, cols, A, ald, B, bld, unrolled=False, name=None):
        s = np.array([alpha], dtype=_scale_dtype(op))
        fn = getattr(self.L, f"c_{name or LEGACY_NAME[op]}_accumulate_2d{'_u' if unrolled else ''}_")
        fn.restype = None
        r, c, a, b = ctypes.c_int(rows), ctypes.c_int(cols), ctypes.c_int(ald), ctypes.c_int(bld)
        fn(_ptr(s), ctypes.byref(r), ctypes.byref(c), _ptr(A), ctypes.byref(a), _ptr(B), ctypes.byref(b))

    def acc_1d(self, op, alpha, A, B, rows, name=None):
        s = np.array([alpha], dtype=_scale_dtype(op))
        fn = getattr(self.L, f"c_{name or LEGACY_NAME[op]}_accumulate_1d_")
        fn.restype = None
        r = ctypes.c_int(rows)
        fn(_ptr(s), _ptr(A), _ptr(B), ctypes.byref(r))


class IterRef:
    """The reference's stride iterator: armci_write_strided / armci_read_strided
    (iterator.c:156-194).  Its descriptors are the non-overlapping ones the
    iterator asserts (stride[0] >= count[0], stride[i] >= stride[i-1] * count[i])."""

    def __init__(self, path=ITER_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        L = ctypes.CDLL(path)
        for n in ("armci_write_strided", "armci_read_strided"):
            f = getattr(L, n)
            f.restype = None
            f.argtypes = [_vp, ctypes.c_int, _ip, _ip, _vp]
        self.L = L

    def write_strided(self, src, src_off, src_stride, count, levels, packed_size):
        """strided bytes of `src` (numpy uint8) -> a new contiguous buffer"""
        out = np.zeros(max(1, packed_size), dtype=np.uint8)
        self.L.armci_write_strided(_vp(src.ctypes.data + src_off), levels, _ints(src_stride), _ints(count), _ptr(out))
        return out[:packed_size]

    def read_strided(self, packed, dst, dst_off, dst_stride, count, levels):
        """contiguous `packed` -> the strided bytes of `dst` (in place)"""
        self.L.armci_read_strided(_vp(dst.ctypes.data + dst_off), levels, _ints(dst_stride), _ints(count), _ptr(packed))


def iter_ref_available():
    return os.path.exists(ITER_SO)


def legacy_ref_available():
    return os.path.exists(LEGACY_SO)


def ref_available():
    return os.path.exists(REF_SO)


def _scale_dtype(op):
    return {37: np.int32, 38: np.float64, 39: np.float32, 40: np.complex64, 41: np.complex128, 42: np.int64}[op]
