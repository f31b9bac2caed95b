"""ga_amd -- MI355X-native GA/ComEx strided pack/unpack + typed accumulate.

Python mirror of the C ABI in ``include/comex.h``, ``include/armci.h`` and
``include/ga_amd.h``.  The compute path is libga_amd.so (hand-written gfx950
HIP kernels); this package only marshals arguments.  Names follow the reference
(comex/src-common/comex.h, comex/src-armci/armci.h).
"""
import ctypes

import numpy as np

from ._lib import load, ALLGATHER_FN, BARRIER_FN  # noqa: F401

# comex.h:35-43 / armci.h:183-191
COMEX_GROUP_WORLD = 0
COMEX_SUCCESS = 0
COMEX_ACC_INT = 37
COMEX_ACC_DBL = 38
COMEX_ACC_FLT = 39
COMEX_ACC_CPL = 40
COMEX_ACC_DCP = 41
COMEX_ACC_LNG = 42
COMEX_MAX_STRIDE_LEVEL = 8
GAAMD_OP_COPY = 0

# op -> numpy dtype of one element (complex: the complex numpy type)
OP_DTYPE = {
    COMEX_ACC_INT: np.dtype(np.int32),
    COMEX_ACC_DBL: np.dtype(np.float64),
    COMEX_ACC_FLT: np.dtype(np.float32),
    COMEX_ACC_CPL: np.dtype(np.complex64),
    COMEX_ACC_DCP: np.dtype(np.complex128),
    COMEX_ACC_LNG: np.dtype(np.int64),
}
OP_NAME = {COMEX_ACC_INT: "int", COMEX_ACC_DBL: "dbl", COMEX_ACC_FLT: "flt", COMEX_ACC_CPL: "cpl",
           COMEX_ACC_DCP: "dcp", COMEX_ACC_LNG: "lng"}

KIND_NAME = {0: "auto", 1: "rows", 2: "flat", 3: "serial", 4: "ordered"}


def lib():
    return load()


def build_id():
    """sha256 of the sources libga_amd.so was compiled from (gaamd_build_id)."""
    return lib().gaamd_build_id().decode()


def check_build():
    """Raise when libga_amd.so was not built from the sources beside it (a stale
    prebuilt library shipped with a newer tree); returns the build id."""
    from .provenance import tree_hash
    built, tree = build_id(), tree_hash()
    if built != tree:
        raise RuntimeError(f"libga_amd.so is stale: built from sources {built[:16]}..., the tree here is "
                           f"{tree[:16]}... -- rebuild it (make -C ga_amd/csrc)")
    return built


def int_array(vals):
    vals = list(vals) if vals is not None else []
    arr = (ctypes.c_int * max(1, len(vals)))(*vals)
    return arr


def scale_buffer(op, scale):
    """The `void *scale` argument: one element of the op's type (complex = {re, im})."""
    dt = OP_DTYPE[op]
    a = np.array([scale], dtype=dt)
    return a, a.ctypes.data_as(ctypes.c_void_p)


class DeviceBuffer:
    """HBM allocation through the library (hipMalloc); never a torch tensor."""

    def __init__(self, nbytes, host=False):
        self.nbytes = int(nbytes)
        self.host = host
        L = lib()
        p = L.gaamd_host_malloc(self.nbytes) if host else L.gaamd_dev_malloc(max(1, self.nbytes))
        if not p:
            raise MemoryError(f"allocation of {nbytes} bytes failed")
        self.ptr = p

    def upload(self, arr, offset=0):
        arr = np.ascontiguousarray(arr)
        assert offset + arr.nbytes <= self.nbytes
        rc = lib().gaamd_memcpy(ctypes.c_void_p(self.ptr + offset), arr.ctypes.data_as(ctypes.c_void_p), arr.nbytes)
        if rc:
            raise RuntimeError("upload failed")

    def download(self, dtype, count=None, offset=0):
        dtype = np.dtype(dtype)
        if count is None:
            count = (self.nbytes - offset) // dtype.itemsize
        out = np.empty(count, dtype=dtype)
        rc = lib().gaamd_memcpy(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(self.ptr + offset), out.nbytes)
        if rc:
            raise RuntimeError("download failed")
        return out

    def free(self):
        if self.ptr:
            (lib().gaamd_host_free if self.host else lib().gaamd_dev_free)(ctypes.c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


# ---- kernel-level API (ga_amd.h section 2) ---------------------------------
def strided(op, scale, src, src_stride, dst, dst_stride, count, stride_levels, stream=None):
    """Enqueue dst (+)= op(src) over a strided patch; src/dst are device addresses (ints)."""
    if op == GAAMD_OP_COPY:
        sp = None
    else:
        keep, sp = scale_buffer(op, scale)
    rc = lib().gaamd_strided(op, sp, ctypes.c_void_p(src), int_array(src_stride), ctypes.c_void_p(dst),
                             int_array(dst_stride), int_array(count), stride_levels, stream)
    if rc:
        raise RuntimeError(f"gaamd_strided failed with {rc}")


def pack(src, src_stride, count, stride_levels, packed, stream=None):
    rc = lib().gaamd_pack(ctypes.c_void_p(src), int_array(src_stride), int_array(count), stride_levels,
                          ctypes.c_void_p(packed), stream)
    if rc:
        raise RuntimeError(f"gaamd_pack failed with {rc}")


def unpack(packed, dst, dst_stride, count, stride_levels, stream=None):
    rc = lib().gaamd_unpack(ctypes.c_void_p(packed), ctypes.c_void_p(dst), int_array(dst_stride),
                            int_array(count), stride_levels, stream)
    if rc:
        raise RuntimeError(f"gaamd_unpack failed with {rc}")


def unpack_acc(op, scale, packed, dst, dst_stride, count, stride_levels, stream=None):
    keep, sp = scale_buffer(op, scale)
    rc = lib().gaamd_unpack_acc(op, sp, ctypes.c_void_p(packed), ctypes.c_void_p(dst), int_array(dst_stride),
                                int_array(count), stride_levels, stream)
    if rc:
        raise RuntimeError(f"gaamd_unpack_acc failed with {rc}")


def last_launch():
    k, w, u, n = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    b = ctypes.c_ulonglong()
    lib().gaamd_last_launch(ctypes.byref(k), ctypes.byref(w), ctypes.byref(u), ctypes.byref(n), ctypes.byref(b))
    return {"kind": KIND_NAME.get(k.value, k.value), "width": w.value, "unroll": u.value,
            "launches": n.value, "blocks": b.value}


def plan_strided(op, src, src_stride, dst, dst_stride, count, stride_levels, row_begin=0, row_end=None):
    """The launcher's plan for a strided op (no launch, no GPU): dict or raises on an error code."""
    out = (ctypes.c_longlong * 8)()
    rc = lib().gaamd_plan_strided(op, ctypes.c_void_p(src), int_array(src_stride), ctypes.c_void_p(dst),
                                  int_array(dst_stride), int_array(count), stride_levels, row_begin,
                                  (1 << 64) - 1 if row_end is None else row_end, out)
    if rc:
        raise ValueError(f"plan error {rc}")
    return {"kind": KIND_NAME.get(out[0], out[0]), "width": out[1], "unroll": out[2], "block": out[3],
            "launches": out[4], "blocks": out[5], "levels": out[6], "aligned": bool(out[7])}


def kernel_counts():
    """launches so far by kind (this process): {'rows': n, 'flat': n, 'serial': n, 'ordered': n}"""
    c = (ctypes.c_ulonglong * 5)()
    lib().gaamd_kernel_counts(c)
    return {"rows": c[1], "flat": c[2], "serial": c[3], "ordered": c[4]}


def device_topology():
    """after comex_init: ranks on this rank's GPU (itself included), distinct GPUs among
    this node's ranks, and the peer-load mode (0 auto, 1 all peers as other GPUs, 2 off)"""
    a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    if lib().gaamd_device_topology(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)) != 0:
        return None
    return {"ranks_on_gpu": a.value, "gpus_on_node": b.value,
            "peer_loads": {0: "auto", 1: "all", 2: "off"}.get(c.value, c.value)}


def route_counts():
    """requests this rank posted to same-node owners, by route"""
    c = (ctypes.c_ulonglong * 4)()
    lib().gaamd_route_counts(c)
    return {"packed": c[0], "direct_src": c[1], "iov": c[2], "rmw": c[3], "one_pass": lib().gaamd_one_pass_count()}


def toggle_counts():
    """operations that took the reference's PACKED / IOV / GET_SELF+SMP toggle routes"""
    c = (ctypes.c_ulonglong * 3)()
    lib().gaamd_toggle_counts(c)
    return {"rows": c[0], "pairs": c[1], "owner_gets": c[2]}


def iov_path_counts():
    """local io-vector launches with repeated-destination ordering, by path"""
    c = (ctypes.c_ulonglong * 4)()
    lib().gaamd_iov_path_counts(c)
    return {"hashed": c[0], "hashed_then_radix": c[1], "radix": c[2], "lds": c[3]}


def owner_counts():
    """requests this rank's progress thread applied, by kind"""
    c = (ctypes.c_ulonglong * 4)()
    lib().gaamd_owner_counts(c)
    return {"packed": c[0], "iov": c[1], "rmw": c[2], "direct_src": c[3]}


def set_tuning(key, value):
    return lib().gaamd_set_tuning(key.encode(), int(value))


def get_tuning(key):
    return lib().gaamd_get_tuning(key.encode())


def sync(stream=None):
    rc = lib().gaamd_sync(stream)
    if rc:
        raise RuntimeError(f"device sync failed ({rc})")


def fill(ptr, n, type_code, seed, stream=None):
    rc = lib().gaamd_fill(ctypes.c_void_p(ptr), int(n), int(type_code), int(seed), stream)
    if rc:
        raise RuntimeError("gaamd_fill failed")


# ---- io-vector descriptors (comex.h:13-18, armci.h:17-22) ------------------
def fill_const(ptr, nbytes, value, dtype="float64"):
    """Fill nbytes of device memory at ptr with a constant of an 8-byte dtype (one
    kernel; enqueued on the library's primary stream -- sync() before use)."""
    import numpy as np
    word = int(np.array([value], dtype=dtype).view(np.uint64)[0])
    assert np.dtype(dtype).itemsize == 8 and nbytes % 8 == 0
    if lib().gaamd_fill_word(ctypes.c_void_p(ptr), nbytes // 8, word, None) != 0:
        raise RuntimeError("gaamd_fill_word failed")


class GIOV(ctypes.Structure):
    _fields_ = [("src", ctypes.POINTER(ctypes.c_void_p)), ("dst", ctypes.POINTER(ctypes.c_void_p)),
                ("count", ctypes.c_int), ("bytes", ctypes.c_int)]


def make_giov(descs):
    """descs: list of (src_addrs, dst_addrs, bytes) -> (array of GIOV, keep-alive list)."""
    arr = (GIOV * len(descs))()
    keep = []
    for k, (src, dst, nbytes) in enumerate(descs):
        s = (ctypes.c_void_p * max(1, len(src)))(*src)
        d = (ctypes.c_void_p * max(1, len(dst)))(*dst)
        keep += [s, d]
        arr[k].src = ctypes.cast(s, ctypes.POINTER(ctypes.c_void_p))
        arr[k].dst = ctypes.cast(d, ctypes.POINTER(ctypes.c_void_p))
        arr[k].count = len(src)
        arr[k].bytes = nbytes
    return arr, keep


def comex_accv(op, scale, descs, proc, group=COMEX_GROUP_WORLD):
    keep_s, sp = scale_buffer(op, scale)
    arr, keep = make_giov(descs)
    return lib().comex_accv(op, sp, ctypes.cast(arr, ctypes.c_void_p), len(descs), proc, group)


def comex_putv(descs, proc, group=COMEX_GROUP_WORLD):
    arr, keep = make_giov(descs)
    return lib().comex_putv(ctypes.cast(arr, ctypes.c_void_p), len(descs), proc, group)


def comex_getv(descs, proc, group=COMEX_GROUP_WORLD):
    arr, keep = make_giov(descs)
    return lib().comex_getv(ctypes.cast(arr, ctypes.c_void_p), len(descs), proc, group)


# ---- ComEx API (comex.h) ----------------------------------------------------
def comex_init():
    return lib().comex_init()


def comex_finalize():
    return lib().comex_finalize()


def comex_accs(op, scale, src, src_stride, dst, dst_stride, count, stride_levels, proc,
               group=COMEX_GROUP_WORLD):
    keep, sp = scale_buffer(op, scale)
    return lib().comex_accs(op, sp, ctypes.c_void_p(src), int_array(src_stride), ctypes.c_void_p(dst),
                            int_array(dst_stride), int_array(count), stride_levels, proc, group)


def comex_nbaccs(op, scale, src, src_stride, dst, dst_stride, count, stride_levels, proc,
                 group=COMEX_GROUP_WORLD):
    keep, sp = scale_buffer(op, scale)
    h = ctypes.c_int(-1)
    rc = lib().comex_nbaccs(op, sp, ctypes.c_void_p(src), int_array(src_stride), ctypes.c_void_p(dst),
                            int_array(dst_stride), int_array(count), stride_levels, proc, group, ctypes.byref(h))
    return rc, h


def comex_acc(op, scale, src, dst, nbytes, proc, group=COMEX_GROUP_WORLD):
    keep, sp = scale_buffer(op, scale)
    return lib().comex_acc(op, sp, ctypes.c_void_p(src), ctypes.c_void_p(dst), int(nbytes), proc, group)


def comex_puts(src, src_stride, dst, dst_stride, count, stride_levels, proc, group=COMEX_GROUP_WORLD):
    return lib().comex_puts(ctypes.c_void_p(src), int_array(src_stride), ctypes.c_void_p(dst),
                            int_array(dst_stride), int_array(count), stride_levels, proc, group)


def comex_gets(src, src_stride, dst, dst_stride, count, stride_levels, proc, group=COMEX_GROUP_WORLD):
    return lib().comex_gets(ctypes.c_void_p(src), int_array(src_stride), ctypes.c_void_p(dst),
                            int_array(dst_stride), int_array(count), stride_levels, proc, group)


def comex_wait(h):
    return lib().comex_wait(ctypes.byref(h))


def comex_fence_all(group=COMEX_GROUP_WORLD):
    return lib().comex_fence_all(group)


def comex_barrier(group=COMEX_GROUP_WORLD):
    return lib().comex_barrier(group)


def comex_malloc(nbytes, size, group=COMEX_GROUP_WORLD):
    arr = (ctypes.c_void_p * size)()
    rc = lib().comex_malloc(arr, int(nbytes), group)
    if rc:
        raise RuntimeError("comex_malloc failed")
    return [a or 0 for a in arr]


def comex_free(ptr, group=COMEX_GROUP_WORLD):
    return lib().comex_free(ctypes.c_void_p(ptr), group)
