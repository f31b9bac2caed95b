"""Golden-case catalogue shared by make_golden.py and the parity tests.

Each case is one comex_accs call (comex/src-common/comex.h:327): an op, a scale,
a src buffer + byte offset + byte strides, a dst buffer + offset + strides, and
count[] (count[0] in bytes).  Buffers are filled with the SURVEY.md §8(d)
splitmix64 generator (seed 0x5EED0000 for src, +1 for dst) and then patched for
the edge cases.  The expected dst is produced by the REFERENCE's own _acc
(oracle/_ref, compiled from comex/src-common/acc.h) -- see make_golden.py.
"""
import numpy as np

SEED = 0x5EED0000
INT, DBL, FLT, CPL, DCP, LNG = 37, 38, 39, 40, 41, 42
ESZ = {INT: 4, DBL: 8, FLT: 4, CPL: 8, DCP: 16, LNG: 8}
REAL = {INT: np.int32, DBL: np.float64, FLT: np.float32, CPL: np.float32, DCP: np.float64, LNG: np.int64}
SCALE = {DBL: 0.7071067811865476, FLT: np.float32(0.70710677), INT: 3, LNG: -5,
         CPL: np.complex64(0.6 - 0.8j), DCP: 0.6 - 0.8j}
NAMES = {INT: "int", DBL: "dbl", FLT: "flt", CPL: "cpl", DCP: "dcp", LNG: "lng"}


def splitmix64(seed, n):
    """Vectorised splitmix64 element i (state after i+1 increments)."""
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def fill_real(dtype, n, seed):
    x = splitmix64(seed, n)
    dtype = np.dtype(dtype)
    if dtype == np.float64:
        return ((x >> np.uint64(11)).astype(np.float64) * 2.0 ** -53) * 2.0 - 1.0
    if dtype == np.float32:
        return ((x >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)) * np.float32(2.0) - np.float32(1.0)
    if dtype == np.int32:
        return ((x >> np.uint64(43)).astype(np.int64) - (1 << 20)).astype(np.int32)
    if dtype == np.int64:
        return (x >> np.uint64(43)).astype(np.int64) - (1 << 20)
    raise ValueError(dtype)


def fill_bytes(op, nbytes, seed):
    """A byte buffer of nbytes filled with op's element type (complex = reals)."""
    rt = np.dtype(REAL[op])
    n = nbytes // rt.itemsize
    buf = np.zeros(nbytes, dtype=np.uint8)
    buf[: n * rt.itemsize] = fill_real(rt, n, seed).view(np.uint8)
    return buf


def span(strides, count, levels):
    """(lo, hi) byte span of a strided side relative to its base."""
    lo, hi = 0, count[0]
    for j in range(levels):
        e = strides[j] * (count[j + 1] - 1)
        if e < 0:
            lo += e
        else:
            hi += e
    return lo, hi


def array_case(name, op, shape_elems, ld_src, ld_dst, lo_src=None, lo_dst=None):
    """Patch of `shape_elems` (fastest first) inside column-major arrays with leading
    dims ld_src/ld_dst (lists, elements), placed at lo_src/lo_dst (element coords)."""
    esz = ESZ[op]
    L = len(shape_elems) - 1
    count = [shape_elems[0] * esz] + list(shape_elems[1:])
    def strides(ld):
        s, acc = [], esz
        for j in range(L):
            acc *= ld[j]
            s.append(acc)
        return s
    ss, ds = strides(ld_src), strides(ld_dst)
    def off(lo, ld):
        if lo is None:
            return 0
        o, acc = 0, esz
        for j, c in enumerate(lo):
            o += c * acc
            if j < len(ld):
                acc *= ld[j]
        return o
    so, do = off(lo_src, ld_src), off(lo_dst, ld_dst)
    return dict(name=name, op=op, count=count, levels=L, src_stride=ss, dst_stride=ds,
                src_off=so, dst_off=do, src_bytes=so + span(ss, count, L)[1],
                dst_bytes=do + span(ds, count, L)[1], edge=None)


def cases():
    out = []
    for op in (DBL, FLT, INT, LNG, CPL, DCP):
        n = NAMES[op]
        # C1/C2 reduced: 1-D contiguous (stride_levels 0)
        out.append(array_case(f"{n}_1d_contig", op, [4099], [], []))
        # H reduced: 2-D patch in larger leading dims (src & dst strided)
        out.append(array_case(f"{n}_2d_h", op, [64, 48], [128], [128], [3, 5], [7, 2]))
        # C3-style odd leading dimension (ld 8200 analogue)
        out.append(array_case(f"{n}_2d_oddld", op, [61, 33], [67], [71], [1, 2], [5, 3]))
        # C4 reduced: 3-D patch, src contiguous, dst in a padded array
        out.append(array_case(f"{n}_3d", op, [12, 10, 8], [12, 10], [15, 13]))
        # run lengths around the 64-lane wave
        for r in (1, 7, 63, 64, 65):
            out.append(array_case(f"{n}_run{r}", op, [r, 9], [r + 3], [r + 1]))
        # every stride level 0..6 (ndim 1..7): 2^ndim patch at the far corner,
        # as comex/testing/test.c:1028-1128 test_acc does
        for ndim in range(1, 8):
            dims_a = [3] * ndim
            dims_b = [4] * ndim
            out.append(array_case(f"{n}_nd{ndim}", op, [2] * ndim, dims_a[:-1], dims_b[:-1],
                                  [0] * ndim, [2] * ndim))
    # FP edge fixtures
    for op in (DBL, FLT, CPL, DCP):
        n = NAMES[op]
        for edge in ("cancel", "subnormal", "signed_zero", "inf_nan"):
            if edge == "cancel":   # same layout on both sides so dst = -(alpha*src) lines up
                c = array_case(f"{n}_edge_{edge}", op, [37, 5], [40], [40], [1, 0], [1, 0])
            else:
                c = array_case(f"{n}_edge_{edge}", op, [37, 5], [40], [41], [1, 0], [2, 1])
            c["edge"] = edge
            out.append(c)
    for op in (INT, LNG):
        c = array_case(f"{NAMES[op]}_edge_wrap", op, [37, 5], [40], [41], [1, 0], [2, 1])
        c["edge"] = "wrap"
        out.append(c)
    # partial trailing element: count[0] not a multiple of the element size
    # (_acc processes bytes/sizeof(T) elements, acc.h:122)
    c = array_case("dbl_partial_elem", DBL, [10, 4], [12], [12])
    c["count"][0] = 10 * 8 + 5
    # the buffers must hold the partial bytes too: pack/unpack/put/get move all
    # count[0] bytes of every row (comex.c:1308-1325), only _acc stops at whole elements
    c["src_bytes"] = c["src_off"] + span(c["src_stride"], c["count"], 1)[1]
    c["dst_bytes"] = c["dst_off"] + span(c["dst_stride"], c["count"], 1)[1]
    out.append(c)
    # overlapping destination rows: reference order decides the result
    c = array_case("dbl_overlap_dst_rows", DBL, [6, 5], [8], [8])
    c["dst_stride"] = [16]          # rows of 48 B, 16 B apart -> overlap
    c["dst_bytes"] = c["dst_off"] + span(c["dst_stride"], c["count"], 1)[1]
    out.append(c)
    c = array_case("int_zero_dst_stride", INT, [5, 7], [8], [8])
    c["dst_stride"] = [0]           # every row onto the same run
    c["dst_bytes"] = 5 * 4
    out.append(c)
    out.extend(alias_cases())
    return out


def alias_case(name, op, count, src_stride, dst_stride, src_off, dst_off, nbytes):
    """src and dst inside ONE buffer (the dst buffer): comex_accs on a patch of an
    array into another patch of the same array, where the reference's row and
    element order (comex.c:6936-6961, acc.h:137-143) decides the bytes wherever
    the two share memory.  `alias` cases carry no src array: src = dst + src_off."""
    L = len(count) - 1
    return dict(name=name, op=op, count=list(count), levels=L, src_stride=list(src_stride),
                dst_stride=list(dst_stride), src_off=src_off, dst_off=dst_off, src_bytes=0, dst_bytes=nbytes,
                edge=None, alias=True)


def alias_cases():
    out = []
    e = 8
    ld = 64 * e
    # columns 0..15 into columns 16..31 of one ld-64 array: interleaved spans, no byte shared
    out.append(alias_case("dbl_alias_columns", DBL, [16 * e, 40], [ld], [ld], 0, 16 * e, ld * 40))
    # src row i is dst row i+1 (written later) / dst row i-1 (written earlier)
    out.append(alias_case("dbl_alias_next_row", DBL, [40 * e, 30], [ld], [ld], ld, 0, ld * 32))
    out.append(alias_case("dbl_alias_prev_row", DBL, [40 * e, 30], [ld], [ld], 0, ld, ld * 32))
    # a row's src run one element below its dst run: a recurrence inside one _acc loop
    out.append(alias_case("dbl_alias_shift_down", DBL, [40 * e, 12], [ld], [ld], 0, e, ld * 13))
    # one element above: element m reads element m+1's old value
    out.append(alias_case("dbl_alias_shift_up", DBL, [40 * e, 12], [ld], [ld], e, 0, ld * 13))
    # a 3-D patch onto itself shifted by one plane and one row
    out.append(alias_case("flt_alias_3d_shift", FLT, [24 * 4, 6, 5], [32 * 4, 32 * 4 * 8], [32 * 4, 32 * 4 * 8],
                          32 * 4 * 8 + 32 * 4, 0, 32 * 4 * 8 * 7))
    # in place (src is dst): real forms are dst + a*dst; the complex forms' second
    # statement reads the real part the first one wrote (acc.h:47-49)
    for op in (DBL, CPL, DCP, INT):
        es = ESZ[op]
        out.append(alias_case(f"{NAMES[op]}_alias_inplace", op, [33 * es, 9], [48 * es], [48 * es], 0, 0,
                              48 * es * 9))
    # complex src half an element above / a quarter element above its dst run
    out.append(alias_case("dcp_alias_half_up", DCP, [20 * 16, 7], [32 * 16], [32 * 16], 8, 0, 32 * 16 * 8))
    out.append(alias_case("dcp_alias_quarter_up", DCP, [20 * 16, 7], [32 * 16], [32 * 16], 4 + 16, 16,
                          32 * 16 * 8))
    out.append(alias_case("cpl_alias_half_down", CPL, [20 * 8, 7], [32 * 8], [32 * 8], 0, 4, 32 * 8 * 8))
    # dst rows overlapping each other AND the src rows (zero dst stride onto the first row)
    out.append(alias_case("lng_alias_zero_dst_stride", LNG, [12 * 8, 9], [16 * 8], [0], 16 * 8, 0, 16 * 8 * 10))
    return out


def make_inputs(case):
    """(src, dst) byte buffers; an alias case has an empty src (its src is in dst)."""
    op = case["op"]
    src = fill_bytes(op, case["src_bytes"], SEED)
    dst = fill_bytes(op, case["dst_bytes"], SEED + 1)
    edge = case.get("edge")
    rt = np.dtype(REAL[op])
    if edge:
        s = src[: (src.size // rt.itemsize) * rt.itemsize].view(rt)
        d = dst[: (dst.size // rt.itemsize) * rt.itemsize].view(rt)
        if edge == "cancel":
            # identical layouts: dst = -(alpha*src) element for element, so the
            # reference's mul-then-add cancels exactly (an FMA would not)
            m = min(s.size, d.size)
            if op in (DBL, FLT):
                a = rt.type(SCALE[op])
                d[:m] = -(s[:m] * a)
            else:
                a = np.complex128(SCALE[op])
                sr, si = rt.type(a.real), rt.type(a.imag)
                m -= m % 2
                br, bi = s[0:m:2], s[1:m:2]
                d[0:m:2] = -((br * sr) - (bi * si))
                d[1:m:2] = -((br * si) + (bi * sr))
        elif edge == "subnormal":
            tiny = np.finfo(rt).tiny
            s[::3] = tiny * np.float64(0.375).astype(rt)
            d[::2] = -tiny * np.float64(0.25).astype(rt)
        elif edge == "signed_zero":
            s[::2] = rt.type(0.0)
            d[::3] = rt.type(-0.0)
            s[1::4] = rt.type(-0.0)
        elif edge == "inf_nan":
            s[::5] = np.inf
            s[1::7] = -np.inf
            d[::6] = np.nan
            s[2::11] = np.nan
        elif edge == "wrap":
            info = np.iinfo(rt)
            s[::2] = info.max - 1
            d[::3] = info.max
            s[1::3] = info.min + 2
    return src, dst
