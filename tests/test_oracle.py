"""CPU: the oracle restatement against the reference's golden vectors and
independent formulations.  No GPU."""
import itertools

import numpy as np
import pytest

import cases as C
from helpers import same_bits_nan_aware
from oracle import Ref, ref_available


def _case_ids(manifest):
    return [c["name"] for c in manifest["cases"]]


def test_golden_catalogue_matches_cases(manifest):
    assert _case_ids(manifest) == [c["name"] for c in C.cases()]


def test_oracle_accs_matches_reference_golden(oracle, manifest, golden):
    """ora_accs (comex_oracle.c) == the reference's _acc output, bit for bit."""
    for case in manifest["cases"]:
        n = case["name"]
        src, dst = golden[f"{n}/src"], golden[f"{n}/dst_in"].copy()
        if case.get("alias"):
            src = dst   # src and dst in one buffer
        oracle.accs(case["op"], C.SCALE[case["op"]], src, case["src_off"], case["src_stride"], dst,
                    case["dst_off"], case["dst_stride"], case["count"], case["levels"])
        assert np.array_equal(dst, golden[f"{n}/dst_out"]), n


def test_alias_cases_exercise_every_ordering_class(manifest):
    """The aliased golden cases (one buffer, reference outputs from oracle/_ref) reach
    each of the launcher's ordering classes: parallel, ordered and one-lane serial."""
    import ga_amd
    kinds = set()
    base = 0x7F0000000000
    for c in manifest["cases"]:
        if c.get("alias"):
            kinds.add(ga_amd.plan_strided(c["op"], base + c["src_off"], c["src_stride"], base + c["dst_off"],
                                          c["dst_stride"], c["count"], c["levels"])["kind"])
    assert {"ordered", "serial"} <= kinds and kinds & {"rows", "flat"}, kinds


def test_oracle_packed_route_matches_direct(oracle, manifest, golden):
    """pack -> unpack-acc (comex.c:6965-7109 + 4238-4268) == per-row nb_accs result
    for every case whose dst rows do not overlap."""
    for case in manifest["cases"]:
        n = case["name"]
        if "overlap" in n or "zero_dst_stride" in n or case.get("alias"):
            continue
        src, dst = golden[f"{n}/src"], golden[f"{n}/dst_in"].copy()
        oracle.accs_packed(case["op"], C.SCALE[case["op"]], src, case["src_off"], case["src_stride"], dst,
                           case["dst_off"], case["dst_stride"], case["count"], case["levels"])
        assert same_bits_nan_aware(dst, golden[f"{n}/dst_out"], case["op"]), n


def test_inputs_regenerate_from_seeds(manifest, golden):
    """The committed inputs are exactly the §8(d) generator's output."""
    for case in C.cases()[:40]:
        src, dst = C.make_inputs(case)
        assert np.array_equal(src, golden[f"{case['name']}/src"])
        assert np.array_equal(dst, golden[f"{case['name']}/dst_in"])


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.int32, np.int64])
def test_numpy_generator_matches_c_generator(oracle, dtype):
    n = 10007
    a = oracle.fill(np.empty(n, dtype=dtype), C.SEED)
    b = C.fill_real(dtype, n, C.SEED)
    assert np.array_equal(a.view(np.uint8), b.view(np.uint8))


def _np_strided_view(buf, off, strides, count, levels):
    """Independent formulation of the odometer: numpy as_strided over the patch.
    Returns an array indexed [d_L, ..., d_1, byte] (slowest first)."""
    shape = [count[j] for j in range(levels, 0, -1)] + [count[0]]
    st = [strides[j - 1] for j in range(levels, 0, -1)] + [1]
    return np.lib.stride_tricks.as_strided(buf[off:], shape=shape, strides=st)


@pytest.mark.parametrize("levels", [0, 1, 2, 3, 6])
def test_pack_unpack_vs_numpy(oracle, levels):
    rng = np.random.default_rng(levels)
    count = [int(rng.integers(1, 9)) * 4] + [int(rng.integers(1, 5)) for _ in range(levels)]
    strides, acc = [], count[0] + 4 * int(rng.integers(0, 3))
    for j in range(levels):
        strides.append(acc)
        acc = acc * count[j + 1] + 4 * int(rng.integers(0, 3))
    lo, hi = C.span(strides, count, levels)
    buf = rng.integers(0, 256, size=hi + 16, dtype=np.uint8)
    packed = oracle.pack(buf, 8, strides, count, levels)
    want = _np_strided_view(buf, 8, strides, count, levels).reshape(-1)
    assert np.array_equal(packed, want)
    out = np.zeros_like(buf)
    oracle.unpack(packed, out, 8, strides, count, levels)
    assert np.array_equal(_np_strided_view(out, 8, strides, count, levels).reshape(-1), want)


def test_accs_vs_numpy_float64(oracle):
    """Fused strided acc == numpy dst_view += src_view*alpha (elementwise mul then add)."""
    rng = np.random.default_rng(7)
    src = rng.standard_normal(64 * 40)
    dst = rng.standard_normal(70 * 40)
    want = dst.copy()
    sv = want.reshape(40, 70)[3:33, 5:55]
    sv += src.reshape(40, 64)[2:32, 1:51] * 0.3
    got = dst.copy()
    oracle.accs(C.DBL, 0.3, src.view(np.uint8), (2 * 64 + 1) * 8, [64 * 8], got.view(np.uint8),
                (3 * 70 + 5) * 8, [70 * 8], [50 * 8, 30], 1)
    assert np.array_equal(got, want)


CONTIG_CASES = [
    # (src_stride, dst_stride, count, n_stride, expected) -- armci.c:114-170 semantics
    ([80], [80], [80, 4], 1, 1),        # full rows back to back
    ([96], [80], [80, 4], 1, 0),        # src has a gap
    ([80], [80], [40, 1], 1, 1),        # single partial row
    ([80], [80], [40, 2], 1, 0),        # two partial rows
    ([80, 320], [80, 320], [80, 4, 3], 2, 1),
    ([80, 400], [80, 320], [80, 4, 3], 2, 0),
    ([80, 320], [80, 320], [80, 2, 1], 2, 1),
    ([80, 320], [80, 320], [80, 2, 2], 2, 0),
]


@pytest.mark.parametrize("ss,ds,count,n,want", CONTIG_CASES)
def test_check_contiguous(oracle, ss, ds, count, n, want):
    assert oracle.check_contiguous(ss, ds, count, n) == want


@pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built (no reference tree)")
def test_restatement_vs_reference_random(oracle):
    """Random small patches for every op: restated _acc == compiled reference _acc."""
    ref = Ref()
    rng = np.random.default_rng(11)
    for op, levels in itertools.product((C.INT, C.DBL, C.FLT, C.CPL, C.DCP, C.LNG), (0, 1, 2, 4)):
        esz = C.ESZ[op]
        count = [int(rng.integers(1, 20)) * esz] + [int(rng.integers(1, 4)) for _ in range(levels)]
        ss, ds, a1, a2 = [], [], count[0], count[0] + esz
        for j in range(levels):
            ss.append(a1)
            ds.append(a2)
            a1 *= count[j + 1] + 1
            a2 *= count[j + 1]
        src = C.fill_bytes(op, C.span(ss, count, levels)[1], 99)
        dst = C.fill_bytes(op, C.span(ds, count, levels)[1], 98)
        d1, d2 = dst.copy(), dst.copy()
        oracle.accs(op, C.SCALE[op], src, 0, ss, d1, 0, ds, count, levels)
        ref.accs(op, C.SCALE[op], src, 0, ss, d2, 0, ds, count, levels)
        assert np.array_equal(d1, d2), (op, levels)


@pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built (no reference tree)")
def test_accv_restatement_vs_reference(oracle):
    """io-vector accumulate: the restated per-pair loop (ora_accv) == the reference's
    _acc per pair (ref_accv over acc.h), with repeated and overlapping destinations,
    every op, 1..5 elements per pair."""
    ref = Ref()
    rng = np.random.default_rng(12)
    for op in (C.INT, C.DBL, C.FLT, C.CPL, C.DCP, C.LNG):
        esz = C.ESZ[op]
        for nel in (1, 2, 5):
            nbytes, n = esz * nel, 3000
            src = C.fill_bytes(op, n * nbytes, 31)
            dst = C.fill_bytes(op, 200 * esz + nbytes, 32)
            so = (rng.integers(0, n, n) * nbytes).astype(np.uint64)
            do = (rng.integers(0, 200, n) * esz).astype(np.uint64)   # repeats, and overlaps when nel > 1
            d1, d2 = dst.copy(), dst.copy()
            oracle.accv(op, C.SCALE[op], so + np.uint64(src.ctypes.data), do + np.uint64(d1.ctypes.data), nbytes)
            ref.accv(op, C.SCALE[op], so + np.uint64(src.ctypes.data), do + np.uint64(d2.ctypes.data), nbytes)
            assert np.array_equal(d1, d2), (op, nel)


@pytest.mark.parametrize("nthreads", [1, 3, 8])
def test_multi_worker_baseline_matches_single(oracle, manifest, golden, nthreads):
    """The P-worker CPU baseline (mt_split.h) splits a patch into disjoint slabs:
    same bytes as one worker on every non-overlapping golden case."""
    impls = [oracle] + ([Ref()] if ref_available() else [])
    for case in manifest["cases"]:
        n = case["name"]
        if "overlap" in n or "zero_dst_stride" in n or case.get("alias"):   # slabs would race on shared bytes
            continue
        src = golden[f"{n}/src"]
        for impl in impls:
            dst = golden[f"{n}/dst_in"].copy()
            impl.accs_mt(case["op"], C.SCALE[case["op"]], src, case["src_off"], case["src_stride"], dst,
                         case["dst_off"], case["dst_stride"], case["count"], case["levels"], nthreads)
            assert np.array_equal(dst, golden[f"{n}/dst_out"]), (n, type(impl).__name__)
