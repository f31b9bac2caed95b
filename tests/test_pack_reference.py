"""Pack / unpack and the odometer order, pinned against the reference's own code.

ComEx-ARMCI's stride iterator (comex/src-armci/iterator.c, compiled as it lies into
oracle/_ref/libref_iterator.so) walks a strided descriptor's contiguous segments in
the reference's odometer order; armci_write_strided copies them into a contiguous
buffer (a pack) and armci_read_strided back (an unpack) -- what GA's ghost updates
call (global/src/ghosts.c:1792, 1841).  src-mpi-pr's pack/unpack (comex.c:1267-1384)
visit the rows in the same order (their index loop, 1308-1322) but are static
functions of a file that needs the generated config.h, so the iterator is the
reference code for this that compiles here.

CPU: the oracle's restatement (ora_pack / ora_unpack, which the accumulate paths'
row order also comes from) equals the reference's copies byte for byte on random
descriptors of 0..7 stride levels.
GPU: gaamd_pack / gaamd_unpack (the copy kernel with packed strides) equal them too.
The iterator accepts only the non-overlapping descriptors it asserts
(stride[0] >= count[0], stride[i] >= stride[i-1] * count[i]), so overlapping ones
stay pinned by the restatement alone (test_gpu_semantics)."""
import numpy as np
import pytest

import ga_amd
from oracle import IterRef, Oracle, iter_ref_available

pytestmark = pytest.mark.skipif(not iter_ref_available(), reason="oracle/_ref/libref_iterator.so not built")


def descriptor(rng, levels):
    """count (bytes first), strides: a non-overlapping layout with random gaps"""
    count = [int(rng.integers(1, 65))]
    for _ in range(levels):
        count.append(int(rng.integers(1, 5)))
    strides = []
    prev = count[0]
    for j in range(levels):
        s = prev + int(rng.integers(0, 17))
        strides.append(s)
        prev = s * count[j + 1]
    span = count[0] + sum((count[j + 1] - 1) * strides[j] for j in range(levels))
    return count, strides, span


CASES = [(lv, seed) for lv in range(8) for seed in range(6)]


@pytest.mark.parametrize("levels,seed", CASES)
def test_restated_pack_unpack_equal_reference_iterator(levels, seed):
    rng = np.random.default_rng(1000 * levels + seed)
    ora, ref = Oracle(), IterRef()
    count, strides, span = descriptor(rng, levels)
    P = ora.packed_size(count, levels)
    off = int(rng.integers(0, 8))
    src = rng.integers(0, 256, span + off + 8, dtype=np.uint8)
    assert np.array_equal(ora.pack(src, off, strides, count, levels),
                          ref.write_strided(src, off, strides, count, levels, P))
    packed = rng.integers(0, 256, P, dtype=np.uint8)
    want = rng.integers(0, 256, span + off + 8, dtype=np.uint8)
    got = want.copy()
    ref.read_strided(packed, want, off, strides, count, levels)
    ora.unpack(packed, got, off, strides, count, levels)
    assert np.array_equal(got, want)


def test_reference_iterator_edge_descriptors():
    """single-byte rows, unit counts at every level, tight (gap-free) layouts"""
    ora, ref = Oracle(), IterRef()
    for count, strides in [([1], []), ([1, 1], [1]), ([3, 1, 1, 1], [3, 3, 3]), ([8, 4], [8]),
                           ([5, 2, 3], [7, 14]), ([2, 1, 1, 1, 1, 1, 1, 2], [2, 2, 2, 2, 2, 2, 2])]:
        levels = len(strides)
        span = count[0] + sum((count[j + 1] - 1) * strides[j] for j in range(levels))
        src = np.arange(span + 4, dtype=np.uint8)
        P = ora.packed_size(count, levels)
        assert np.array_equal(ora.pack(src, 1, strides, count, levels),
                              ref.write_strided(src, 1, strides, count, levels, P)), (count, strides)


@pytest.mark.gpu
@pytest.mark.parametrize("levels", range(8))
def test_gpu_pack_unpack_equal_reference_iterator(gpu_lib, levels):
    rng = np.random.default_rng(77 + levels)
    ref, ora = IterRef(), Oracle()
    for _ in range(4):
        count, strides, span = descriptor(rng, levels)
        P = ora.packed_size(count, levels)
        src = rng.integers(0, 256, span + 16, dtype=np.uint8)
        sb, pb, db = ga_amd.DeviceBuffer(src.size), ga_amd.DeviceBuffer(max(P, 1)), ga_amd.DeviceBuffer(src.size)
        sb.upload(src)
        ga_amd.pack(sb.ptr + 3, strides, count, levels, pb.ptr)
        ga_amd.sync()
        packed = pb.download(np.uint8, P)
        assert np.array_equal(packed, ref.write_strided(src, 3, strides, count, levels, P))
        base = rng.integers(0, 256, span + 16, dtype=np.uint8)
        db.upload(base)
        ga_amd.unpack(pb.ptr, db.ptr + 5, strides, count, levels)
        ga_amd.sync()
        want = base.copy()
        ref.read_strided(packed, want, 5, strides, count, levels)
        assert np.array_equal(db.download(np.uint8, base.size), want)
