"""Host logic of the strided launcher, on the CPU (no GPU): gaamd_plan_strided
runs the launcher's planning -- level merging, ordering/aliasing checks, vector
width, kernel family, block size, chunk alignment, row ranges -- and returns the
plan without launching.  Addresses are synthetic (nothing is dereferenced)."""
import pytest

import ga_amd

DBL, FLT, DCP = 38, 39, 41
COPY = 0
SRC, DST = 0x7F0000000000, 0x7F4000000000   # far apart, 64 KiB-aligned


def plan(op, src, ss, dst, ds, count, levels, rb=0, re=None):
    return ga_amd.plan_strided(op, src, ss, dst, ds, count, levels, rb, re)


def test_headline_shape():
    p = plan(DBL, SRC, [65536], DST, [65536], [16384, 4096], 1)
    assert p["kind"] == "rows" and p["width"] == 16 and p["levels"] == 1
    assert p["block"] == 64 and p["blocks"] == 4096 * 16 and p["launches"] == 1 and not p["aligned"]


def test_misaligned_rows_take_128_threads_and_aligned_chunks():
    p = plan(DBL, SRC, [65600], DST, [65600], [16384, 4096], 1)
    assert p["block"] == 128 and p["aligned"]


def test_contiguous_rows_collapse_to_one_run():
    p = plan(DBL, SRC, [16384], DST, [16384], [16384, 4096], 1)
    assert p["levels"] == 0 and p["kind"] == "rows"


def test_continuing_levels_merge():
    # level 2 continues level 1 on both sides (stride2 = stride1 * count1)
    p = plan(DBL, SRC, [8192, 8192 * 10], DST, [4096 * 3, 4096 * 3 * 10], [4096, 10, 7], 2)
    assert p["levels"] == 1


def test_overlapping_destination_rows_are_ordered():
    """dst rows sharing bytes with each other at other offsets: rows in the
    reference's order, each row wave-parallel (one 1024-thread workgroup), not one lane"""
    p = plan(DBL, SRC, [64], DST, [32], [64, 100], 1)
    assert p["kind"] == "ordered" and p["width"] == 16 and p["block"] == 1024 and p["blocks"] == 1
    assert p["unroll"] == 0


def test_coinciding_destination_rows_take_column_slices():
    """Rows that share bytes only at the same offset (a zero dst stride: every row
    into one run, a column reduction): 8-byte column slices, each walked in row order
    by one lane; the rows are loaded by seven loader waves of an
    eight-wave workgroup and applied from LDS by the eighth: the
    narrowest of 16/32/64 slices per workgroup that keeps the workgroups within one
    pass over the 256 CUs."""
    p = plan(DBL, SRC, [65536], DST, [0], [65536, 2048], 1)
    assert p["kind"] == "ordered" and p["unroll"] == 1 and p["width"] == 8
    assert p["block"] == 512 and p["blocks"] == 65536 // 8 // 32
    p = plan(DBL, SRC, [262144], DST, [0], [262144, 64], 1)
    assert p["block"] == 512 and p["blocks"] == 262144 // 8 // 64
    # ordered_cols = 1: one lane per slice loading its own rows, one-wave workgroups
    old = ga_amd.set_tuning("ordered_cols", 1)
    try:
        p = plan(DBL, SRC, [65536], DST, [0], [65536, 2048], 1)
        assert p["unroll"] == 1 and p["block"] == 64 and p["blocks"] == 65536 // 8 // 64
    finally:
        ga_amd.set_tuning("ordered_cols", old)
    # src and dst the same zero-stride run (dst += a*dst per row): slices without prefetch
    p = plan(DBL, SRC, [0], SRC, [0], [65536, 16], 1)
    assert p["kind"] == "ordered" and p["unroll"] == 2
    # src row i is dst row i+7 (same start): column slices without prefetch
    a = SRC
    p = plan(DBL, a, [65536], a + 65536 * 7, [65536], [16384, 64], 1)
    assert p["kind"] == "ordered" and p["unroll"] == 2
    # 3-D: planes accumulated into one plane (repeated dst level), rows disjoint within it
    p = plan(DBL, SRC, [8192, 8192 * 32], DST, [8192, 0], [8192, 32, 16], 2)
    assert p["kind"] == "ordered" and p["unroll"] == 1
    # a shifted src run inside a coinciding dst: order across columns -> one workgroup
    p = plan(DBL, DST + 8, [0], DST, [0], [4096, 16], 1)
    assert p["kind"] == "ordered" and p["unroll"] == 0
    old = ga_amd.set_tuning("ordered_cols", 0)
    try:
        assert plan(DBL, SRC, [65536], DST, [0], [65536, 2048], 1)["unroll"] == 0
    finally:
        ga_amd.set_tuning("ordered_cols", old)


def test_src_starting_inside_its_dst_row_below_it_is_serial_in_place_is_not():
    # src run at d - 8: element m reads what element m-1 of the same _acc loop wrote
    assert plan(DBL, SRC, [64], SRC + 8, [64], [64, 100], 1)["kind"] == "serial"
    # src run at d + 8: element m reads element m+1's old value -> ordered, parallel rows
    assert plan(DBL, SRC + 8, [64], SRC, [64], [64, 100], 1)["kind"] == "ordered"
    p = plan(DBL, SRC, [64], SRC, [64], [64, 100], 1)
    assert p["kind"] not in ("serial", "ordered")


def test_interleaved_spans_without_shared_bytes_are_parallel():
    """Columns 0..2047 accumulated into columns 2048..4095 of one ld-8192 f64 array:
    the spans interleave but no byte is shared -> the full-speed rows kernel
    (the round-1 span test sent this to the one-lane kernel)."""
    a = SRC
    p = plan(DBL, a, [65536], a + 16384, [65536], [16384, 4096], 1)
    assert p["kind"] == "rows" and p["width"] == 16 and p["blocks"] == 4096 * 16, p
    # 3-D with interleaved planes, still disjoint
    p = plan(DBL, a, [65536, 65536 * 64], a + 8192, [65536, 65536 * 64], [8192, 32, 16], 2)
    assert p["kind"] == "rows", p


def test_rows_sharing_bytes_across_rows_are_ordered():
    a = SRC
    # src row i is dst row i+1 (written later) and dst row i is src row i-1 (written earlier)
    assert plan(DBL, a, [65536], a + 65536, [65536], [16384, 4096], 1)["kind"] == "ordered"
    assert plan(DBL, a + 65536, [65536], a, [65536], [16384, 4096], 1)["kind"] == "ordered"
    # partial overlap of a neighbouring row
    assert plan(DBL, a, [65536], a + 65536 - 64, [65536], [16384, 64], 1)["kind"] == "ordered"


def test_one_stride_2d_closed_form_is_exact_at_any_size():
    """2-D, one stride on both sides: src row i meets dst row j iff |delta + (i-j) S| < row
    (closed form, any number of rows)"""
    a = SRC
    n = (1 << 20) + 10
    assert plan(DBL, a, [256], a + 64, [256], [64, n], 1)["kind"] in ("rows", "flat")   # interleaved, disjoint
    assert plan(DBL, a, [256], a + 32, [256], [64, n], 1)["kind"] == "serial"           # d - s = 32 < 64
    assert plan(DBL, a + 32, [256], a, [256], [64, n], 1)["kind"] == "ordered"          # src 32 B above
    assert plan(DBL, a, [256], a + 256 * 7, [256], [64, n], 1)["kind"] == "ordered"     # row i+7 = row i
    assert plan(DBL, a, [256], a + 256 * n, [256], [64, n], 1)["kind"] in ("rows", "flat")


def test_many_rows_with_meeting_spans_take_the_conservative_bound():
    """above 2^18 rows (and not the one-stride 2-D form) the analysis bounds spans and
    dst - src instead of sorting rows"""
    a = SRC
    n = (1 << 18) + 10
    assert plan(DBL, a, [256], a + 64, [264], [64, n], 1)["kind"] == "ordered"
    assert plan(DBL, a, [256], a + 32, [264], [64, n], 1)["kind"] == "serial"


def test_row_range_of_a_rebased_packed_side_is_not_serial():
    """The remote unpack-acc of rows [1000, 1100): the packed side is rebased so
    row 1000 lands at its staging slice; the full-range span of that rebased
    pointer would reach across dst and force the one-lane serial kernel."""
    row, rows = 16384, 4096
    staging = DST + (1 << 30)
    packed0 = staging - 1000 * row                # rebased base
    dst = staging - (8 << 20)                     # inside the rebased side's full span
    p = plan(DBL, packed0, [row], dst, [65536], [row, rows], 1, 1000, 1100)
    assert p["kind"] == "rows", p
    assert p["blocks"] == 100 * (row // 1024)
    # the same rows but overlapping for real (src run starting 8 B below its dst run)
    p2 = plan(DBL, packed0, [row], packed0 + 8, [row], [row, rows], 1, 1000, 1100)
    assert p2["kind"] == "serial"


@pytest.mark.parametrize("off,op,want", [(0, DBL, 16), (8, DBL, 8), (4, FLT, 4), (8, DCP, 16), (4, DBL, 8)])
def test_vector_width_follows_alignment(off, op, want):
    p = plan(op, SRC + off, [65536], DST, [65536], [4096, 64], 1)
    assert p["width"] == want


def test_sub_dword_alignment_is_rejected():
    """Elements below natural alignment run one per (dword-aligned) vector; below 4 bytes: refused."""
    with pytest.raises(ValueError):
        plan(DBL, SRC + 2, [65536], DST, [65536], [4096, 64], 1)


def test_short_rows_take_the_flat_kernel():
    p = plan(DBL, SRC, [1024], DST, [1024], [512, 1000], 1)
    assert p["kind"] == "flat"
    # one-wave blocks of one 16-byte vector per lane: 32 vectors x 1000 rows
    assert p["block"] == 64 and p["blocks"] == 32 * 1000 // 64
    # narrower vectors: 256 threads x 4
    p = plan(DBL, SRC + 8, [1024], DST, [1024], [512, 1000], 1)
    assert p["width"] == 8 and p["block"] == 256 and p["blocks"] == (64 * 1000 + 1023) // 1024
    assert plan(DBL, SRC, [4096], DST, [4096], [2048, 1000], 1)["kind"] == "rows"


def test_empty_patch_launches_nothing():
    p = plan(DBL, SRC, [64], DST, [64], [64, 0], 1)
    assert p["launches"] == 0


def test_eight_gib_block_is_one_launch():
    p = plan(DBL, SRC, [262144], DST, [262144 + 4096], [262144, 32768], 1)
    assert p["kind"] == "rows" and p["launches"] == 1 and p["blocks"] == 32768 * 256


def test_too_many_rows_is_an_error():
    with pytest.raises(ValueError):
        plan(COPY, SRC, [16, 16 * 65536], DST, [16, 16 * 65536], [16, 65536, 65536], 2)


def test_block_knob_overrides_auto():
    old = ga_amd.set_tuning("block", 128)
    try:
        assert plan(DBL, SRC, [65536], DST, [65536], [16384, 4096], 1)["block"] == 128
    finally:
        ga_amd.set_tuning("block", old)
    # the losing variants of rounds 1-2 are no longer knobs
    for key in ("unroll16", "nontemporal", "direct", "flat_nt", "flat_shape", "wide_unaligned"):
        assert ga_amd.set_tuning(key, 1) == -1, key
    assert ga_amd.set_tuning("block", 256) == -1


def test_rows_off_lines_on_both_sides_take_the_rows_kernel():
    # 2032 B rows (127 vectors) at ld 4064: rows start off 128 B lines -> rows kernel
    assert plan(DBL, SRC, [4064], DST, [4064], [2032, 1000], 1)["kind"] == "rows"
    # line-aligned rows of the same length stay flat
    assert plan(DBL, SRC, [4096], DST, [4096], [2032, 1000], 1)["kind"] == "flat"
    # one side on lines: flat
    assert plan(DBL, SRC, [4096], DST, [4064], [2032, 1000], 1)["kind"] == "flat"
    # short rows (16 vectors) stay flat even off lines
    assert plan(DBL, SRC, [528], DST, [528], [256, 1000], 1)["kind"] == "flat"
    old = ga_amd.set_tuning("flat_line_min", 0)
    try:
        assert plan(DBL, SRC, [4064], DST, [4064], [2032, 1000], 1)["kind"] == "flat"
    finally:
        ga_amd.set_tuning("flat_line_min", old)
