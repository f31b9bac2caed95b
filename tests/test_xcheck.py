"""The cross-GPU self-check (ga_amd/xcheck.py) computes its expected bytes in closed
form, without the oracle, so that bench.py can run it on the driver's 8-GPU node.
CPU: that closed form agrees with the oracle (pinned to the reference's own _acc,
acc.h:106-154, and pack/unpack, comex.c:1267-1384) on every descriptor the check
generates.  GPU: the check runs between ranks on one MI355X with every peer treated
as another GPU, and a dropped packed chunk is caught and classified as a logic fault
(tests/test_multiproc.py launches those)."""
import numpy as np
import pytest

from ga_amd import xcheck as X


@pytest.mark.parametrize("seed", [20260, 7, 99])
def test_closed_form_matches_oracle(oracle, seed):
    for rnd in range(2):
        for src_rank in range(3):
            descs, iov, rmw_off, total = X._program(seed, rnd, src_rank)
            assert total <= X.SEG_BYTES
            ops = {d.op for d in descs}
            assert ops == set(X.ACC_OPS) | {X.PUT}
            assert any(d.src_kind == "seg" and d.count[0] * np.prod(d.count[1:]) >= 1 << 20 for d in descs)
            assert {d.levels for d in descs} - {0, 1, 2} and any(d.dphase % d.esz for d in descs if d.esz >= 8)
            for d in descs:
                src = d.src_bytes()
                want = d.init.copy()
                if d.op == X.PUT:
                    oracle.puts(src, d.sphase, d.sstr, want, d.dphase, d.dstr, d.count, d.levels)
                else:
                    sc = np.array([X.ALPHA[d.op]], dtype=X.DTYPE[d.op])
                    oracle.accs(d.op, sc[0], src, d.sphase, d.sstr, want, d.dphase, d.dstr, d.count, d.levels)
                assert np.array_equal(d.expected(), want), (X.OP_NAME[d.op], d.levels, d.count, d.dstr, d.dphase)


def test_patches_do_not_overlap():
    descs, iov, rmw_off, total = X._program(20260, 0, 1)
    spans = sorted((d.off, d.off + d.dspan) for d in descs)
    spans.append((iov["off"], iov["off"] + iov["init"].nbytes))
    spans.append((rmw_off, rmw_off + 64))
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 <= b0
    # rows of one patch share no byte (every stride at least the span below it)
    for d in descs:
        idx = d.elems(d.dstr, 0)
        assert np.unique(idx).size == idx.size


def test_iov_closed_form_sums_repeats(oracle):
    """the io-vector expectation (repeated destinations summed, put slots copied) is
    the oracle's pair-by-pair _acc / memcpy (comex.c:7342-7351)"""
    for rnd in range(len(X.ACC_OPS)):
        _, iov, _, _ = X._program(5, rnd, 0)
        m, nslot, nb = iov["m"], iov["nslot"], iov["bytes"]
        want = iov["init"].copy()
        src, psrc = iov["src"], iov["put_src"]
        base = want.ctypes.data
        sa = np.array([src.ctypes.data + k * nb for k in range(len(iov["acc_dst"]))], dtype=np.uint64)
        da = np.array([base + int(j) * nb for j in iov["acc_dst"]], dtype=np.uint64)
        oracle.accv(iov["op"], X.ALPHA[iov["op"]], sa, da, nb)
        sp = np.array([psrc.ctypes.data + k * nb for k in range(len(iov["put_dst"]))], dtype=np.uint64)
        dp = np.array([base + (nslot + int(j)) * nb for j in iov["put_dst"]], dtype=np.uint64)
        oracle.copyv(sp, dp, nb)
        assert np.array_equal(X._iov_expected(iov).view(np.uint8), want.view(np.uint8)), X.OP_NAME[iov["op"]]
        assert len(set(iov["acc_dst"].tolist())) < len(iov["acc_dst"])     # repeats present
