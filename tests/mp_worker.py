"""Worker for the multi-process tests (one rank per process).

Modes:
  boot-env   : built-in node-shm bootstrap from RANK/WORLD_SIZE; bootstrap
               self-test only (no GPU).
  boot-gloo  : torch.distributed gloo as the bootstrap hooks; self-test only.
  boot-nodes : gloo hooks + COMEX_AMD_NODE (several "nodes" on one host): per-node
               shm, cross-node collectives through the hooks, and the cross-node
               TCP transport (PING frames between all ranks).  No GPU.
  remote-gloo / ga-gloo: as remote / ga with gloo hooks; with COMEX_AMD_NODE set
               the ranks of different nodes talk through the wire protocol.
  remote     : comex on the GPU (every rank may share one device): segments by
               comex_malloc, remote accumulate through the owner's progress
               thread, remote put/get through IPC mappings, checked against the
               oracle.  Integer-valued f64 data so concurrent accumulates from
               several ranks sum exactly in any order.
Prints "RANK <r> OK" on success.
"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(HERE, "golden"))

import numpy as np  # noqa: E402


def torch_hooks(rank, size):
    import torch
    import torch.distributed as td
    import ga_amd
    td.init_process_group("gloo", rank=rank, world_size=size)

    def allgather(send, recv, nbytes, ctx):
        buf = torch.frombuffer(bytearray(ctypes.string_at(send, nbytes)), dtype=torch.uint8)
        out = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(size)]
        td.all_gather(out, buf)
        cat = torch.cat(out).numpy()   # keep alive across the memmove
        ctypes.memmove(recv, cat.ctypes.data, nbytes * size)
        return 0

    def barrier(ctx):
        td.barrier()
        return 0

    return ga_amd.ALLGATHER_FN(allgather), ga_amd.BARRIER_FN(barrier)


def main():
    import faulthandler
    # a hung rank prints where it is stuck before the test's timeout kills it
    faulthandler.dump_traceback_later(int(os.environ.get("TEST_STACK_DUMP_S", "600")), exit=False)
    mode = sys.argv[1]
    rank, size = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import ga_amd
    L = ga_amd.lib()
    if mode in ("boot-gloo", "remote-gloo", "boot-nodes", "ga-gloo", "stress-gloo", "scatremote-gloo",
                "armcimisc-gloo", "rdesc-gloo"):
        ag, bar = torch_hooks(rank, size)
        keep = (ag, bar)  # noqa: F841
        assert L.gaamd_set_bootstrap(rank, size, rank, ctypes.cast(ag, ctypes.c_void_p),
                                     ctypes.cast(bar, ctypes.c_void_p), None) == 0
    if mode.startswith("boot"):
        assert L.gaamd_bootstrap_selftest(5) == 0
        assert L.gaamd_rank() == rank and L.gaamd_size() == size
        if mode == "boot-nodes":
            nodes = [int(x) for x in os.environ["TEST_NODES"].split(",")]
            nd, nn, ns = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
            assert L.gaamd_node_info(ctypes.byref(nd), ctypes.byref(nn), ctypes.byref(ns)) == 0
            order = list(dict.fromkeys(nodes))
            assert nd.value == order.index(nodes[rank]), (nd.value, nodes)
            assert nn.value == len(order) and ns.value == nodes.count(nodes[rank])
            assert L.gaamd_wire_selftest(3) == 0
        if mode == "boot-fdx":
            assert L.gaamd_vmm_exchange_selftest(5) == 0
        print(f"RANK {rank} OK", flush=True)
        return
    if mode in ("ga", "ga-gloo"):
        ga_test(L, rank, size)
    elif mode in ("stress", "stress-gloo"):
        stress_test(L, rank, size)
    elif mode == "testacc":
        test_acc_ref(L, rank, size)
    elif mode == "testdim":
        test_dim_ref(L, rank, size)
    elif mode == "testvec":
        test_vector_ref(L, rank, size)
    elif mode in ("scatremote", "scatremote-gloo"):
        scatter_remote_test(L, rank, size)
    elif mode == "ngags":
        ngatest_gs(L, rank, size)
    elif mode == "armciacc":
        armci_test_acc_ref(L, rank, size)
    elif mode == "garef":
        ga_ref_test(L, rank, size)
    elif mode == "order":
        order_test(L, rank, size)
    elif mode == "selforder":
        self_order_test(L, rank, size)
    elif mode == "c1":
        c1_test(L, rank, size)
    elif mode == "onepass":
        one_pass_test(L, rank, size)
    elif mode == "hostself":
        host_self_test(L, rank, size)
    elif mode == "hostseg-ga":
        host_segment_ga_test(L, rank, size)
    elif mode == "c5full":
        c5_full_test(L, rank, size)
    elif mode == "directsrc":
        direct_src_test(L, rank, size)
    elif mode == "segcache":
        segment_cache_test(L, rank, size)
    elif mode == "stalefix":
        stale_fix_test(L, rank, size)
    elif mode == "oddseg":
        odd_segment_test(L, rank, size)
    elif mode == "xcheck":
        xcheck_test(L, rank, size)
    elif mode in ("armcimisc", "armcimisc-gloo"):
        armci_misc_test(L, rank, size)
    elif mode in ("rdesc", "rdesc-gloo"):
        random_remote_descriptors_test(L, rank, size)
    else:
        remote_test(L, rank, size)
    print(f"RANK {rank} OK", flush=True)


def say(rank, msg):
    print(f"rank {rank}: {msg}", file=sys.stderr, flush=True)


def remote_test(L, rank, size):
    import ga_amd
    from oracle import Oracle
    ora = Oracle()
    DBL = 38
    assert ga_amd.comex_init() == 0
    if os.environ.get("TEST_DISTINCT_DEVICES"):
        # one rank per GPU: the peer segments are opened by IPC on another device (xGMI)
        assert L.gaamd_device() == rank, (L.gaamd_device(), rank)
    # each rank owns a 300 x 260 f64 block (column-major, ld 300)
    ld, ncol = 300, 260
    nbytes = ld * ncol * 8
    seg = ga_amd.comex_malloc(nbytes, size)
    assert all(seg), seg
    base = np.arange(ld * ncol, dtype=np.float64) % 1000 + 1000 * rank     # integer-valued
    h = base.copy()
    assert ga_amd.lib().comex_put(h.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(seg[rank]), nbytes,
                                  rank, 0) == 0
    ga_amd.comex_barrier()

    # every rank accumulates the same integer-valued 120 x 90 patch into every
    # rank's block at (7, 11) with alpha = rank+1 (remote ranks through the
    # owner's progress thread, itself through the fused local kernel)
    src_ld = 128
    src = (np.arange(src_ld * 90, dtype=np.float64) % 97 - 48).reshape(90, src_ld)
    count = [120 * 8, 90]
    for t in range(size):
        off = (7 + 11 * ld) * 8
        rc = ga_amd.comex_accs(DBL, float(rank + 1), src.ctypes.data, [src_ld * 8], seg[t] + off, [ld * 8],
                               count, 1, t)
        assert rc == 0
    say(rank, "remote accs posted")
    # a strided put into the next rank and a get from the previous one
    nxt, prv = (rank + 1) % size, (rank - 1) % size
    patch = np.full((20, 16), 1e6 + rank, dtype=np.float64)
    put_off = (200 + 230 * ld) * 8 + rank * 16 * 8
    assert ga_amd.comex_puts(patch.ctypes.data, [16 * 8], seg[nxt] + put_off, [ld * 8], [16 * 8, 20], 1,
                             nxt) == 0
    ga_amd.comex_barrier()

    # check my block: base + sum_r (r+1) * src on the patch, puts from prev rank
    want = base.copy().view(np.uint8)
    total = float(sum(r + 1 for r in range(size)))
    ora.accs(DBL, total, src.reshape(-1).view(np.uint8), 0, [src_ld * 8], want, (7 + 11 * ld) * 8, [ld * 8],
             count, 1)
    ora.puts(np.full((20, 16), 1e6 + prv, dtype=np.float64).reshape(-1).view(np.uint8), 0, [16 * 8], want,
             (200 + 230 * ld) * 8 + prv * 16 * 8, [ld * 8], [16 * 8, 20], 1)
    got = np.zeros(ld * ncol, dtype=np.float64)
    assert ga_amd.lib().comex_get(ctypes.c_void_p(seg[rank]), got.ctypes.data_as(ctypes.c_void_p), nbytes,
                                  rank, 0) == 0
    ga_amd.comex_fence_all()
    if not np.array_equal(got.view(np.uint8), want):
        bad = np.nonzero(got != want.view(np.float64))[0]
        raise SystemExit(f"rank {rank}: {bad.size} elements differ, first {bad[:5]}")

    say(rank, "block checked")
    ga_amd.comex_barrier()   # nobody accumulates into a block (many-small below) while its owner checks it
    # remote strided get of the previous rank's patch
    out = np.zeros((90, 120), dtype=np.float64)
    assert ga_amd.comex_gets(seg[prv] + (7 + 11 * ld) * 8, [ld * 8], out.ctypes.data, [120 * 8], count, 1,
                             prv) == 0
    ga_amd.comex_fence_all()
    pb = (np.arange(ld * ncol, dtype=np.float64) % 1000 + 1000 * prv).reshape(ncol, ld)
    exp = pb[11:101, 7:127] + total * src[:, :120]
    assert np.array_equal(out, exp), f"rank {rank}: remote get mismatch"

    say(rank, "remote get checked")
    # many small remote accumulates in flight (inbox wrap, staging reuse)
    for it in range(300):
        t = (rank + 1 + it) % size
        assert ga_amd.comex_accs(DBL, 1.0, src.ctypes.data, [src_ld * 8], seg[t] + (250 * ld + 3) * 8,
                                 [ld * 8], [4 * 8, 3], 1, t) == 0
    ga_amd.comex_barrier()
    got2 = np.zeros(3 * ld, dtype=np.float64)
    assert ga_amd.lib().comex_get(ctypes.c_void_p(seg[rank] + 250 * ld * 8), got2.ctypes.data_as(ctypes.c_void_p),
                                  3 * ld * 8, rank, 0) == 0
    ga_amd.comex_fence_all()
    cnt_into_me = sum(1 for r in range(size) for it in range(300) if (r + 1 + it) % size == rank)
    exp2 = base.reshape(ncol, ld)[250:253].copy()
    exp2[:, 3:7] += cnt_into_me * src[:3, :4]
    assert np.array_equal(got2.reshape(3, ld), exp2), f"rank {rank}: many-small mismatch"

    say(rank, "many-small checked")
    # remote io-vector accumulate (scatter-acc with duplicates) into the next rank
    ga_amd.comex_barrier()
    vsrc = np.arange(64, dtype=np.float64) + 1.0 + rank
    vb = ga_amd.DeviceBuffer(vsrc.nbytes)
    vb.upload(vsrc)
    idx = [(7 * i) % 20 for i in range(64)]        # duplicates: 64 pairs onto 20 slots
    vbase = (260 * ld - 40) * 8                    # last 40 elements of my block stay free
    descs = [([vb.ptr + 8 * i for i in range(64)], [seg[nxt] + vbase + 8 * j for j in idx], 8)]
    assert ga_amd.comex_accv(DBL, 2.0, descs, nxt) == 0
    ga_amd.comex_barrier()
    tail = np.zeros(40, dtype=np.float64)
    assert ga_amd.lib().comex_get(ctypes.c_void_p(seg[rank] + vbase), tail.ctypes.data_as(ctypes.c_void_p), 320,
                                  rank, 0) == 0
    ga_amd.comex_fence_all()
    exp_t = base[-40:].copy()
    psrc = np.arange(64, dtype=np.float64) + 1.0 + prv
    for i, j in enumerate(idx):
        exp_t[j] += 2.0 * psrc[i]
    assert np.array_equal(tail, exp_t), f"rank {rank}: remote accv mismatch"

    # remote io-vector get of the next rank's tail (what I accumulated there)
    gb = ga_amd.DeviceBuffer(40 * 8)
    gdesc = [([seg[nxt] + vbase + 8 * j for j in range(40)], [gb.ptr + 8 * (39 - j) for j in range(40)], 8)]
    assert ga_amd.comex_getv(gdesc, nxt) == 0
    ga_amd.comex_fence_all()
    exp_n = (np.arange(ld * ncol, dtype=np.float64) % 1000 + 1000 * nxt)[-40:].copy()
    for i, j in enumerate(idx):
        exp_n[j] += 2.0 * vsrc[i]
    assert np.array_equal(gb.download(np.float64, 40)[::-1], exp_n), f"rank {rank}: remote getv mismatch"
    say(rank, "accv/getv checked")
    # remote io-vector put of 8 singles into the next rank's tail slots 32..39
    ga_amd.comex_barrier()
    pv = ga_amd.DeviceBuffer(64)
    pv.upload(np.arange(8, dtype=np.float64) - 100.0 * rank)
    pdesc = [([pv.ptr + 8 * i for i in range(8)], [seg[nxt] + vbase + 8 * (32 + i) for i in range(8)], 8)]
    assert ga_amd.comex_putv(pdesc, nxt) == 0
    ga_amd.comex_barrier()
    assert ga_amd.lib().comex_get(ctypes.c_void_p(seg[rank] + vbase), tail.ctypes.data_as(ctypes.c_void_p), 320,
                                  rank, 0) == 0
    ga_amd.comex_fence_all()
    assert np.array_equal(tail[32:], np.arange(8, dtype=np.float64) - 100.0 * prv), f"rank {rank}: putv"

    say(rank, "putv checked")
    # a remote accumulate larger than the staging sub-ring travels as row ranges
    # (pack -> staging slice -> owner's unpack-acc with a rebased packed base);
    # no chunk may fall back to the one-lane serial kernel, which a full-range
    # span of the rebased side once triggered (gaamd_kernels.hip range_span)
    ga_amd.comex_barrier()
    rows, rowb, ldb = 1024, 16384, 20480          # 16 MiB of payload per rank
    seg2 = ga_amd.comex_malloc(ldb * rows, size)
    ga_amd.lib().gaamd_memset(ctypes.c_void_p(seg2[rank]), 0, ldb * rows)

    def big_src(r):
        return (np.arange(rows * ldb // 8, dtype=np.float64) % 251 - 125 + r).reshape(rows, ldb // 8)
    bs = ga_amd.DeviceBuffer(ldb * rows)
    bs.upload(big_src(rank))
    ga_amd.sync()
    serial0 = ga_amd.kernel_counts()["serial"]
    ga_amd.comex_barrier()
    assert ga_amd.comex_accs(DBL, 2.0, bs.ptr, [ldb], seg2[nxt], [ldb], [rowb, rows], 1, nxt) == 0
    say(rank, "chunked remote acc posted")
    ga_amd.comex_barrier()
    mine = np.zeros((rows, ldb // 8), dtype=np.float64)
    assert ga_amd.lib().comex_get(ctypes.c_void_p(seg2[rank]), mine.ctypes.data_as(ctypes.c_void_p), ldb * rows,
                                  rank, 0) == 0
    ga_amd.comex_fence_all()
    exp3 = np.zeros_like(mine)
    exp3[:, :rowb // 8] = 2.0 * big_src(prv)[:, :rowb // 8]
    assert np.array_equal(mine, exp3), f"rank {rank}: chunked remote acc mismatch"
    assert ga_amd.kernel_counts()["serial"] == serial0, f"rank {rank}: a chunk ran on the serial kernel"
    bs.free()

    ga_amd.comex_barrier()
    assert ga_amd.comex_free(seg2[rank]) == 0
    assert ga_amd.comex_free(seg[rank]) == 0
    if os.environ.get("TEST_EXPECT_TOGGLES"):
        # COMEX_ENABLE_*_PACKED / _IOV / GET_SELF+SMP = 0: the routes they select ran
        tc = ga_amd.toggle_counts()
        assert tc["rows"] > 0 and tc["pairs"] > 0 and tc["owner_gets"] > 0, (rank, tc)
        say(rank, f"toggle routes {tc}")
    ga_amd.comex_finalize()


def order_test(L, rank, size):
    """A non-blocking HBM-source put of 32 MiB into the next rank's segment, then --
    with no fence -- a strided accumulate into the same patch.  The put kernel runs
    on this rank's stream through the IPC mapping, the accumulate is applied by the
    owner's progress thread on the owner's stream: the library must order the
    accumulate's pack (and so its post) after the put, as the reference's
    synchronous same-node put and accumulate are (comex.c:6084-6101, 6241-6260).
    The owner checks dst == A + 2*B bit for bit (one fixed order: put, then acc)."""
    import ga_amd
    DBL = 38
    assert ga_amd.comex_init() == 0
    rows, rowb, ldb = 1024, 32768, 32768 + 4096   # 32 MiB of payload, strided rows
    nbytes = rows * ldb
    seg = ga_amd.comex_malloc(nbytes, size)
    nxt, prv = (rank + 1) % size, (rank - 1) % size
    a, b = ga_amd.DeviceBuffer(nbytes), ga_amd.DeviceBuffer(nbytes)
    ss, cnt = ga_amd.int_array([ldb]), ga_amd.int_array([rowb, rows])
    for it in range(3):
        ga_amd.fill(a.ptr, nbytes // 8, 0, 7000 + 10 * rank + it)
        ga_amd.fill(b.ptr, nbytes // 8, 0, 8000 + 10 * rank + it)
        ga_amd.sync()
        ga_amd.comex_barrier()
        h = ctypes.c_int(-1)
        assert L.comex_nbputs(ctypes.c_void_p(a.ptr), ss, ctypes.c_void_p(seg[nxt]), ss, cnt, 1, nxt, 0,
                              ctypes.byref(h)) == 0
        assert ga_amd.comex_accs(DBL, 2.0, b.ptr, [ldb], seg[nxt], [ldb], [rowb, rows], 1, nxt) == 0
        assert L.comex_wait(ctypes.byref(h)) == 0
        ga_amd.comex_barrier()
        got = np.zeros(nbytes // 8, dtype=np.float64)
        assert L.comex_get(ctypes.c_void_p(seg[rank]), got.ctypes.data_as(ctypes.c_void_p), nbytes, rank, 0) == 0
        sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
        import cases as C
        A = C.fill_real(np.float64, nbytes // 8, 7000 + 10 * prv + it).reshape(rows, ldb // 8)
        B = C.fill_real(np.float64, nbytes // 8, 8000 + 10 * prv + it).reshape(rows, ldb // 8)
        g = got.reshape(rows, ldb // 8)[:, :rowb // 8]
        want = A[:, :rowb // 8] + B[:, :rowb // 8] * 2.0
        assert np.array_equal(g.view(np.uint64), want.view(np.uint64)), f"rank {rank}: round {it}: acc overtook put"
        say(rank, f"order round {it} checked")
    ga_amd.comex_barrier()
    assert ga_amd.comex_free(seg[rank]) == 0
    ga_amd.comex_finalize()


def one_pass_expected():
    """ranks on one GPU with the one-pass route enabled (see comex.cpp one_pass_acc)"""
    return (not os.environ.get("TEST_DISTINCT_DEVICES") and os.environ.get("COMEX_AMD_PEER_LOADS") != "all"
            and os.environ.get("COMEX_AMD_ONE_PASS", "1") != "0")


def one_pass_test(L, rank, size):
    """Ranks sharing one GPU: accumulates from plain device
    buffers into other ranks' segments take the one-pass route (the requester's
    fused kernel writes the owner's block under the owner's memory lock), while
    every owner keeps accumulating into its own block too.  Every rank adds the
    constant 2**rank into EVERY rank's 8 MiB block (itself included), ROUNDS
    times, blocking and non-blocking alternately, no barrier in between: a lost
    update (two unexcluded read-modify-writes of one element) shows as a wrong
    sum; each element must read exactly ROUNDS * (2**size - 1)."""
    import ga_amd
    DBL = 38
    assert ga_amd.comex_init() == 0
    n = 1 << 20                               # 8 MiB of f64 per block
    rounds = 12
    seg = ga_amd.comex_malloc(n * 8, size)
    zero = np.zeros(n)
    assert L.comex_put(zero.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(seg[rank]), n * 8, rank, 0) == 0
    ga_amd.comex_barrier()
    src = ga_amd.DeviceBuffer(n * 8)
    ga_amd.fill_const(src.ptr, n * 8, float(2 ** rank))
    ga_amd.sync()
    r0 = ga_amd.route_counts()
    one = ctypes.c_double(1.0)
    handles = []
    for it in range(rounds):
        for k in range(size):
            t = (rank + k + it) % size           # every rank visits the targets in a different order
            if it % 2:
                h = ctypes.c_int(-1)
                assert L.comex_nbacc(38, ctypes.byref(one), ctypes.c_void_p(src.ptr), ctypes.c_void_p(seg[t]), n * 8,
                                     t, 0, ctypes.byref(h)) == 0
                handles.append(h)
            else:
                assert L.comex_acc(DBL, ctypes.byref(one), ctypes.c_void_p(src.ptr), ctypes.c_void_p(seg[t]), n * 8,
                                   t, 0) == 0
        while len(handles) > 8:
            assert L.comex_wait(ctypes.byref(handles.pop(0))) == 0
    for h in handles:
        assert L.comex_wait(ctypes.byref(h)) == 0
    ga_amd.comex_barrier()
    r1 = ga_amd.route_counts()
    got = np.zeros(n)
    assert L.comex_get(ctypes.c_void_p(seg[rank]), got.ctypes.data_as(ctypes.c_void_p), n * 8, rank, 0) == 0
    want = float(rounds * (2 ** size - 1))
    bad = int(np.count_nonzero(got != want))
    assert bad == 0, f"rank {rank}: {bad} wrong, e.g. {got[np.nonzero(got != want)[0][0]]} != {want}"
    if size > 1 and one_pass_expected():
        assert r1["one_pass"] - r0["one_pass"] == rounds * (size - 1), (r0, r1)
    say(rank, f"one-pass exchange exact; routes {dict((k, r1[k] - r0[k]) for k in r1)}")
    src.free()
    ga_amd.comex_barrier()
    assert ga_amd.comex_free(seg[rank]) == 0
    ga_amd.comex_finalize()


def host_self_test(L, rank, size):
    """an owner accumulating into its OWN block from pageable host
    memory (the host-side route: its pages are registered for the call and the launch
    joins every library stream) while same-GPU peers accumulate large device-buffer
    patches into the same elements on the one-pass route (their kernels write the
    owner's segment under the owner's memory lock).  The owner's host-side launch
    must take its own memory lock too, or two read-modify-write kernels run on the
    same bytes at once and updates are lost.  Every rank adds 2**rank into rank 0's
    4 MiB block ROUNDS times with no barrier in between; each element must read
    exactly ROUNDS * (2**size - 1)."""
    import ga_amd
    DBL = 38
    assert ga_amd.comex_init() == 0
    n = 1 << 19                               # 4 MiB of f64: every peer call >= 64 KiB (one-pass)
    rounds = 24
    seg = ga_amd.comex_malloc(n * 8, size)
    zero = np.zeros(n)
    assert L.comex_put(zero.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(seg[rank]), n * 8, rank, 0) == 0
    ga_amd.comex_barrier()
    one = ctypes.c_double(1.0)
    r0 = ga_amd.route_counts()
    if rank == 0:
        for it in range(rounds):
            # a fresh pageable buffer each time: registered for the call only
            h = np.full(n, float(2 ** rank))
            assert L.comex_acc(DBL, ctypes.byref(one), h.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(seg[0]),
                               n * 8, 0, 0) == 0
    else:
        src = ga_amd.DeviceBuffer(n * 8)
        ga_amd.fill_const(src.ptr, n * 8, float(2 ** rank))
        ga_amd.sync()
        handles = []
        for it in range(rounds):
            h = ctypes.c_int(-1)
            assert L.comex_nbacc(DBL, ctypes.byref(one), ctypes.c_void_p(src.ptr), ctypes.c_void_p(seg[0]), n * 8,
                                 0, 0, ctypes.byref(h)) == 0
            handles.append(h)
            if len(handles) > 4:
                assert L.comex_wait(ctypes.byref(handles.pop(0))) == 0
        for h in handles:
            assert L.comex_wait(ctypes.byref(h)) == 0
        src.free()
    ga_amd.comex_barrier()
    r1 = ga_amd.route_counts()
    if rank == 0:
        got = np.zeros(n)
        assert L.comex_get(ctypes.c_void_p(seg[0]), got.ctypes.data_as(ctypes.c_void_p), n * 8, 0, 0) == 0
        want = float(rounds * (2 ** size - 1))
        bad = int(np.count_nonzero(got != want))
        assert bad == 0, f"owner block: {bad} wrong, e.g. {got[np.nonzero(got != want)[0][0]]} != {want}"
    elif one_pass_expected():
        assert r1["one_pass"] - r0["one_pass"] == rounds, (r0, r1)
    say(rank, "host-source self accumulates vs one-pass peers exact")
    ga_amd.comex_barrier()
    assert ga_amd.comex_free(seg[rank]) == 0
    ga_amd.comex_finalize()


def host_segment_ga_test(L, rank, size):
    """VERDICT r3 item 3, run with COMEX_AMD_SEGMENT=host: GA partitions in host
    segments (one POSIX shm object per rank, mapped and HIP-registered by every rank
    of the node), which GA's global/src dereferences on the host -- pnga_zero takes
    pnga_access_ptr and memsets the block (global.nalg.c:94-129).  Each rank fills its
    block on the HOST through NGA_Access; every rank reads the whole array back with
    NGA_Get (remote gets from other ranks' host segments); every rank NGA_Acc's the
    whole array (remote accumulates into host segments, applied by their owners) and
    each owner checks its block on the host; then each rank zeroes its block with a
    host memset through NGA_Access, exactly as pnga_zero, and the peers' NGA_Get must
    see zeros.  Integer-valued f64: exact."""
    import ga_amd
    ia = ga_amd.int_array
    C_DBL = 1004
    n, m = 1000, 700
    assert L.GA_Initialize() == 0
    g = L.NGA_Create(C_DBL, 2, ia([n, m]), b"hostseg", None)
    assert g > 0
    los, his = [], []
    for q in range(size):
        lo_, hi_ = (ctypes.c_int * 2)(), (ctypes.c_int * 2)()
        L.NGA_Distribution(g, q, lo_, hi_)
        los.append(list(lo_))
        his.append(list(hi_))
    blo, bhi = ia(los[rank]), ia(his[rank])
    rows, cols = his[rank][0] - los[rank][0] + 1, his[rank][1] - los[rank][1] + 1

    def access():
        ptr, ld = ctypes.c_void_p(), (ctypes.c_int * 1)()
        L.NGA_Access(g, blo, bhi, ctypes.byref(ptr), ld)
        assert ld[0] == cols, (ld[0], cols)
        assert L.gaamd_segment_kind(ptr) == 2, "the GA block is not in a host segment"
        return np.ctypeslib.as_array((ctypes.c_double * (rows * cols)).from_address(ptr.value)).reshape(rows, cols)

    def init_of(q):
        r_, c_ = his[q][0] - los[q][0] + 1, his[q][1] - los[q][1] + 1
        return 1000.0 * q + (np.arange(r_ * c_) % 997).reshape(r_, c_)

    def whole():
        out = np.empty(n * m)
        L.NGA_Get(g, ia([0, 0]), ia([n - 1, m - 1]), out.ctypes.data_as(ctypes.c_void_p), ia([m]))
        return out.reshape(n, m)

    blk = access()
    blk[:] = init_of(rank)               # host writes straight into the segment
    L.NGA_Release_update(g, blo, bhi)
    L.GA_Sync()
    got = whole()
    for q in range(size):
        sub = got[los[q][0]:his[q][0] + 1, los[q][1]:his[q][1] + 1]
        assert np.array_equal(sub, init_of(q)), f"rank {rank}: host-written block of rank {q} not seen by NGA_Get"
    say(rank, "host-written blocks read back through NGA_Get")
    # every rank accumulates the whole array: a device source of 2**rank and a pageable one of 3
    src = ga_amd.DeviceBuffer(n * m * 8)
    ga_amd.fill_const(src.ptr, n * m * 8, float(2 ** rank))
    ga_amd.sync()
    hsrc = np.full(n * m, 3.0)
    one = ctypes.c_double(1.0)
    L.NGA_Acc(g, ia([0, 0]), ia([n - 1, m - 1]), ctypes.c_void_p(src.ptr), ia([m]), ctypes.byref(one))
    L.NGA_Acc(g, ia([0, 0]), ia([n - 1, m - 1]), hsrc.ctypes.data_as(ctypes.c_void_p), ia([m]), ctypes.byref(one))
    L.GA_Sync()
    blk = access()                       # read on the host, after the owners applied everything
    want = init_of(rank) + float(2 ** size - 1) + 3.0 * size
    bad = int(np.count_nonzero(blk != want))
    assert bad == 0, f"rank {rank}: {bad} elements of the host block wrong after the accumulates"
    L.NGA_Release(g, blo, bhi)
    say(rank, "remote accumulates into host segments exact (checked on the host)")
    # pnga_zero's way: pnga_access_ptr + memset of the local block, then sync
    blk = access()
    ctypes.memset(blk.ctypes.data, 0, rows * cols * 8)
    L.NGA_Release_update(g, blo, bhi)
    L.GA_Sync()
    assert not np.any(whole()), f"rank {rank}: a peer's host memset is not visible through NGA_Get"
    # and the library's own GA_Zero on host segments after some data
    L.NGA_Acc(g, ia([0, 0]), ia([n - 1, m - 1]), ctypes.c_void_p(src.ptr), ia([m]), ctypes.byref(one))
    L.GA_Sync()
    L.GA_Zero(g)
    assert not np.any(whole()), f"rank {rank}: GA_Zero left data in a host segment"
    assert not np.any(access()), f"rank {rank}: GA_Zero not seen on the host"
    say(rank, "host memset through NGA_Access (pnga_zero) and GA_Zero visible to every rank")
    src.free()
    L.GA_Sync()
    L.GA_Destroy(g)
    L.GA_Terminate()


def c1_test(L, rank, size):
    """BASELINE config C1: 1-D contiguous f64 accumulate of 1 MiB
    (131 072 elements) between ranks, rank r -> rank (r+1) % size, the survey's
    synthetic data (splitmix64, seed 0x5EED0000 + rank, dst seed + 1; alpha =
    0.7071067811865476), bit-exact against the oracle's _acc (acc.h:137-143) on
    the same bytes.  One source per target, so the order is fixed and the f64
    result exact.  Three source kinds, each into a fresh dst: pageable host memory
    (MA-style, the packed route), a plain device buffer (packed route) and the
    rank's own segment (1 MiB: the direct-source route's threshold); the device
    buffer takes the one-pass route when both ranks share the GPU."""
    import ga_amd
    import cases as C
    from oracle import Oracle
    ora = Oracle()
    DBL, n = 38, 131072
    nbytes = n * 8
    alpha = 0.7071067811865476
    assert ga_amd.comex_init() == 0
    seg = ga_amd.comex_malloc(nbytes, size)
    srcseg = ga_amd.comex_malloc(nbytes, size)
    nxt, prv = (rank + 1) % size, (rank - 1) % size
    src = C.fill_real(np.float64, n, C.SEED + rank)
    dst0 = C.fill_real(np.float64, n, C.SEED + rank + 1)       # this rank's own dst (seed + 1)
    want = dst0.copy()
    ora_src = C.fill_real(np.float64, n, C.SEED + prv)         # what the previous rank sends us
    sc = np.array([alpha])
    dbuf = ga_amd.DeviceBuffer(nbytes)
    dbuf.upload(src)
    assert L.gaamd_memcpy(ctypes.c_void_p(srcseg[rank]), src.ctypes.data_as(ctypes.c_void_p), nbytes) == 0
    routes = []
    for kind in ("host", "device", "segment"):
        assert L.gaamd_memcpy(ctypes.c_void_p(seg[rank]), dst0.ctypes.data_as(ctypes.c_void_p), nbytes) == 0
        ga_amd.comex_barrier()
        r0 = ga_amd.route_counts()
        sp = {"host": src.ctypes.data, "device": dbuf.ptr, "segment": srcseg[rank]}[kind]
        assert ga_amd.comex_acc(DBL, alpha, sp, seg[nxt], nbytes, nxt) == 0
        ga_amd.comex_barrier()
        r1 = ga_amd.route_counts()
        routes.append((kind, {k: r1[k] - r0[k] for k in r1}))
        got = np.zeros(n)
        assert L.comex_get(ctypes.c_void_p(seg[rank]), got.ctypes.data_as(ctypes.c_void_p), nbytes, rank, 0) == 0
        w = dst0.copy()
        assert ora.L.ora_acc(DBL, nbytes, w.ctypes.data_as(ctypes.c_void_p), ora_src.ctypes.data_as(ctypes.c_void_p),
                             sc.ctypes.data_as(ctypes.c_void_p)) == 0
        assert np.array_equal(got.view(np.uint64), w.view(np.uint64)), f"rank {rank}: C1 {kind} source not bit-exact"
        ga_amd.comex_barrier()
    if size > 1:
        d = dict(routes)
        assert d["host"]["packed"] > 0, routes
        if one_pass_expected():
            # an owner on this GPU: the one-pass route for any device source
            assert d["device"]["one_pass"] > 0 and d["device"]["packed"] == 0, routes
            assert d["segment"]["one_pass"] > 0 and d["segment"]["direct_src"] == 0, routes
        else:
            assert d["device"]["packed"] > 0 and d["device"]["one_pass"] == 0, routes
            assert d["segment"]["direct_src"] > 0, routes
    say(rank, f"C1 1 MiB f64 remote acc bit-exact; routes {routes}")
    dbuf.free()
    ga_amd.comex_barrier()
    assert ga_amd.comex_free(srcseg[rank]) == 0
    assert ga_amd.comex_free(seg[rank]) == 0
    ga_amd.comex_finalize()


def c5_full_test(L, rank, size):
    """BASELINE config C5 at its stated size: NGA_Acc into a 32768 x 32768 f64 GA
    (8 GiB, REGULAR distribution over `size` ranks, ddb_h2 grid: 4 x 2 blocks of
    8192 x 16384 = 1 GiB at 8 ranks), every rank on this one GPU.
      M1: every rank NGA_Acc's its own block from a device buffer of the constant
          2**rank (alpha 1): the block must read 2**rank exactly.
      M2: every rank NGA_Acc's the WHOLE array from an 8 GiB source of 2**rank --
          even ranks from a plain device buffer, odd ranks from their own comex
          segment -- so every element must read exactly 2**size - 1; a lost, doubled
          or stale contribution shows as a wrong value that says whose
          (onesided.c:1387-1440; comex.c:6965-7109, 4133-4281).
    Which route M2 takes depends on where the owners are (asserted below): ranks
    sharing this GPU -- the one-pass route for every rank (the requester's kernel
    writes the owner's block under its memory lock); owners on other GPUs, or every
    peer treated as one (COMEX_AMD_PEER_LOADS=all) -- the packed route for the even
    ranks (pack -> staging -> the owner's unpack-acc pulling with system-scope loads)
    and the direct-source route for the odd ones (the owner reads the segment in
    place with system-scope loads)."""
    import time
    import ga_amd
    ia = ga_amd.int_array
    C_DBL = 1004
    n = int(os.environ.get("TEST_C5_N", "32768"))
    assert L.GA_Initialize() == 0
    if os.environ.get("TEST_DISTINCT_DEVICES"):
        assert L.gaamd_device() == rank, (L.gaamd_device(), rank)
    t0 = time.perf_counter()
    g = L.NGA_Create(C_DBL, 2, ia([n, n]), b"C5", None)
    assert g > 0
    blo, bhi = (ctypes.c_int * 2)(), (ctypes.c_int * 2)()
    L.NGA_Distribution(g, rank, blo, bhi)
    rows, cols = bhi[0] - blo[0] + 1, bhi[1] - blo[1] + 1
    if size == 8 and n == 32768:
        # ddb_h2's 4 x 2 grid in GA's Fortran order: C-order blocks of
        # 16384 rows x 8192 columns, ld 8192 (64 KiB), 1 GiB each
        assert (rows, cols) == (16384, 8192), (rows, cols)
    L.GA_Zero(g)
    L.GA_Sync()

    def check_block(want, what):
        out = np.empty(rows * cols)
        L.NGA_Get(g, blo, bhi, out.ctypes.data_as(ctypes.c_void_p), ia([cols]))
        bad = np.count_nonzero(out != want)
        assert bad == 0, f"rank {rank} {what}: {bad} wrong elements, e.g. {out[np.nonzero(out != want)[0][0]]} != {want}"

    # M1: own block, device-resident source
    one = ctypes.c_double(1.0)
    b1 = ga_amd.DeviceBuffer(rows * cols * 8)
    ga_amd.fill_const(b1.ptr, rows * cols * 8, float(2 ** rank))
    ga_amd.sync()
    L.GA_Sync()
    t1 = time.perf_counter()
    L.NGA_Acc(g, blo, bhi, ctypes.c_void_p(b1.ptr), ia([cols]), ctypes.byref(one))
    L.GA_Sync()
    t_m1 = time.perf_counter() - t1
    check_block(float(2 ** rank), "M1")
    b1.free()
    L.GA_Zero(g)
    L.GA_Sync()
    say(rank, f"C5 M1 exact ({rows}x{cols} block, {t_m1 * 1e3:.0f} ms)")

    # M2: the whole array from every rank; even ranks packed, odd ranks direct-source
    whole = n * n * 8
    use_seg = rank % 2 == 1
    seg = ga_amd.comex_malloc(whole if use_seg else 0, size)
    if use_seg:
        ptr, buf = seg[rank], None
    else:
        buf = ga_amd.DeviceBuffer(whole)
        ptr = buf.ptr
    ga_amd.fill_const(ptr, whole, float(2 ** rank))
    ga_amd.sync()
    L.GA_Sync()
    say(rank, f"C5 M2 sources ready ({time.perf_counter() - t0:.1f} s)")
    r0 = ga_amd.route_counts()
    t1 = time.perf_counter()
    L.NGA_Acc(g, ia([0, 0]), ia([n - 1, n - 1]), ctypes.c_void_p(ptr), ia([n]), ctypes.byref(one))
    L.GA_Sync()
    t_m2 = time.perf_counter() - t1
    r1 = ga_amd.route_counts()
    routes = {k: r1[k] - r0[k] for k in r1}
    check_block(float(2 ** size - 1), "M2")
    if size > 1:
        if one_pass_expected():
            assert routes["one_pass"] > 0 and routes["packed"] == 0 and routes["direct_src"] == 0, routes
        elif use_seg:
            assert routes["direct_src"] > 0 and routes["packed"] == 0 and routes["one_pass"] == 0, routes
        else:
            assert routes["packed"] > 0 and routes["direct_src"] == 0 and routes["one_pass"] == 0, routes
    L.GA_Sync()
    if buf is not None:
        buf.free()
    assert ga_amd.comex_free(seg[rank]) == 0
    L.GA_Destroy(g)
    route = "one-pass" if one_pass_expected() else ("direct-source" if use_seg else "packed")
    say(rank, f"C5 M2 exact ({route} route {routes}, {t_m2:.1f} s; total {time.perf_counter() - t0:.1f} s)")
    L.GA_Terminate()


def self_order_test(L, rank, size):
    """Run with COMEX_ENABLE_{ACC,PUT}_{SELF,SMP}=0: puts and accumulates to this
    rank's own segment take the packed route (the progress thread applies them
    after the call returns).  With NO barrier or fence in between, a put to self,
    then an accumulate to self, then a get / an io-vector get / an rmw on the same
    bytes must see them applied (the reference flushes before a
    self/SMP operation, comex.c:6073-6080, 6228-6235).  32 MiB patches, so the
    packed chunks are still in flight when the direct operation is issued.  Also,
    a same-node accumulate of >= 1 MiB from a segment source must take the packed
    route with COMEX_ENABLE_ACC_SMP=0 (comex.c:6911-6915), not the direct-source one."""
    import ga_amd
    DBL = 38
    assert ga_amd.comex_init() == 0
    n = 4 << 20                                   # 4 Mi f64 = 32 MiB
    seg = ga_amd.comex_malloc(n * 8, size)
    me = seg[rank]
    for it in range(3):
        a = (np.arange(n, dtype=np.float64) % 4093) + it
        b = (np.arange(n, dtype=np.float64) % 511) - 255
        assert L.comex_put(a.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(me), n * 8, rank, 0) == 0
        assert L.comex_acc(DBL, ctypes.byref(ctypes.c_double(3.0)), b.ctypes.data_as(ctypes.c_void_p),
                           ctypes.c_void_p(me), n * 8, rank, 0) == 0
        got = np.zeros(n, dtype=np.float64)
        assert L.comex_get(ctypes.c_void_p(me), got.ctypes.data_as(ctypes.c_void_p), n * 8, rank, 0) == 0
        want = a + 3.0 * b
        assert np.array_equal(got, want), f"rank {rank} round {it}: get overtook the packed put/acc to self"
        # the same through an io-vector get of the last 1000 elements
        a2 = a + 7
        assert L.comex_put(a2.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(me), n * 8, rank, 0) == 0
        tail = np.zeros(1000, dtype=np.float64)
        descs = [([me + (n - 1000 + i) * 8 for i in range(1000)], [tail.ctypes.data + i * 8 for i in range(1000)], 8)]
        assert ga_amd.comex_getv(descs, rank) == 0
        assert np.array_equal(tail, a2[-1000:]), f"rank {rank} round {it}: getv overtook the packed put to self"
        # and an rmw on the first word right after a packed put of it
        one = np.zeros(2, dtype=np.int64)
        one[0] = 40 + it
        assert L.comex_put(one.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(me), 16, rank, 0) == 0
        old = ctypes.c_long(0)
        assert L.comex_rmw(13, ctypes.byref(old), ctypes.c_void_p(me), 5, rank, 0) == 0   # COMEX_FETCH_AND_ADD_LONG
        assert old.value == 40 + it, (old.value, it)
    before = ga_amd.route_counts()
    ga_amd.comex_barrier()
    if size > 1:
        # >= 1 MiB same-node accumulate whose source is in our segment: with ACC_SMP=0 packed
        nxt = (rank + 1) % size
        src2 = ga_amd.comex_malloc(n * 8, size)
        assert L.comex_acc(DBL, ctypes.byref(ctypes.c_double(1.0)), ctypes.c_void_p(src2[rank]), ctypes.c_void_p(seg[nxt]),
                           n * 8, nxt, 0) == 0
        after = ga_amd.route_counts()
        assert after["direct_src"] == before["direct_src"] and after["packed"] > before["packed"], (before, after)
        ga_amd.comex_barrier()
        assert ga_amd.comex_free(src2[rank]) == 0
    ga_amd.comex_barrier()
    assert ga_amd.comex_free(me) == 0
    ga_amd.comex_finalize()


def stale_fix_test(L, rank, size):
    """TEST_STALE_GEN=2 (gaamd_diag "stale_gen"): every peer treats its first mapping of
    each rank's second segment as stale (the runtime binding a new block to other
    memory); or, with TEST_STALE_GRANULE=G too ("stale_granule"),
    every owner writes a foreign tag into granule G of that segment, an interior 2 MiB
    granule, so the peers' whole-block tag check has to find the mismatch itself.
    Either way every owner sets that block aside, allocates another and the exchange
    repeats.  Three segments (TEST_STALE_N f64 each), each accumulated into by its owner
    and the previous rank, checked exactly; the remap counter must show the replacement."""
    import ga_amd
    assert L.gaamd_diag(b"stale_gen", int(os.environ.get("TEST_STALE_GEN", "2")), None, 0) == 0
    assert L.gaamd_diag(b"stale_granule", int(os.environ.get("TEST_STALE_GRANULE", "-1")), None, 0) == 0
    assert ga_amd.comex_init() == 0
    r0 = L.gaamd_segment_remaps()
    one = ctypes.c_double(1.0)
    n = int(os.environ.get("TEST_STALE_N", str(1 << 18)))
    segs = []
    for it in range(3):
        seg = ga_amd.comex_malloc(n * 8, size)
        segs.append(seg)
        L.gaamd_memset(ctypes.c_void_p(seg[rank]), 0, n * 8)
        ga_amd.sync()
        ga_amd.comex_barrier()
        src = ga_amd.DeviceBuffer(n * 8)
        ga_amd.fill_const(src.ptr, n * 8, float(2 ** rank))
        ga_amd.sync()
        for t in {rank, (rank + 1) % size}:
            assert L.comex_acc(38, ctypes.byref(one), ctypes.c_void_p(src.ptr), ctypes.c_void_p(seg[t]), n * 8, t,
                               0) == 0
        ga_amd.comex_barrier()
        got = np.zeros(n)
        assert L.comex_get(ctypes.c_void_p(seg[rank]), got.ctypes.data_as(ctypes.c_void_p), n * 8, rank, 0) == 0
        prv = (rank - 1) % size
        want = float(2 ** rank + (2 ** prv if prv != rank else 0))
        bad = int(np.count_nonzero(got != want))
        assert bad == 0, f"rank {rank} segment {it}: {bad} wrong"
        src.free()
        ga_amd.comex_barrier()
    remaps = L.gaamd_segment_remaps() - r0
    assert remaps >= 1, f"rank {rank}: no segment replaced"
    for seg in segs:
        assert ga_amd.comex_free(seg[rank]) == 0
    say(rank, f"stale segment replaced ({remaps} remap), all exact")
    # the set-aside blocks go back at comex_finalize (GA_Terminate's path); without it the
    # process leaves through the exit hook (STALEFIX_NO_FINALIZE=1)
    if os.environ.get("STALEFIX_NO_FINALIZE") != "1":
        assert ga_amd.comex_finalize() == 0


def xcheck_test(L, rank, size):
    """ga_amd/xcheck.py, the check bench.py's N > 1 extras open with: every remote
    operation between rank pairs, exact by closed form, route counters summed over
    ranks.  XCHECK_DROP=N: the owners drop every N-th packed chunk (gaamd_diag
    "drop_chunk"), so the check must read MISMATCH and the conservative rerun must
    classify it "persists: logic".  Rank 0 prints the report as one XCHECK line."""
    import json
    import ga_amd
    from ga_amd.xcheck import xdev_check_diagnosed
    assert ga_amd.comex_init() == 0
    drop = int(os.environ.get("XCHECK_DROP", "0"))
    if drop:
        assert L.gaamd_diag(b"drop_chunk", drop, None, 0) == 0
    res = xdev_check_diagnosed(rank, size, seed=int(os.environ.get("XCHECK_SEED", "20260")), budget_s=90.0)
    if rank == 0:
        print("XCHECK " + json.dumps(res), flush=True)
    if drop:
        assert res["result"] == "MISMATCH", res
        assert res["diagnosis"].startswith("persists: logic"), res
        assert res["conservative_rerun"]["result"] == "MISMATCH"
        say(rank, "dropped chunks read MISMATCH, classified " + res["diagnosis"][:16])
    else:
        assert res["result"] == "exact", json.dumps(res)[:3000]
        routes = res["routes_all_ranks"]
        assert routes["peer_gets"] + routes["one_pass"] + routes["packed"] > 0, routes
        if L.gaamd_device_count() >= 1 and os.environ.get("COMEX_AMD_PEER_LOADS") == "all":
            # every peer another GPU: puts and accumulates packed, >= 1 MiB segment sources
            # direct, gets read with system-scope loads
            assert routes["packed"] > 0 and routes["direct_src"] > 0 and routes["peer_gets"] > 0, routes
            assert routes["owner_packed"] > 0 and routes["owner_direct_src"] > 0, routes
            assert routes["iov"] > 0 and routes["rmw"] > 0, routes
    ga_amd.comex_barrier()
    assert ga_amd.comex_finalize() == 0


def odd_segment_test(L, rank, size):
    """segments whose size is not a multiple of 8, just past a 2 MiB
    granule (2 MiB + 9..15 bytes put a granule tag and the end tag on shared bytes before
    the fix, so every peer found its mapping "stale" and comex_malloc aborted after four
    replacements), and small ones.  Each size: no block replaced, then every rank puts
    `bytes` bytes of its own pattern into the next rank's segment and reads its own back
    exactly, so the peers' mappings reach the owner's block end to end."""
    import ga_amd
    assert ga_amd.comex_init() == 0
    r0 = L.gaamd_segment_remaps()
    mib2 = 2 << 20
    for nbytes in (mib2 + 12, mib2 + 9, mib2 + 15, mib2 + 8, mib2 + 16, 2 * mib2 + 4, 16, 17, 23, 3):
        seg = ga_amd.comex_malloc(nbytes, size)
        assert L.gaamd_segment_remaps() == r0, f"rank {rank}: a {nbytes}-byte segment was replaced"
        nxt, prv = (rank + 1) % size, (rank - 1) % size
        pat = ((np.arange(nbytes, dtype=np.int64) * 7 + 13 * rank + nbytes) % 251).astype(np.uint8)
        assert L.comex_put(pat.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(seg[nxt]), nbytes, nxt, 0) == 0
        ga_amd.comex_fence_all()
        ga_amd.comex_barrier()
        got = np.zeros(nbytes, dtype=np.uint8)
        assert L.comex_get(ctypes.c_void_p(seg[rank]), got.ctypes.data_as(ctypes.c_void_p), nbytes, rank, 0) == 0
        want = ((np.arange(nbytes, dtype=np.int64) * 7 + 13 * prv + nbytes) % 251).astype(np.uint8)
        bad = int(np.count_nonzero(got != want))
        assert bad == 0, f"rank {rank}: {nbytes}-byte segment, {bad} bytes wrong"
        ga_amd.comex_barrier()
        assert ga_amd.comex_free(seg[rank]) == 0
    say(rank, "odd-size segments mapped without replacement, exact")
    assert ga_amd.comex_finalize() == 0


def segment_cache_test(L, rank, size):
    """comex_malloc / remote accumulates / comex_free of same-size segments, over and
    over (GA creating and destroying arrays): a freed block is kept with its IPC export
    and serves the next comex_malloc of its size, the peers opening it again from the
    same handle.  Every round: zero, every rank accumulates 2**rank into the next
    rank's block (one-pass or packed route) and into its own, barrier, exact check.
    A different size every third round takes a fresh block."""
    import ga_amd
    assert ga_amd.comex_init() == 0
    cache_on = os.environ.get("COMEX_AMD_SEGMENT_CACHE_MB", "1") != "0"   # both allocators cache
    reuse0 = L.gaamd_segment_cache_reuse()
    one = ctypes.c_double(1.0)
    for it in range(9):
        n = (1 << 18) if it % 3 != 2 else (1 << 18) + 512 * it   # f64 elements
        seg = ga_amd.comex_malloc(n * 8, size)
        L.gaamd_memset(ctypes.c_void_p(seg[rank]), 0, n * 8)
        ga_amd.sync()
        ga_amd.comex_barrier()
        src = ga_amd.DeviceBuffer(n * 8)
        ga_amd.fill_const(src.ptr, n * 8, float(2 ** rank))
        ga_amd.sync()
        for t in {rank, (rank + 1) % size}:
            assert L.comex_acc(38, ctypes.byref(one), ctypes.c_void_p(src.ptr), ctypes.c_void_p(seg[t]), n * 8, t,
                               0) == 0
        ga_amd.comex_barrier()
        got = np.zeros(n)
        assert L.comex_get(ctypes.c_void_p(seg[rank]), got.ctypes.data_as(ctypes.c_void_p), n * 8, rank, 0) == 0
        prv = (rank - 1) % size
        want = float(2 ** rank + (2 ** prv if prv != rank else 0))
        bad = int(np.count_nonzero(got != want))
        assert bad == 0, f"rank {rank} round {it}: {bad} wrong, e.g. {got[np.nonzero(got != want)[0][0]]} != {want}"
        src.free()
        ga_amd.comex_barrier()
        assert ga_amd.comex_free(seg[rank]) == 0
    reused = L.gaamd_segment_cache_reuse() - reuse0
    if cache_on:
        assert reused >= 5, f"rank {rank}: {reused} segments served from the cache"
    else:
        assert reused == 0, reused
    say(rank, f"segment cache: {reused} of 9 comex_malloc served by a kept block")
    ga_amd.comex_finalize()


def direct_src_test(L, rank, size):
    """Same-node accumulates whose source patch lies in the caller's own HBM
    segment: the owner applies them straight from that segment (kind-3 request,
    no pack pass).  Blocking and non-blocking, f64 and double complex, a patch
    below the direct route's 1 MiB floor (packed route), and the source
    overwritten right after the blocking call returns (the owner must have read
    it by then).  Integer-valued data: every order of the ranks' accumulates
    sums exactly; the result is checked against the oracle's restatement."""
    import ga_amd
    from oracle import Oracle
    ora = Oracle()
    DBL, DCP = 38, 41
    assert ga_amd.comex_init() == 0
    rows, ld = 512, 4096                      # 16 MiB segment: src half, dst half
    half = rows * ld * 8
    seg = ga_amd.comex_malloc(2 * half, size)
    nxt, prv = (rank + 1) % size, (rank - 1) % size

    def srcvals(r, it):
        return (np.arange(rows * ld, dtype=np.float64) % 61 - 30 + r + it).astype(np.float64)

    base = (np.arange(rows * ld, dtype=np.float64) % 7).astype(np.float64)
    counts0 = ga_amd.route_counts()
    for it, (op, alpha, rowb, nb) in enumerate([(DBL, 2.0, 2048 * 8, False), (DBL, -1.0, 3000 * 8, True),
                                                (DCP, 1 + 2j, 1024 * 16, False), (DBL, 3.0, 64 * 8, False)]):
        src_h = srcvals(rank, it)
        assert L.comex_put(src_h.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(seg[rank]), half, rank, 0) == 0
        b = base.copy()
        assert L.comex_put(b.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(seg[rank] + half), half, rank, 0) == 0
        ga_amd.comex_barrier()
        scale = ga_amd.scale_buffer(op, alpha)
        cnt = [rowb, rows]
        args = (op, scale[1], ctypes.c_void_p(seg[rank]), ga_amd.int_array([ld * 8]), ctypes.c_void_p(seg[nxt] + half),
                ga_amd.int_array([ld * 8]), ga_amd.int_array(cnt), 1, nxt, 0)
        if nb:
            h = ctypes.c_int(-1)
            assert L.comex_nbaccs(*args, ctypes.byref(h)) == 0
            assert L.comex_wait(ctypes.byref(h)) == 0
        else:
            assert L.comex_accs(*args) == 0
        # the source is reusable once the call (or its wait) returned
        junk = np.full(rows * ld, 1e300)
        assert L.comex_put(junk.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(seg[rank]), half, rank, 0) == 0
        ga_amd.comex_barrier()
        got = np.zeros(rows * ld, dtype=np.float64)
        assert L.comex_get(ctypes.c_void_p(seg[rank] + half), got.ctypes.data_as(ctypes.c_void_p), half, rank, 0) == 0
        want = base.copy().view(np.uint8)
        ora.accs(op, alpha, srcvals(prv, it).view(np.uint8), 0, [ld * 8], want, 0, [ld * 8], cnt, 1)
        assert np.array_equal(got.view(np.uint8), want), f"rank {rank}: case {it} differs"
        say(rank, f"direct-source case {it} checked")
    counts = ga_amd.route_counts()
    if size > 1:
        # with the owner on this GPU every case takes the one-pass route (the caller's
        # kernel, no owner hand-off; its floor is 64 KiB); otherwise the 64-column case
        # (256 KiB) is below the direct-source route's 1 MiB floor and packs
        if one_pass_expected():
            assert counts["one_pass"] - counts0["one_pass"] == 4, (counts0, counts)
        else:
            assert counts["direct_src"] - counts0["direct_src"] == 3, (counts0, counts)
            assert counts["packed"] > counts0["packed"]
    ga_amd.comex_barrier()
    assert ga_amd.comex_free(seg[rank]) == 0
    ga_amd.comex_finalize()


class MemInfo(ctypes.Structure):   # armci_meminfo_t (include/armci.h)
    _fields_ = [("armci_addr", ctypes.c_void_p), ("addr", ctypes.c_void_p), ("size", ctypes.c_size_t),
                ("cpid", ctypes.c_int), ("idlist", ctypes.c_long * 128)]


def armci_misc_test(L, rank, size):
    """The rest of the ARMCI surface GA calls: the message
    layer (message.c), processor groups (groups.c), rmw and mutexes (armci.c:
    282-292, 755-771), single values, flagged puts, domains, Memget and
    armci_read/write_strided -- each checked for its reference result."""
    import ga_amd
    c_int, byref, vp = ctypes.c_int, ctypes.byref, ctypes.c_void_p
    assert L.ARMCI_Init() == 0
    assert (L.armci_msg_me(), L.armci_msg_nproc()) == (rank, size)
    nxt, prv = (rank + 1) % size, (rank - 1) % size

    # point to point: a ring, then everybody to rank 0 through rcvany
    out = (c_int * 4)(*[100 * rank + i for i in range(4)])
    inp, ln = (c_int * 4)(), c_int()
    L.armci_msg_snd(77, out, 16, nxt)
    L.armci_msg_rcv(77, inp, 16, byref(ln), prv)
    assert ln.value == 16 and list(inp) == [100 * prv + i for i in range(4)], list(inp)
    if rank:
        L.armci_msg_snd(78, out, 8, 0)
    else:
        seen = set()
        for _ in range(size - 1):
            src = L.armci_msg_rcvany(78, inp, 16, byref(ln))
            assert ln.value == 8 and inp[0] == 100 * src and inp[1] == 100 * src + 1
            seen.add(src)
        assert seen == set(range(1, size))
    say(rank, "snd/rcv/rcvany")

    # gops (message.c:188-225)
    x = (c_int * 3)(rank + 1, rank, -rank)
    L.armci_msg_igop(x, 3, b"+")
    n1 = size * (size + 1) // 2
    assert list(x) == [n1, n1 - size, -(n1 - size)], list(x)
    x = (c_int * 2)(rank, -rank)
    L.armci_msg_igop(x, 2, b"max")
    assert list(x) == [size - 1, 0]
    lx = (ctypes.c_long * 1)(1 << rank)
    L.armci_msg_lgop(lx, 1, b"or")
    assert lx[0] == (1 << size) - 1
    llx = (ctypes.c_longlong * 1)(rank + 2)
    L.armci_msg_llgop(llx, 1, b"*")
    assert llx[0] == int(np.prod([r + 2 for r in range(size)]))
    fx = (ctypes.c_float * 1)(float(rank) + 0.5)
    L.armci_msg_fgop(fx, 1, b"min")
    assert fx[0] == 0.5
    dx = (ctypes.c_double * 2)(-(rank + 1.5), rank * 0.25)
    L.armci_msg_dgop(dx, 2, b"absmax")
    assert list(dx) == [size + 0.5, (size - 1) * 0.25], list(dx)
    dx = (ctypes.c_double * 1)(rank + 1.0)
    L.armci_msg_gop_scope(333, dx, 1, b"+", -307)
    assert dx[0] == float(n1)
    say(rank, "gops")

    # bcast from the last rank, sel by max / min of the leading value
    b = (ctypes.c_double * 3)(*([rank * 1.5] * 3))
    L.armci_msg_bcast(b, 24, size - 1)
    assert list(b) == [(size - 1) * 1.5] * 3
    sel = (c_int * 3)((rank * 7) % size, rank, 1000 + rank)
    L.armci_msg_sel_scope(333, sel, 12, b"max", -99, 1)
    winner = max(range(size), key=lambda r: ((r * 7) % size, -r))
    assert list(sel) == [(winner * 7) % size, winner, 1000 + winner], (list(sel), winner)
    sel = (c_int * 3)((rank * 7) % size, rank, 1000 + rank)
    L.armci_msg_sel_scope(333, sel, 12, b"min", -99, 1)
    winner = min(range(size), key=lambda r: ((r * 7) % size, r))
    assert list(sel) == [(winner * 7) % size, winner, 1000 + winner], (list(sel), winner)
    root, up, left, right = c_int(), c_int(), c_int(), c_int()
    L.armci_msg_bintree(333, byref(root), byref(up), byref(left), byref(right))
    want_l = 2 * rank + 1 if 2 * rank + 1 < size else -1
    want_r = 2 * rank + 2 if 2 * rank + 2 < size else -1
    # message.c:553 in C: (index-1)/2 truncates toward zero, so the root's Up is 0, not -1
    assert (root.value, up.value, left.value, right.value) == (0, int((rank - 1) / 2), want_l, want_r)
    addrs = (vp * size)()
    addrs[rank] = 0x1000 * (rank + 1)
    L.armci_exchange_address(addrs, size)
    assert [a or 0 for a in addrs] == [0x1000 * (r + 1) for r in range(size)]
    L.armci_msg_barrier()
    say(rank, "bcast/sel/bintree/exchange")

    # segments: values, rmw, mutexes, flagged puts
    seg = (vp * size)()
    nbytes = 1 << 20
    assert L.ARMCI_Malloc(seg, nbytes) == 0
    zero = np.zeros(nbytes // 8, dtype=np.int64)
    assert L.ARMCI_Put(zero.ctypes.data_as(vp), vp(seg[rank]), nbytes, rank) == 0
    L.ARMCI_Barrier()
    assert L.ARMCI_PutValueInt(1000 + rank, vp(seg[nxt] + 0), nxt) == 0
    assert L.ARMCI_PutValueLong(-(1 << 40) - rank, vp(seg[nxt] + 8), nxt) == 0
    assert L.ARMCI_PutValueFloat(0.25 + rank, vp(seg[nxt] + 16), nxt) == 0
    assert L.ARMCI_PutValueDouble(1e300 * (rank + 1), vp(seg[nxt] + 24), nxt) == 0
    h = c_int(-1)
    assert L.ARMCI_NbPutValueInt(7 + rank, vp(seg[nxt] + 32), nxt, byref(h)) == 0
    assert L.ARMCI_Wait(byref(h)) == 0
    L.ARMCI_Barrier()
    assert L.ARMCI_GetValueInt(vp(seg[rank] + 0), rank) == 1000 + prv
    assert L.ARMCI_GetValueLong(vp(seg[rank] + 8), rank) == -(1 << 40) - prv
    assert L.ARMCI_GetValueFloat(vp(seg[rank] + 16), rank) == 0.25 + prv
    assert L.ARMCI_GetValueDouble(vp(seg[rank] + 24), rank) == 1e300 * (prv + 1)
    assert L.ARMCI_GetValueInt(vp(seg[nxt] + 32), nxt) == 7 + rank
    say(rank, "put/get values")

    # fetch-and-add: every rank adds (rank+1) 50 times to rank 0's int and long
    FETCH_AND_ADD, FETCH_AND_ADD_LONG, SWAP, SWAP_LONG = 12, 13, 10, 11
    if rank == 0:   # a 64-bit base: the long form must carry past 32 bits (extra itself is an int)
        assert L.ARMCI_PutValueLong(1 << 40, vp(seg[0] + 72), 0) == 0
    L.ARMCI_Barrier()
    olds = []
    for _ in range(50):
        old = c_int()
        assert L.ARMCI_Rmw(FETCH_AND_ADD, byref(old), vp(seg[0] + 64), rank + 1, 0) == 0
        olds.append(old.value)
        oldl = ctypes.c_long()
        assert L.ARMCI_Rmw(FETCH_AND_ADD_LONG, byref(oldl), vp(seg[0] + 72), rank + 1, 0) == 0
        assert oldl.value >= 1 << 40
    assert len(set(olds)) == 50 and all(0 <= o < 50 * n1 for o in olds)
    L.ARMCI_Barrier()
    assert L.ARMCI_GetValueInt(vp(seg[0] + 64), 0) == 50 * n1
    assert L.ARMCI_GetValueLong(vp(seg[0] + 72), 0) == (1 << 40) + 50 * n1
    # swap: a token passes through every rank; the values seen are a permutation
    if rank == 0:
        assert L.ARMCI_PutValueInt(-1, vp(seg[0] + 80), 0) == 0
    L.ARMCI_Barrier()
    v = c_int(rank)
    assert L.ARMCI_Rmw(SWAP, byref(v), vp(seg[0] + 80), 0, 0) == 0
    got = (c_int * 1)(v.value)
    L.armci_msg_igop(got, 1, b"+")
    L.ARMCI_Barrier()
    last = L.ARMCI_GetValueInt(vp(seg[0] + 80), 0)
    assert got[0] + last == -1 + n1 - size, (got[0], last)
    vl = ctypes.c_long(5 << 40)
    if rank == size - 1:
        assert L.ARMCI_Rmw(SWAP_LONG, byref(vl), vp(seg[1 % size] + 88), 0, 1 % size) == 0
        assert vl.value == 0
    L.ARMCI_Barrier()
    assert L.ARMCI_GetValueLong(vp(seg[1 % size] + 88), 1 % size) == 5 << 40
    say(rank, "rmw")

    # mutexes: a get / +1 / put critical section on rank (size-1)'s counter
    assert L.ARMCI_Create_mutexes(3) == 0
    owner = size - 1
    for it in range(20):
        L.ARMCI_Lock(it % 3, owner)
        cur = L.ARMCI_GetValueLong(vp(seg[owner] + 128 + 8 * (it % 3)), owner)
        assert L.ARMCI_PutValueLong(cur + 1, vp(seg[owner] + 128 + 8 * (it % 3)), owner) == 0
        L.ARMCI_Unlock(it % 3, owner)
    L.ARMCI_Barrier()
    tot = sum(L.ARMCI_GetValueLong(vp(seg[owner] + 128 + 8 * k), owner) for k in range(3))
    assert tot == 20 * size, tot
    assert L.ARMCI_Destroy_mutexes() == 0
    say(rank, "mutexes")

    # flagged put: a strided patch then the flag; the receiver spins on its flag
    rows, rowb = 64, 512
    pat = np.arange(rows * rowb // 8, dtype=np.float64) + 1e6 * rank
    ss, ds, cnt = ga_amd.int_array([rowb]), ga_amd.int_array([2 * rowb]), ga_amd.int_array([rowb, rows])
    flag_off, data_off = 4096, 8192
    assert L.ARMCI_PutS_flag(pat.ctypes.data_as(vp), ss, vp(seg[nxt] + data_off), ds, cnt, 1,
                             ctypes.cast(vp(seg[nxt] + flag_off), ctypes.POINTER(c_int)), 1 + rank, nxt) == 0
    while L.ARMCI_GetValueInt(vp(seg[rank] + flag_off), rank) != 1 + prv:
        pass
    back = np.zeros(rows * 2 * rowb // 8, dtype=np.float64)
    assert L.ARMCI_Get(vp(seg[rank] + data_off), back.ctypes.data_as(vp), rows * 2 * rowb, rank) == 0
    want = np.arange(rows * rowb // 8, dtype=np.float64) + 1e6 * prv
    assert np.array_equal(back.reshape(rows, -1)[:, :rowb // 8].ravel(), want)
    L.ARMCI_Barrier()
    say(rank, "PutS_flag")

    # domains: one node here (or COMEX_AMD_NODE's binning)
    nd, nn, ns = c_int(), c_int(), c_int()
    L.gaamd_node_info(byref(nd), byref(nn), byref(ns))
    if nn.value == 1:
        assert L.armci_domain_count(0) == 1 and L.armci_domain_nprocs(0, 0) == size
        assert L.armci_domain_my_id(0) == 0 and L.armci_domain_id(0, prv) == 0
        assert all(L.armci_domain_same_id(0, q) for q in range(size))
        assert L.armci_domain_glob_proc_id(0, 0, size - 1) == size - 1
    assert L.ARMCI_Same_node(nxt) == 0 and L.ARMCI_Uses_shm() == 0

    # groups: the even ranks (groups.c); every rank creates it, members use it
    evens = [q for q in range(size) if q % 2 == 0]
    g = c_int()
    L.ARMCI_Group_create(len(evens), ga_amd.int_array(evens), byref(g))
    w = c_int()
    L.ARMCI_Group_get_world(byref(w))
    assert w.value == 0
    if rank % 2 == 0:
        gr, gs = c_int(), c_int()
        L.ARMCI_Group_rank(byref(g), byref(gr))
        L.ARMCI_Group_size(byref(g), byref(gs))
        assert (gr.value, gs.value) == (rank // 2, len(evens))
        assert L.ARMCI_Absolute_id(byref(g), gs.value - 1) == evens[-1]
        gx = (ctypes.c_double * 1)(rank + 1.0)
        L.armci_msg_group_dgop(gx, 1, b"+", byref(g))
        assert gx[0] == float(sum(q + 1 for q in evens))
        gi = (c_int * 1)(rank)
        L.armci_msg_group_igop(gi, 1, b"max", byref(g))
        assert gi[0] == evens[-1]
        gb = (c_int * 2)(rank, rank)
        L.armci_msg_group_bcast_scope(333, gb, 8, evens[-1], byref(g))
        assert list(gb) == [evens[-1]] * 2
        # GA's gai_get_shmem (base.c:3494-3512) on a group: ptr_arr[group rank] set, the
        # rest zero, then armci_exchange_address_grp fills every member's entry in
        # group-rank order (the reference's ComEx ARMCI aborts there, message.c:694-713,
        # whose disabled MPI_Allgather this implements)
        ga_addr = (vp * len(evens))()
        ga_addr[gr.value] = 0x5000 + 0x100 * rank
        L.armci_exchange_address_grp(ga_addr, len(evens), byref(g))
        assert [a or 0 for a in ga_addr] == [0x5000 + 0x100 * q for q in evens], list(ga_addr)
        gseg = (vp * len(evens))()
        assert L.ARMCI_Malloc_group(gseg, 4096, byref(g)) == 0
        peer = evens[(gr.value + 1) % len(evens)]
        assert L.ARMCI_PutValueInt(500 + rank, vp(gseg[(gr.value + 1) % len(evens)]), peer) == 0
        L.ARMCI_GroupFence(byref(g))
        L.armci_msg_group_barrier(byref(g))
        src_r = evens[(gr.value - 1) % len(evens)]
        assert L.ARMCI_GetValueInt(vp(gseg[gr.value]), rank) == 500 + src_r
        L.armci_msg_group_barrier(byref(g))
        assert L.ARMCI_Free_group(vp(gseg[gr.value]), byref(g)) == 0
    L.ARMCI_Barrier()
    L.ARMCI_Group_free(byref(g))
    say(rank, "groups")

    # Memget (armci.c:460-538) and armci_write/read_strided (iterator.c:158-193)
    mi = MemInfo()
    L.ARMCI_Memget(4096, byref(mi), 0)
    assert mi.size == 4096 and mi.cpid == rank and L.ARMCI_Memat(byref(mi), 0) == mi.addr
    ctypes.memset(mi.addr, 7, 4096)
    L.ARMCI_Memctl(byref(mi))
    patch = np.zeros((6, 10), dtype=np.float64)
    packed = np.arange(4 * 3, dtype=np.float64) + rank
    L.armci_write_strided(patch[1:, 2:].ctypes.data_as(vp), 1, ga_amd.int_array([80]), ga_amd.int_array([24, 4]),
                          packed.ctypes.data_as(vp))
    assert np.array_equal(patch[1:5, 2:5].ravel(), packed) and patch.sum() == packed.sum()
    back = np.zeros(12, dtype=np.float64)
    L.armci_read_strided(patch[1:, 2:].ctypes.data_as(vp), 1, ga_amd.int_array([80]), ga_amd.int_array([24, 4]),
                         back.ctypes.data_as(vp))
    assert np.array_equal(back, packed)
    say(rank, "memget/strided")

    ARMCI_ACC_DBL, ARMCI_LONG, ARMCI_DOUBLE, SCOPE_ALL = 38, -101, -307, 333   # armci.h, message.h
    # the rest of the one-sided surface GA links against: contiguous non-blocking put/get,
    # WaitProc, non-blocking single values, the contiguous flagged put, PutS_flag_dir,
    # non-blocking io-vectors, aggregate-handle no-ops, ARMCI_Test (armci.c / capi.c)
    base = 1 << 19
    pv = np.arange(512, dtype=np.float64) + 100.0 * rank
    h1, h2 = c_int(-1), c_int(-1)
    L.ARMCI_SET_AGGREGATE_HANDLE(byref(h1))
    assert L.ARMCI_NbPut(pv.ctypes.data_as(vp), vp(seg[nxt] + base), 4096, nxt, byref(h1)) == 0
    L.ARMCI_UNSET_AGGREGATE_HANDLE(byref(h1))
    assert L.ARMCI_Wait(byref(h1)) == 0
    hv = [c_int(-1) for _ in range(3)]
    assert L.ARMCI_NbPutValueLong(ctypes.c_long(-(3 << 33) - rank), vp(seg[nxt] + base + 4096), nxt, byref(hv[0])) == 0
    assert L.ARMCI_NbPutValueFloat(ctypes.c_float(1.5 + rank), vp(seg[nxt] + base + 4104), nxt, byref(hv[1])) == 0
    assert L.ARMCI_NbPutValueDouble(ctypes.c_double(2.25e-300 * (rank + 1)), vp(seg[nxt] + base + 4112), nxt,
                                    byref(hv[2])) == 0
    assert L.ARMCI_WaitProc(nxt) == 0
    for x in hv:
        assert L.ARMCI_Test(byref(x)) == 0   # complete: status 0
    L.ARMCI_Barrier()
    g1 = np.zeros(512)
    assert L.ARMCI_NbGet(vp(seg[rank] + base), g1.ctypes.data_as(vp), 4096, rank, byref(h2)) == 0
    assert L.ARMCI_Wait(byref(h2)) == 0
    assert np.array_equal(g1, np.arange(512) + 100.0 * prv)
    assert L.ARMCI_GetValueLong(vp(seg[rank] + base + 4096), rank) == -(3 << 33) - prv
    assert L.ARMCI_GetValueFloat(vp(seg[rank] + base + 4104), rank) == 1.5 + prv
    assert L.ARMCI_GetValueDouble(vp(seg[rank] + base + 4112), rank) == 2.25e-300 * (prv + 1)
    L.ARMCI_Barrier()
    # contiguous flagged put, then the strided one with the _dir form
    fl_off, d_off = base + 8192, base + 12288
    blob = np.arange(300, dtype=np.int32) * (rank + 3)
    assert L.ARMCI_Put_flag(blob.ctypes.data_as(vp), vp(seg[nxt] + d_off), blob.nbytes,
                            ctypes.cast(vp(seg[nxt] + fl_off), ctypes.POINTER(c_int)), 10 + rank, nxt) == 0
    while L.ARMCI_GetValueInt(vp(seg[rank] + fl_off), rank) != 10 + prv:
        pass
    rb = np.zeros(300, dtype=np.int32)
    assert L.ARMCI_Get(vp(seg[rank] + d_off), rb.ctypes.data_as(vp), rb.nbytes, rank) == 0
    assert np.array_equal(rb, np.arange(300, dtype=np.int32) * (prv + 3))
    L.ARMCI_Barrier()
    pat2 = np.arange(16 * 20, dtype=np.float64).reshape(16, 20) - rank
    assert L.ARMCI_PutS_flag_dir(pat2.ctypes.data_as(vp), ga_amd.int_array([160]), vp(seg[nxt] + d_off),
                                 ga_amd.int_array([320]), ga_amd.int_array([160, 16]), 1,
                                 ctypes.cast(vp(seg[nxt] + fl_off + 4), ctypes.POINTER(c_int)), 20 + rank, nxt) == 0
    while L.ARMCI_GetValueInt(vp(seg[rank] + fl_off + 4), rank) != 20 + prv:
        pass
    rb2 = np.zeros(16 * 40, dtype=np.float64)
    assert L.ARMCI_Get(vp(seg[rank] + d_off), rb2.ctypes.data_as(vp), rb2.nbytes, rank) == 0
    assert np.array_equal(rb2.reshape(16, 40)[:, :20], np.arange(16 * 20, dtype=np.float64).reshape(16, 20) - prv)
    L.ARMCI_Barrier()
    # non-blocking io-vectors: put 64 scattered doubles into nxt, accumulate them twice
    # more (alpha 2), get them back with NbGetV
    v_off = base + 65536
    nv = 64
    src = np.arange(nv, dtype=np.float64) + 10.0 * rank
    idx = (np.arange(nv) * 7) % 97
    s_arr = (vp * nv)(*[src.ctypes.data + 8 * i for i in range(nv)])
    d_arr = (vp * nv)(*[seg[nxt] + v_off + 8 * int(j) for j in idx])
    iov = ga_amd.GIOV()
    iov.src = ctypes.cast(s_arr, ctypes.POINTER(vp))
    iov.dst = ctypes.cast(d_arr, ctypes.POINTER(vp))
    iov.count, iov.bytes = nv, 8
    h3, h4, h5 = c_int(-1), c_int(-1), c_int(-1)
    assert L.ARMCI_NbPutV(byref(iov), 1, nxt, byref(h3)) == 0
    assert L.ARMCI_Wait(byref(h3)) == 0
    two = ctypes.c_double(2.0)
    assert L.ARMCI_NbAccV(ARMCI_ACC_DBL, byref(two), byref(iov), 1, nxt, byref(h4)) == 0
    assert L.ARMCI_Wait(byref(h4)) == 0
    L.ARMCI_AllFence()
    L.ARMCI_Barrier()
    out = np.zeros(nv)
    g_src = (vp * nv)(*[seg[rank] + v_off + 8 * int(j) for j in idx])
    g_dst = (vp * nv)(*[out.ctypes.data + 8 * i for i in range(nv)])
    giov = ga_amd.GIOV()
    giov.src = ctypes.cast(g_src, ctypes.POINTER(vp))
    giov.dst = ctypes.cast(g_dst, ctypes.POINTER(vp))
    giov.count, giov.bytes = nv, 8
    assert L.ARMCI_NbGetV(byref(giov), 1, rank, byref(h5)) == 0
    assert L.ARMCI_Wait(byref(h5)) == 0
    assert np.array_equal(out, 3.0 * (np.arange(nv) + 10.0 * prv)), out[:4]
    L.ARMCI_Barrier()
    say(rank, "nb put/get, values, flags, io-vectors")

    # processor groups through the ARMCI default / child forms and comex's own group API
    dflt, child = c_int(-1), c_int(-1)
    L.ARMCI_Group_get_default(byref(dflt))
    members = list(range(size - 1, -1, -1))            # every rank, in reverse order
    L.ARMCI_Group_create_child(size, ga_amd.int_array(members), byref(child), byref(dflt))
    cr, cs = c_int(), c_int()
    L.ARMCI_Group_rank(byref(child), byref(cr))
    L.ARMCI_Group_size(byref(child), byref(cs))
    assert (cr.value, cs.value) == (size - 1 - rank, size)
    L.ARMCI_Group_free(byref(child))
    cg = c_int(-1)
    assert L.comex_group_create(size, ga_amd.int_array(members), 0, byref(cg)) == 0
    gsz, wr = c_int(), c_int()
    assert L.comex_group_size(cg, byref(gsz)) == 0 and gsz.value == size
    assert L.comex_group_translate_world(cg, 0, byref(wr)) == 0 and wr.value == size - 1
    tr = (c_int * size)()
    assert L.comex_group_translate_ranks(size, cg, ga_amd.int_array(list(range(size))), 0, tr) == 0
    assert list(tr) == members
    assert L.comex_group_free(cg) == 0
    say(rank, "groups (default, child, comex)")

    # message layer: brdcst, reduce (+ scope), timer
    bb = (c_int * 4)(*([rank] * 4))
    L.armci_msg_brdcst(bb, 16, size - 1)
    assert list(bb) == [size - 1] * 4
    rx = (ctypes.c_long * 2)(rank, -rank)
    L.armci_msg_reduce(rx, 2, b"+", ARMCI_LONG)
    assert list(rx) == [sum(range(size)), -sum(range(size))]
    ry = (ctypes.c_double * 1)(float(rank))
    L.armci_msg_reduce_scope(SCOPE_ALL, ry, 1, b"max", ARMCI_DOUBLE)
    assert ry[0] == float(size - 1)
    t0 = L.armci_timer()
    t1 = L.armci_timer()
    assert t1 >= t0 > 0
    L.ARMCI_Barrier()
    say(rank, "brdcst/reduce/timer")

    L.ARMCI_Barrier()
    assert L.ARMCI_Free(vp(seg[rank])) == 0
    L.ARMCI_Finalize()


def ga_test(L, rank, size):
    """GA caller layer (onesided.c:1334-1453) on device partitions: NGA_Acc of a
    host patch spanning several owners, the testc.c:69-89 exact KAT, put/get,
    a 3-D int array, NGA_Access."""
    import ga_amd
    ia = ga_amd.int_array
    C_DBL, C_INT = 1004, 1001
    assert L.GA_Initialize() == 0
    assert L.GA_Nnodes() == size and L.GA_Nodeid() == rank
    dims = [300, 200]                          # C order: 300 rows x 200 columns
    g = L.NGA_Create(C_DBL, 2, ia(dims), b"a", None)
    assert g > 0
    # the blocks tile the array exactly
    cover = np.zeros(dims, dtype=np.int32)
    for p in range(size):
        lo, hi = (ctypes.c_int * 2)(), (ctypes.c_int * 2)()
        L.NGA_Distribution(g, p, lo, hi)
        if hi[0] >= lo[0]:
            cover[lo[0]:hi[0] + 1, lo[1]:hi[1] + 1] += 1
    assert (cover == 1).all(), "distribution does not tile the array"

    # every rank accumulates an integer-valued patch spanning several owners
    lo, hi = [10 + rank, 5], [250, 190]
    rows, cols = hi[0] - lo[0] + 1, hi[1] - lo[1] + 1
    ldc = cols + 3
    buf = (np.arange(rows * ldc, dtype=np.float64) % 37 - 18).reshape(rows, ldc)
    alpha = ctypes.c_double(rank + 1)
    L.NGA_Acc(g, ia(lo), ia(hi), buf.ctypes.data_as(ctypes.c_void_p), ia([ldc]), ctypes.byref(alpha))
    L.GA_Sync()
    say(rank, "ga sync 1")
    if rank == 0:
        got = np.zeros(dims, dtype=np.float64)
        L.NGA_Get(g, ia([0, 0]), ia([dims[0] - 1, dims[1] - 1]), got.ctypes.data_as(ctypes.c_void_p), ia([dims[1]]))
        want = np.zeros(dims)
        for r in range(size):
            lo_r = [10 + r, 5]
            rr = hi[0] - lo_r[0] + 1
            b = (np.arange(rr * (cols + 3), dtype=np.float64) % 37 - 18).reshape(rr, cols + 3)
            want[lo_r[0]:hi[0] + 1, lo_r[1]:hi[1] + 1] += (r + 1) * b[:, :cols]
        assert np.array_equal(got, want), "NGA_Acc result differs"
    L.GA_Sync()
    say(rank, "ga sync 2")

    # testc.c:69-89: everybody accumulates buf[i] = i into the same row, alpha 1
    L.GA_Zero(g)
    row = dims[0] // 2
    b = np.arange(dims[1], dtype=np.float64)
    one = ctypes.c_double(1.0)
    L.NGA_Acc(g, ia([row, 0]), ia([row, dims[1] - 1]), b.ctypes.data_as(ctypes.c_void_p), ia([dims[1]]),
              ctypes.byref(one))
    L.GA_Sync()
    say(rank, "ga sync 3")
    if rank == 0:
        out = np.zeros(dims[1])
        L.NGA_Get(g, ia([row, 0]), ia([row, dims[1] - 1]), out.ctypes.data_as(ctypes.c_void_p), ia([dims[1]]))
        assert np.array_equal(out, size * np.arange(dims[1], dtype=np.float64)), "testc.c KAT failed"
    L.GA_Sync()
    say(rank, "ga sync 4")

    # put / get round trip of a patch owned by several ranks
    p = (np.arange(40 * 50, dtype=np.float64) + 1e5 * (rank + 1)).reshape(40, 50)
    plo, phi = [100 + 45 * rank, 60], [139 + 45 * rank, 109]
    if phi[0] < dims[0]:
        L.NGA_Put(g, ia(plo), ia(phi), p.ctypes.data_as(ctypes.c_void_p), ia([50]))
    L.GA_Sync()
    say(rank, "ga sync 5")
    q = np.zeros((40, 50))
    if phi[0] < dims[0]:
        L.NGA_Get(g, ia(plo), ia(phi), q.ctypes.data_as(ctypes.c_void_p), ia([50]))
        if not np.array_equal(p, q):
            # diagnostics: the same get again into host memory, and into HBM
            q2 = np.zeros((40, 50))
            L.NGA_Get(g, ia(plo), ia(phi), q2.ctypes.data_as(ctypes.c_void_p), ia([50]))
            qd = ga_amd.DeviceBuffer(q2.nbytes)
            L.NGA_Get(g, ia(plo), ia(phi), ctypes.c_void_p(qd.ptr), ia([50]))
            q3 = qd.download(np.float64, 2000).reshape(40, 50)
            say(rank, f"retry host get ok={np.array_equal(p, q2)}, device get ok={np.array_equal(p, q3)}")
            bad = np.argwhere(p != q)
            rows_bad = sorted(set(int(x) for x in bad[:, 0]))
            raise AssertionError(f"put/get round trip: {len(bad)} differ, rows {rows_bad[:10]}.., cols "
                                 f"{sorted(set(int(x) for x in bad[:, 1]))[:10]}.., first got {q[tuple(bad[0])]} "
                                 f"want {p[tuple(bad[0])]}")

    # strided (skip) accumulate / put / get (pnga_strided_*, onesided.c:4225-4470):
    # every rank accumulates every 3rd row and 2nd column of [7..290] x [4..195]
    L.GA_Zero(g)
    slo, shi, skip = [7, 4], [290, 195], [3, 2]
    n0, n1 = (shi[0] - slo[0]) // skip[0] + 1, (shi[1] - slo[1]) // skip[1] + 1
    sld = n1 + 5
    sbuf = (np.arange(n0 * sld, dtype=np.float64) % 29 - 14 + rank).reshape(n0, sld)
    salpha = ctypes.c_double(rank + 2)
    L.NGA_Strided_acc(g, ia(slo), ia(shi), ia(skip), sbuf.ctypes.data_as(ctypes.c_void_p), ia([sld]),
                      ctypes.byref(salpha))
    L.GA_Sync()
    full = np.zeros(dims)
    L.NGA_Get(g, ia([0, 0]), ia([dims[0] - 1, dims[1] - 1]), full.ctypes.data_as(ctypes.c_void_p), ia([dims[1]]))
    want = np.zeros(dims)
    for r_ in range(size):
        b_ = (np.arange(n0 * sld, dtype=np.float64) % 29 - 14 + r_).reshape(n0, sld)
        want[slo[0]:shi[0] + 1:skip[0], slo[1]:shi[1] + 1:skip[1]] += (r_ + 2) * b_[:, :n1]
    assert np.array_equal(full, want), "NGA_Strided_acc"
    L.GA_Sync()
    say(rank, "strided acc checked")
    # rank 0 strided-puts every 2nd row/5th column, everybody strided-gets it back
    L.GA_Zero(g)
    plo2, phi2, pskip = [1, 0], [298, 199], [2, 5]
    m0, m1 = (phi2[0] - plo2[0]) // pskip[0] + 1, (phi2[1] - plo2[1]) // pskip[1] + 1
    pv = (np.arange(m0 * m1, dtype=np.float64) + 0.5).reshape(m0, m1)
    if rank == 0:
        L.NGA_Strided_put(g, ia(plo2), ia(phi2), ia(pskip), pv.ctypes.data_as(ctypes.c_void_p), ia([m1]))
    L.GA_Sync()
    gv = np.zeros((m0, m1))
    L.NGA_Strided_get(g, ia(plo2), ia(phi2), ia(pskip), gv.ctypes.data_as(ctypes.c_void_p), ia([m1]))
    assert np.array_equal(gv, pv), "NGA_Strided_put/get"
    L.NGA_Get(g, ia([0, 0]), ia([dims[0] - 1, dims[1] - 1]), full.ctypes.data_as(ctypes.c_void_p), ia([dims[1]]))
    want = np.zeros(dims)
    want[plo2[0]:phi2[0] + 1:pskip[0], plo2[1]:phi2[1] + 1:pskip[1]] = pv
    assert np.array_equal(full, want), "NGA_Strided_put layout"
    L.GA_Sync()
    say(rank, "strided put/get checked")

    # non-blocking acc / put / get (pnga_nbacc/nbput/nbget + pnga_nbwait)
    L.GA_Zero(g)
    nbh = ctypes.c_long(0)
    L.NGA_NbAcc(g, ia(lo), ia(hi), buf.ctypes.data_as(ctypes.c_void_p), ia([ldc]), ctypes.byref(alpha),
                ctypes.byref(nbh))
    L.NGA_NbWait(ctypes.byref(nbh))
    assert nbh.value == 0
    L.GA_Sync()
    L.NGA_Get(g, ia([0, 0]), ia([dims[0] - 1, dims[1] - 1]), full.ctypes.data_as(ctypes.c_void_p), ia([dims[1]]))
    want = np.zeros(dims)
    for r_ in range(size):
        lo_r = [10 + r_, 5]
        rr = hi[0] - lo_r[0] + 1
        b_ = (np.arange(rr * (cols + 3), dtype=np.float64) % 37 - 18).reshape(rr, cols + 3)
        want[lo_r[0]:hi[0] + 1, lo_r[1]:hi[1] + 1] += (r_ + 1) * b_[:, :cols]
    assert np.array_equal(full, want), "NGA_NbAcc"
    L.GA_Sync()
    np_ = (np.arange(40 * 50, dtype=np.float64) - 7e4 * (rank + 1)).reshape(40, 50)
    if phi[0] < dims[0]:
        h1, h2 = ctypes.c_long(0), ctypes.c_long(0)
        L.NGA_NbPut(g, ia(plo), ia(phi), np_.ctypes.data_as(ctypes.c_void_p), ia([50]), ctypes.byref(h1))
        L.NGA_NbWait(ctypes.byref(h1))
        nq = np.zeros((40, 50))
        L.NGA_NbGet(g, ia(plo), ia(phi), nq.ctypes.data_as(ctypes.c_void_p), ia([50]), ctypes.byref(h2))
        L.NGA_NbWait(ctypes.byref(h2))
        assert np.array_equal(nq, np_), "NGA_NbPut/NbGet round trip"
    L.GA_Sync()
    say(rank, "nb acc/put/get checked")

    # gather / scatter / scatter-acc (gai_gatscat, onesided.c:2747): random
    # subscripts over every owner, repeated ones included
    L.GA_Zero(g)
    rng = np.random.default_rng(50 + rank)
    nv = 500
    subs = np.stack([rng.integers(0, dims[0], nv), rng.integers(0, dims[1], nv)], axis=1).astype(np.int32)
    subs[nv // 2:nv // 2 + 40] = subs[:40]                     # repeats
    ptrs = (ctypes.POINTER(ctypes.c_int) * nv)(*[subs[k].ctypes.data_as(ctypes.POINTER(ctypes.c_int))
                                                  for k in range(nv)])
    vals = (rng.integers(-50, 50, nv)).astype(np.float64)     # integer-valued: any rank order is exact
    two = ctypes.c_double(2.0)
    L.NGA_Scatter_acc(g, vals.ctypes.data_as(ctypes.c_void_p), ptrs, nv, ctypes.byref(two))
    L.GA_Sync()
    say(rank, "ga sync 6")
    full = np.zeros(dims)
    L.NGA_Get(g, ia([0, 0]), ia([dims[0] - 1, dims[1] - 1]), full.ctypes.data_as(ctypes.c_void_p), ia([dims[1]]))
    want = np.zeros(dims)
    for r in range(size):
        rr = np.random.default_rng(50 + r)
        sb = np.stack([rr.integers(0, dims[0], nv), rr.integers(0, dims[1], nv)], axis=1)
        sb[nv // 2:nv // 2 + 40] = sb[:40]
        vv = rr.integers(-50, 50, nv).astype(np.float64)
        for k in range(nv):
            want[sb[k, 0], sb[k, 1]] += 2.0 * vv[k]
    assert np.array_equal(full, want), "NGA_Scatter_acc (integer-valued) differs"
    # gather the same subscripts (flat form) and compare with the full copy
    got = np.zeros(nv)
    L.NGA_Gather_flat(g, got.ctypes.data_as(ctypes.c_void_p), subs.ravel().ctypes.data_as(ctypes.POINTER(ctypes.c_int)), nv)
    assert np.array_equal(got, full[subs[:, 0], subs[:, 1]]), "NGA_Gather_flat"
    got2 = np.zeros(nv)
    L.NGA_Gather(g, got2.ctypes.data_as(ctypes.c_void_p), ptrs, nv)
    assert np.array_equal(got2, got), "NGA_Gather"
    L.GA_Sync()
    say(rank, "ga sync 7")
    # rank 0 alone: non-integer values with repeated subscripts, applied in input
    # order per owner -> bit-exact against the sequential _acc order
    L.GA_Zero(g)
    if rank == 0:
        fv = rng.standard_normal(nv) * 1e3
        alpha = 0.7071067811865476
        a_c = ctypes.c_double(alpha)
        L.NGA_Scatter_acc_flat(g, fv.ctypes.data_as(ctypes.c_void_p),
                               subs.ravel().ctypes.data_as(ctypes.POINTER(ctypes.c_int)), nv, ctypes.byref(a_c))
        exp = {}
        for k in range(nv):
            key = (int(subs[k, 0]), int(subs[k, 1]))
            exp[key] = exp.get(key, 0.0) + float(fv[k]) * alpha
        got3 = np.zeros(nv)
        L.NGA_Gather(g, got3.ctypes.data_as(ctypes.c_void_p), ptrs, nv)
        want3 = np.array([exp[(int(subs[k, 0]), int(subs[k, 1]))] for k in range(nv)])
        assert np.array_equal(got3.view(np.int64), want3.view(np.int64)), "NGA_Scatter_acc order"
    L.GA_Sync()
    say(rank, "ga sync 8")
    # scatter (put) of unique subscripts
    L.GA_Zero(g)
    rs = np.random.default_rng(77)                              # same subscripts on every rank
    uniq = np.unique(np.stack([rs.integers(0, dims[0], 300), rs.integers(0, dims[1], 300)], axis=1).astype(np.int32),
                     axis=0)
    if rank == size - 1:
        uv = np.arange(1, len(uniq) + 1, dtype=np.float64) * 1.5
        L.NGA_Scatter_flat(g, uv.ctypes.data_as(ctypes.c_void_p),
                           np.ascontiguousarray(uniq).ravel().ctypes.data_as(ctypes.POINTER(ctypes.c_int)), len(uniq))
    L.GA_Sync()
    say(rank, "ga sync 9")
    L.NGA_Get(g, ia([0, 0]), ia([dims[0] - 1, dims[1] - 1]), full.ctypes.data_as(ctypes.c_void_p), ia([dims[1]]))
    want = np.zeros(dims)
    want[uniq[:, 0], uniq[:, 1]] = np.arange(1, len(uniq) + 1) * 1.5
    assert np.array_equal(full, want), "NGA_Scatter"
    L.GA_Sync()
    say(rank, "ga sync 10")
    # large calls: owners located and pairs grouped by several host threads
    # (one per 128 Ki elements); rank 0 alone, 1 Mi non-integer values onto the
    # 60 000 elements of every owner (~17 repeats each) -> bit-exact against
    # the sequential mul-then-add order (np.add.at applies repeats in order)
    L.GA_Zero(g)
    if rank == 0:
        nbig = 1 << 20
        rb = np.random.default_rng(91)
        bsub = np.stack([rb.integers(0, dims[0], nbig), rb.integers(0, dims[1], nbig)], axis=1).astype(np.int32)
        bv = rb.standard_normal(nbig) * 1e3
        alpha = 0.7071067811865476
        L.NGA_Scatter_acc_flat(g, bv.ctypes.data_as(ctypes.c_void_p),
                               bsub.ravel().ctypes.data_as(ctypes.POINTER(ctypes.c_int)), nbig,
                               ctypes.byref(ctypes.c_double(alpha)))
        wb = np.zeros(dims)
        np.add.at(wb, (bsub[:, 0], bsub[:, 1]), bv * alpha)
        L.NGA_Get(g, ia([0, 0]), ia([dims[0] - 1, dims[1] - 1]), full.ctypes.data_as(ctypes.c_void_p),
                  ia([dims[1]]))
        assert np.array_equal(full.view(np.int64), wb.view(np.int64)), "large NGA_Scatter_acc_flat"
        gb = np.zeros(nbig)
        L.NGA_Gather_flat(g, gb.ctypes.data_as(ctypes.c_void_p),
                          bsub.ravel().ctypes.data_as(ctypes.POINTER(ctypes.c_int)), nbig)
        assert np.array_equal(gb.view(np.int64), wb[bsub[:, 0], bsub[:, 1]].view(np.int64)), "large NGA_Gather_flat"
    L.GA_Sync()
    say(rank, "ga sync 10b")

    # local block through NGA_Access is an HBM address
    lo_m, hi_m = (ctypes.c_int * 2)(), (ctypes.c_int * 2)()
    L.NGA_Distribution(g, rank, lo_m, hi_m)
    if hi_m[0] >= lo_m[0]:
        ptr, ld = ctypes.c_void_p(), (ctypes.c_int * 1)()
        L.NGA_Access(g, lo_m, hi_m, ctypes.byref(ptr), ld)
        nr, nc = hi_m[0] - lo_m[0] + 1, hi_m[1] - lo_m[1] + 1
        assert ld[0] == nc
        mine = np.zeros(nr * nc)
        assert L.gaamd_memcpy(mine.ctypes.data_as(ctypes.c_void_p), ptr, mine.nbytes) == 0
        ref = np.zeros((nr, nc))
        L.NGA_Get(g, lo_m, hi_m, ref.ctypes.data_as(ctypes.c_void_p), ia([nc]))
        assert np.array_equal(mine.reshape(nr, nc), ref)
        L.NGA_Release(g, lo_m, hi_m)
    L.GA_Sync()
    say(rank, "ga sync 11")
    L.GA_Destroy(g)

    # 3-D int array, accumulate with alpha 3 (integer arithmetic, exact)
    d3 = [17, 23, 29]
    g3 = L.NGA_Create(C_INT, 3, ia(d3), b"i3", None)
    v = (np.arange(10 * 12 * 14, dtype=np.int32) % 11 - 5).reshape(10, 12, 14)
    three = ctypes.c_int(3)
    L.NGA_Acc(g3, ia([3, 5, 7]), ia([12, 16, 20]), v.ctypes.data_as(ctypes.c_void_p), ia([12, 14]),
              ctypes.byref(three))
    L.GA_Sync()
    say(rank, "ga sync 12")
    out3 = np.zeros(d3, dtype=np.int32)
    L.NGA_Get(g3, ia([0, 0, 0]), ia([16, 22, 28]), out3.ctypes.data_as(ctypes.c_void_p), ia([23, 29]))
    w3 = np.zeros(d3, dtype=np.int32)
    w3[3:13, 5:17, 7:21] = 3 * size * v
    assert np.array_equal(out3, w3), "3-D int NGA_Acc"
    L.GA_Sync()
    say(rank, "ga sync 13")
    L.GA_Destroy(g3)
    ga_irregular_test(L, rank, size)
    if rank == 0:
        L.GA_Print_stats()
    L.GA_Terminate()


def ga_irregular_test(L, rank, size):
    """NGA_Create_irreg (capi.c:244-265 + copy_map): random block boundaries per
    dimension, blocks owned in GA's order (the Fortran-first dimension, i.e. the last C
    dimension, fastest: ga_ComputeIndexM), possibly fewer blocks than ranks (those own
    nothing).  Every rank accumulates a random patch (integer-valued: exact in any order),
    rank 0 puts one, all get them back, and a scatter-accumulate with repeats lands on
    the right owners."""
    import ga_amd
    ia = ga_amd.int_array
    C_DBL = 1004
    rng = np.random.default_rng(41)                      # the same on every rank
    dims = [97, 61, 13]
    # 3 ranks: two blocks, so rank 2 owns nothing
    nblk = {1: [1, 1, 1], 2: [1, 2, 1], 3: [2, 1, 1], 4: [2, 1, 2]}.get(size, [2, 2, 2] if size >= 8 else [2, 2, 1])
    maps = []
    for d, b in enumerate(nblk):
        starts = np.sort(rng.choice(np.arange(1, dims[d]), b - 1, replace=False)) if b > 1 else np.array([], int)
        maps.append([0] + [int(x) for x in starts])
    flat = [x for m in maps for x in m]
    g = L.NGA_Create_irreg(C_DBL, 3, ia(dims), b"irr", ia(nblk), ia(flat))
    assert g > 0
    # ownership: block (i0, i1, i2) in C order belongs to rank i2 + nb2 * (i1 + nb1 * i0)
    bounds = [m + [dims[d]] for d, m in enumerate(maps)]
    for p in range(size):
        lo, hi = (ctypes.c_int * 3)(), (ctypes.c_int * 3)()
        L.NGA_Distribution(g, p, lo, hi)
        nb = nblk[0] * nblk[1] * nblk[2]
        if p >= nb:   # ga_ownsM_no_handle (base.h:157-161): lo 0, hi -1 in Fortran, C lo -1, hi -2
            assert list(lo) == [-1] * 3 and list(hi) == [-2] * 3, (p, list(lo), list(hi))
            continue
        i2, r = p % nblk[2], p // nblk[2]
        i1, i0 = r % nblk[1], r // nblk[1]
        want_lo = [bounds[0][i0], bounds[1][i1], bounds[2][i2]]
        want_hi = [bounds[0][i0 + 1] - 1, bounds[1][i1 + 1] - 1, bounds[2][i2 + 1] - 1]
        assert list(lo) == want_lo and list(hi) == want_hi, (p, list(lo), list(hi), want_lo, want_hi)
    L.GA_Zero(g)

    def patch(r):
        pr = np.random.default_rng(300 + r)
        lo = [int(pr.integers(0, dims[d])) for d in range(3)]
        hi = [int(pr.integers(lo[d], dims[d])) for d in range(3)]
        shape = [hi[d] - lo[d] + 1 for d in range(3)]
        ld = [shape[1] + 2, shape[2] + 1]
        buf = pr.integers(-40, 40, shape[0] * ld[0] * ld[1]).astype(np.float64).reshape(shape[0], ld[0], ld[1])
        return lo, hi, shape, ld, buf

    lo, hi, shape, ld, buf = patch(rank)
    # NGA_Locate_num_blocks (base.c:5591-5627) counts blocks only for block-cyclic
    # distributions; for an array with a map (regular or irregular) the reference returns -1
    assert L.NGA_Locate_num_blocks(g, ia(lo), ia(hi)) == -1
    alpha = ctypes.c_double(rank + 1)
    L.NGA_Acc(g, ia(lo), ia(hi), buf.ctypes.data_as(ctypes.c_void_p), ia(ld), ctypes.byref(alpha))
    L.GA_Sync()
    full = np.zeros(dims)
    L.NGA_Get(g, ia([0, 0, 0]), ia([dims[0] - 1, dims[1] - 1, dims[2] - 1]), full.ctypes.data_as(ctypes.c_void_p),
              ia([dims[1], dims[2]]))
    want = np.zeros(dims)
    for r in range(size):
        lo_r, hi_r, sh, _, b = patch(r)
        want[lo_r[0]:hi_r[0] + 1, lo_r[1]:hi_r[1] + 1, lo_r[2]:hi_r[2] + 1] += (r + 1) * b[:, :sh[1], :sh[2]]
    assert np.array_equal(full, want), "irregular NGA_Acc"
    L.GA_Sync()
    say(rank, "irregular acc checked")
    # rank 0 puts a patch over every block; every rank gets it back
    plo, phi = [5, 3, 1], [90, 57, 11]
    pv = np.arange(86 * 55 * 11, dtype=np.float64).reshape(86, 55, 11) + 0.25
    if rank == 0:
        L.NGA_Put(g, ia(plo), ia(phi), pv.ctypes.data_as(ctypes.c_void_p), ia([55, 11]))
    L.GA_Sync()
    gv = np.zeros_like(pv)
    L.NGA_Get(g, ia(plo), ia(phi), gv.ctypes.data_as(ctypes.c_void_p), ia([55, 11]))
    assert np.array_equal(gv, pv), "irregular NGA_Put/NGA_Get"
    L.GA_Sync()
    # scatter-accumulate with repeated subscripts over every owner
    L.GA_Zero(g)
    sr = np.random.default_rng(60 + rank)
    nv = 3000
    subs = np.stack([sr.integers(0, dims[d], nv) for d in range(3)], axis=1).astype(np.int32)
    subs[nv // 2:nv // 2 + 100] = subs[:100]
    vals = sr.integers(-20, 20, nv).astype(np.float64)
    three = ctypes.c_double(3.0)
    L.NGA_Scatter_acc_flat(g, vals.ctypes.data_as(ctypes.c_void_p),
                           np.ascontiguousarray(subs).ravel().ctypes.data_as(ctypes.POINTER(ctypes.c_int)), nv,
                           ctypes.byref(three))
    L.GA_Sync()
    L.NGA_Get(g, ia([0, 0, 0]), ia([dims[0] - 1, dims[1] - 1, dims[2] - 1]), full.ctypes.data_as(ctypes.c_void_p),
              ia([dims[1], dims[2]]))
    want = np.zeros(dims)
    for r in range(size):
        rr = np.random.default_rng(60 + r)
        sb = np.stack([rr.integers(0, dims[d], nv) for d in range(3)], axis=1)
        sb[nv // 2:nv // 2 + 100] = sb[:100]
        vv = rr.integers(-20, 20, nv).astype(np.float64)
        np.add.at(want, (sb[:, 0], sb[:, 1], sb[:, 2]), 3.0 * vv)
    assert np.array_equal(full, want), "irregular NGA_Scatter_acc"
    L.GA_Sync()
    say(rank, "irregular scatter-acc checked")
    L.GA_Destroy(g)


# ---------------------------------------------------------------------------
# comex/testing/test.c test_acc (1028-1128) and test_cplx_acc (1130-1235),
# restated: for ndim 1..7 every rank accumulates a 2^ndim patch of a host array
# (alpha 0.1, double complex alpha (0, 0.1)) TIMES*nproc times into the far
# corner of the ranks' arrays in a permuted proc order; each rank then gets its
# corner back.  The reference checks rel 1e-4; since every contribution to an
# element is the same rounded product, the sum is the same in any order, so
# this checks bit-exactly against n sequential adds of that product.
def test_acc_ref(L, rank, size):
    import ga_amd
    DBL, DCP, TIMES = 38, 41, 3
    assert ga_amd.comex_init() == 0
    n_acc = TIMES * size
    for ndim in range(1, 8):
        for op in (DBL, DCP):
            esz = 8 if op == DBL else 16
            side = max(3, int(round(2000 ** (1.0 / ndim))))
            dimsA = [side + (j % 2) for j in range(ndim)]
            dimsB = [side + 1 - (j % 2) for j in range(ndim)]
            ea, eb = int(np.prod(dimsA)), int(np.prod(dimsB))
            seg = ga_amd.comex_malloc(eb * esz, size)
            L.gaamd_memset(ctypes.c_void_p(seg[rank]), 0, eb * esz)
            ga_amd.sync()
            if op == DBL:
                a = np.arange(ea, dtype=np.float64) * 1.25 + rank + 0.5       # host (malloc-like) source
                alpha = 0.1
            else:
                a = (np.arange(ea) * 1.25 + rank + 0.5) + 1j * (np.arange(ea) * -0.5 + 2.0 * rank)
                alpha = complex(0.0, 0.1)
            sA, sB = [esz * dimsA[0]], [esz * dimsB[0]]
            for j in range(1, ndim - 1):
                sA.append(sA[-1] * dimsA[j])
                sB.append(sB[-1] * dimsB[j])
            # first dimension fastest (column-major, as the reference's Index())
            offA = 0
            offB = sum((dimsB[j] - 2) * (esz * int(np.prod(dimsB[:j]))) for j in range(ndim))
            count = [2 * esz] + [2] * (ndim - 1)
            order = np.random.default_rng(5 + rank).permutation(size)
            ga_amd.comex_barrier()
            for i in range(n_acc):
                p = int(order[i % size])
                assert ga_amd.comex_accs(op, alpha, a.ctypes.data + offA, sA, seg[p] + offB, sB, count, ndim - 1,
                                         p) == 0
            ga_amd.comex_barrier()
            # get my corner back into a zeroed host array laid out like a
            c = np.zeros_like(a)
            assert ga_amd.comex_gets(seg[rank] + offB, sB, c.ctypes.data + offA, sA, count, ndim - 1, rank) == 0
            ga_amd.comex_fence_all()
            # expected: every rank added n_acc/size ... each rank's own a: sum over sources
            idx = [0]
            for j in range(ndim):
                stride = int(np.prod(dimsA[:j]))
                idx = [x + k * stride for k in range(2) for x in idx]
            idx = np.array(idx)
            want = np.zeros(len(idx), dtype=a.dtype)
            contribs = []
            for s in range(size):
                if op == DBL:
                    a_s = np.arange(ea, dtype=np.float64) * 1.25 + s + 0.5
                    contribs.append(a_s[idx] * 0.1)
                else:
                    a_s = (np.arange(ea) * 1.25 + s + 0.5) + 1j * (np.arange(ea) * -0.5 + 2.0 * s)
                    br, bi = a_s[idx].real, a_s[idx].imag
                    re = br * 0.0 - bi * 0.1          # acc.h:47-49 with C = (0, 0.1)
                    im = br * 0.1 + bi * 0.0
                    contribs.append(re + 1j * im)
            # each source rank targets me TIMES times; sums of different sources
            # depend on order, so compare per the reference (rel 1e-4) and, when a
            # single source exists, exactly
            for s in range(size):
                for _ in range(TIMES):
                    want = want + contribs[s]
            got = c[idx]
            assert np.allclose(got, want, rtol=1e-4, atol=0), (ndim, op, np.max(np.abs(got - want)))
            if size == 1:
                assert np.array_equal(got, want), (ndim, op)
            ga_amd.comex_barrier()
            assert ga_amd.comex_free(seg[rank]) == 0
    say(rank, "test_acc / test_cplx_acc ndim 1..7 ok")
    ga_amd.comex_finalize()


# ---------------------------------------------------------------------------
# stress: every rank runs a seeded random program of remote/local accumulates
# (blocking, non-blocking, host or HBM source, 1-D..3-D, io-vector), puts into
# its own zone of every segment, gets back from those zones, and fences at
# random points.  Integer-valued f64, so concurrent accumulates from all ranks
# sum exactly in any order; every rank regenerates every other rank's program
# from its seed and checks its own segment at the end.
ST_ACC = 96 * 1024          # f64 elements of the accumulate zone
ST_ZONE = 4 * 1024          # f64 elements of one rank's put zone in every segment


def stress_program(s, size, n_ops):
    # STRESS_SEED (campaigns): another family of programs
    rng = np.random.default_rng(1000 + s + 7919 * int(os.environ.get("STRESS_SEED", "0")))
    ops = []
    for _ in range(n_ops):
        u = rng.random()
        t = int(rng.integers(size))
        if u < 0.55:
            lv = int(rng.integers(0, 3))
            cnt = [int(rng.integers(1, 300))] + [int(rng.integers(1, 9)) for _ in range(lv)]
            st = []
            x = cnt[0] + int(rng.integers(0, 40))
            for j in range(lv):
                st.append(x)
                x = x * cnt[j + 1] + int(rng.integers(0, 7))
            span = cnt[0] + sum(st[j] * (cnt[j + 1] - 1) for j in range(lv))
            off = int(rng.integers(0, ST_ACC - span))
            src = rng.integers(-50, 51, span).astype(np.float64)
            ops.append(dict(kind="acc", t=t, count=cnt, st=st, off=off, src=src, alpha=float(rng.integers(-3, 4)),
                            host=bool(rng.random() < 0.3), nb=bool(rng.random() < 0.25)))
        elif u < 0.65:
            n = int(rng.integers(1, 60))
            idx = rng.integers(0, ST_ACC, n)
            idx[n // 2:] = idx[: n - n // 2] if rng.random() < 0.5 else idx[n // 2:]     # duplicates sometimes
            ops.append(dict(kind="accv", t=t, idx=idx, vals=rng.integers(-9, 10, n).astype(np.float64),
                            alpha=float(rng.integers(1, 3))))
        elif u < 0.85:
            n = int(rng.integers(1, ST_ZONE))
            off = int(rng.integers(0, ST_ZONE - n + 1))
            ops.append(dict(kind="put", t=t, off=off, vals=rng.integers(-1000, 1000, n).astype(np.float64)))
        elif u < 0.95:
            ops.append(dict(kind="get", t=t))
        else:
            ops.append(dict(kind="fence", t=t))
    return ops


def stress_expected(me, size, n_ops):
    acc = np.zeros(ST_ACC)
    zones = np.zeros((size, ST_ZONE))
    for s in range(size):
        for op in stress_program(s, size, n_ops):
            if op["t"] != me:
                continue
            if op["kind"] == "acc":
                cnt, st = op["count"], op["st"]
                rows = [0]
                for j, c in enumerate(cnt[1:]):
                    rows = [r + k * st[j] for k in range(c) for r in rows]
                for r in rows:
                    acc[op["off"] + r: op["off"] + r + cnt[0]] += op["alpha"] * op["src"][r: r + cnt[0]]
            elif op["kind"] == "accv":
                np.add.at(acc, op["idx"], op["alpha"] * op["vals"])
            elif op["kind"] == "put":
                zones[s, op["off"]: op["off"] + len(op["vals"])] = op["vals"]
    return acc, zones


def stress_test(L, rank, size):
    import ga_amd
    DBL = 38
    n_ops = int(os.environ.get("STRESS_OPS", "400"))
    assert ga_amd.comex_init() == 0
    nbytes = (ST_ACC + size * ST_ZONE) * 8
    seg = ga_amd.comex_malloc(nbytes, size)
    L.gaamd_memset(ctypes.c_void_p(seg[rank]), 0, nbytes)
    ga_amd.sync()
    ga_amd.comex_barrier()
    serial0 = ga_amd.kernel_counts()["serial"]
    mine = np.zeros((size, ST_ZONE))            # what I have put into every target's zone for me
    keep = []
    pending = []
    for k, op in enumerate(stress_program(rank, size, n_ops)):
        t = op["t"]
        if op["kind"] == "acc":
            cnt, st = op["count"], op["st"]
            if op["host"]:
                buf = op["src"]
                sp = buf.ctypes.data
            else:
                db = ga_amd.DeviceBuffer(op["src"].nbytes)
                db.upload(op["src"])
                keep.append(db)
                sp = db.ptr
            args = (DBL, op["alpha"], sp, [x * 8 for x in op["st"]], seg[t] + op["off"] * 8, [x * 8 for x in st],
                    [cnt[0] * 8] + cnt[1:], len(st), t)
            if op["nb"] and not op["host"]:
                rc, h = ga_amd.comex_nbaccs(*args)
                assert rc == 0
                pending.append(h)
            else:
                assert ga_amd.comex_accs(*args) == 0
        elif op["kind"] == "accv":
            vb = ga_amd.DeviceBuffer(op["vals"].nbytes)
            vb.upload(op["vals"])
            keep.append(vb)
            desc = [([vb.ptr + 8 * i for i in range(len(op["vals"]))],
                     [seg[t] + 8 * int(i) for i in op["idx"]], 8)]
            assert ga_amd.comex_accv(DBL, op["alpha"], desc, t) == 0
        elif op["kind"] == "put":
            v = op["vals"]
            zone = seg[t] + (ST_ACC + rank * ST_ZONE + op["off"]) * 8
            assert L.comex_put(v.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(zone), v.nbytes, t, 0) == 0
            mine[t, op["off"]: op["off"] + len(v)] = v
        elif op["kind"] == "get":
            got = np.zeros(ST_ZONE)
            zone = seg[t] + (ST_ACC + rank * ST_ZONE) * 8
            assert L.comex_get(ctypes.c_void_p(zone), got.ctypes.data_as(ctypes.c_void_p), got.nbytes, t, 0) == 0
            assert np.array_equal(got, mine[t]), f"rank {rank} op {k}: get of my zone at rank {t} differs"
        else:
            L.comex_fence_proc(t, 0)
        if len(pending) > 8:
            for h in pending:
                assert ga_amd.comex_wait(h) == 0
            pending = []
    for h in pending:
        assert ga_amd.comex_wait(h) == 0
    say(rank, f"stress: {n_ops} ops issued")
    ga_amd.comex_barrier()
    out = np.zeros(ST_ACC + size * ST_ZONE)
    assert L.comex_get(ctypes.c_void_p(seg[rank]), out.ctypes.data_as(ctypes.c_void_p), nbytes, rank, 0) == 0
    acc, zones = stress_expected(rank, size, n_ops)
    bad = np.nonzero(out[:ST_ACC] != acc)[0]
    assert bad.size == 0, f"rank {rank}: {bad.size} accumulate-zone elements differ, first {bad[:5]}"
    assert np.array_equal(out[ST_ACC:].reshape(size, ST_ZONE), zones), f"rank {rank}: put zones differ"
    assert ga_amd.kernel_counts()["serial"] == serial0, f"rank {rank}: a serial kernel ran"
    if os.environ.get("COMEX_AMD_ONE_PASS_MIN") and size > 1 and one_pass_expected():
        # the test's point: small device-source accumulates into ranks of this GPU one-pass
        assert ga_amd.route_counts()["one_pass"] > 0, ga_amd.route_counts()
    ga_amd.comex_barrier()
    for b in keep:
        b.free()
    assert ga_amd.comex_free(seg[rank]) == 0
    ga_amd.comex_finalize()


# ---------------------------------------------------------------------------
# comex/testing/test.c test_dim (526-609) and test_nbdim (667-802), restated:
# strided put of a random patch of a host array (init(): value = sum idx[d]*100^d,
# test.c:217-239) into a random position of rank proc's array (dims + 1 in every
# dimension, test.c:38-45), strided get back into another random position of a
# host array, exact comparison (compare_patches with eps 0).  test_dim targets
# proc = nproc-1-me, LOOP times per ndim; test_nbdim posts all ndim 1..7 puts
# non-blocking (nbput for ndim 1, nbputs otherwise) to get_next_RRproc's targets,
# waits, then the gets likewise.  The reference draws ranges with rand(); here a
# seeded numpy generator per rank.
TD_DIMS_A = [5, 3, 8, 9, 7, 3, 2]       # DIM1..DIM7 (test.c:18-35, non-Solaris)
TD_DIMS_B = [d + 1 for d in TD_DIMS_A]  # EDIM = DIM + OFF


def td_index(sub, dims):                # Index(), test.c:275-283
    idx, f = 0, 1
    for s, d in zip(sub, dims):
        idx += s * f
        f *= d
    return idx


def td_init(ndim):                      # init(), test.c:217-239
    dims = TD_DIMS_A[:ndim]
    n = int(np.prod(dims))
    i = np.arange(n)
    val = np.zeros(n)
    field = 1.0
    for d in dims:
        val += field * (i % d)
        i = i // d
        field *= 100.0
    return val


def td_get_range(rng, dims):            # get_range(), test.c:122-140
    lo, hi = [], []
    for d in dims:
        t1, t2 = int(rng.integers(d)), int(rng.integers(d))
        lo.append(min(t1, t2))
        hi.append(max(t1, t2))
    return lo, hi


def td_new_range(rng, dims, lo, hi):    # new_range(), test.c:144-159
    nlo, nhi = [], []
    for d, l, h in zip(dims, lo, hi):
        diff = h - l + 1
        rng_ = d - diff
        t = int(rng.integers(rng_)) if rng_ > 0 else l
        nlo.append(t)
        nhi.append(t + diff - 1)
    return nlo, nhi


def td_strides(ndim):
    sA, sB = [8], [8]
    for i in range(ndim):
        sA[i] *= TD_DIMS_A[i]
        sB[i] *= TD_DIMS_B[i]
        if i < ndim - 1:
            sA.append(sA[i])
            sB.append(sB[i])
    return sA, sB


def td_patch(arr, lo, hi, dims):
    """elements of arr (first index fastest) in the patch lo..hi, in odometer order."""
    v = arr.reshape(list(reversed(dims)))
    sl = tuple(slice(l, h + 1) for l, h in zip(reversed(lo), reversed(hi)))
    return v[sl].copy()


class RRProc:                           # get_next_RRproc(), test.c:615-665
    def __init__(self, me, nproc):
        self.me, self.nproc = me, nproc
        self.distance = nproc // 2 + (nproc % 2)
        if nproc == 1:
            self.distance = 0

    def next(self, ndim):
        me, nproc = self.me, self.nproc
        proc = me + self.distance if me <= ((nproc // 2 - 1) if nproc % 2 == 0 else nproc // 2) else \
            me - self.distance
        if nproc % 2 != 0 and me == nproc // 2:
            proc = me
        if self.distance != 0:
            if me < nproc // 2:
                self.distance += 1
                if me + self.distance >= nproc:
                    self.distance = nproc // 2 + (nproc % 2) - me
            else:
                self.distance -= 1
                if me - self.distance >= nproc // 2:
                    d = nproc // 2 + (nproc % 2)
                    self.distance = d + (me - d)
            if ndim != 1 and 7 > nproc and nproc // 2 and ndim % (nproc // 2) == 0:
                self.distance = nproc // 2 + (nproc % 2)
        return proc


def test_dim_ref(L, rank, size, loop=40):
    import ga_amd
    assert ga_amd.comex_init() == 0
    rng = np.random.default_rng(1234 + rank)
    # ---- test_dim, ndim 1..7
    for ndim in range(1, 8):
        dA, dB = TD_DIMS_A[:ndim], TD_DIMS_B[:ndim]
        sA, sB = td_strides(ndim)
        b = ga_amd.comex_malloc(8 * int(np.prod(dB)), size)
        a = td_init(ndim)
        c = np.zeros_like(a)
        ga_amd.comex_fence_all()
        ga_amd.comex_barrier()
        proc = size - 1 - rank
        for _ in range(loop):
            loA, hiA = td_get_range(rng, dA)
            loB, hiB = td_new_range(rng, dB, loA, hiA)
            loC, hiC = td_new_range(rng, dA, loA, hiA)
            i1, i2, i3 = td_index(loA, dA), td_index(loB, dB), td_index(loC, dA)
            count = [hiA[j] - loA[j] + 1 for j in range(ndim)]
            count[0] *= 8
            assert ga_amd.comex_puts(a.ctypes.data + 8 * i1, sA, b[proc] + 8 * i2, sB, count, ndim - 1, proc) == 0
            # consecutive operations to one process are ordered (test.c:590-591)
            assert ga_amd.comex_gets(b[proc] + 8 * i2, sB, c.ctypes.data + 8 * i3, sA, count, ndim - 1, proc) == 0
            assert np.array_equal(td_patch(a, loA, hiA, dA), td_patch(c, loC, hiC, dA)), (ndim, loA, hiA)
        ga_amd.comex_barrier()
        assert ga_amd.comex_free(b[rank]) == 0
    say(rank, "test_dim ndim 1..7 ok")
    # ---- test_nbdim
    bs, As, Cs, rngs = {}, {}, {}, {}
    for ndim in range(1, 8):
        bs[ndim] = ga_amd.comex_malloc(8 * int(np.prod(TD_DIMS_B[:ndim])), size)
        As[ndim] = td_init(ndim)
        Cs[ndim] = np.zeros_like(As[ndim])
    ga_amd.comex_fence_all()
    ga_amd.comex_barrier()
    hput, hget = {}, {}
    rr = RRProc(rank, size)
    for ndim in range(1, 8):
        dA, dB = TD_DIMS_A[:ndim], TD_DIMS_B[:ndim]
        sA, sB = td_strides(ndim)
        proc = rr.next(ndim)
        loA, hiA = td_get_range(rng, dA)
        loB, hiB = td_new_range(rng, dB, loA, hiA)
        loC, hiC = td_new_range(rng, dA, loA, hiA)
        rngs[ndim] = (proc, loA, hiA, loB, loC, hiC)
        count = [hiA[j] - loA[j] + 1 for j in range(ndim)]
        count[0] *= 8
        h = ctypes.c_int(-1)
        src, dst = ctypes.c_void_p(As[ndim].ctypes.data + 8 * td_index(loA, dA)), \
            ctypes.c_void_p(bs[ndim][proc] + 8 * td_index(loB, dB))
        if ndim == 1:
            rc = L.comex_nbput(src, dst, count[0], proc, 0, ctypes.byref(h))
        else:
            rc = L.comex_nbputs(src, ga_amd.int_array(sA), dst, ga_amd.int_array(sB), ga_amd.int_array(count),
                                ndim - 1, proc, 0, ctypes.byref(h))
        assert rc == 0
        hput[ndim] = h
    ga_amd.comex_barrier()
    for ndim in range(1, 8):
        assert ga_amd.comex_wait(hput[ndim]) == 0
    ga_amd.comex_barrier()
    ga_amd.comex_fence_all()
    rr = RRProc(rank, size)
    for ndim in range(1, 8):
        dA, dB = TD_DIMS_A[:ndim], TD_DIMS_B[:ndim]
        sA, sB = td_strides(ndim)
        proc = rr.next(ndim)
        p0, loA, hiA, loB, loC, hiC = rngs[ndim]
        assert proc == p0
        count = [hiA[j] - loA[j] + 1 for j in range(ndim)]
        count[0] *= 8
        h = ctypes.c_int(-1)
        src, dst = ctypes.c_void_p(bs[ndim][proc] + 8 * td_index(loB, dB)), \
            ctypes.c_void_p(Cs[ndim].ctypes.data + 8 * td_index(loC, dA))
        if ndim == 1:
            rc = L.comex_nbget(src, dst, count[0], proc, 0, ctypes.byref(h))
        else:
            rc = L.comex_nbgets(src, ga_amd.int_array(sB), dst, ga_amd.int_array(sA), ga_amd.int_array(count),
                                ndim - 1, proc, 0, ctypes.byref(h))
        assert rc == 0
        hget[ndim] = h
    ga_amd.comex_barrier()
    for ndim in range(1, 8):
        assert ga_amd.comex_wait(hget[ndim]) == 0
        p0, loA, hiA, loB, loC, hiC = rngs[ndim]
        dA = TD_DIMS_A[:ndim]
        assert np.array_equal(td_patch(As[ndim], loA, hiA, dA), td_patch(Cs[ndim], loC, hiC, dA)), ndim
    ga_amd.comex_barrier()
    for ndim in range(1, 8):
        assert ga_amd.comex_free(bs[ndim][rank]) == 0
    say(rank, "test_nbdim ok")
    ga_amd.comex_finalize()



# ---------------------------------------------------------------------------
# GA-level accumulate tests of the reference, restated on the C API (row-major,
# 0-based: Fortran (i, j) of an n x n array is C [j][i]):
#  * test.F:596-658 disjoint ga_acc: the n x n array is tiled with inc x inc
#    patches (inc = (n-1)/20 + 1, a patch ending at n-1 is stretched to n), tile
#    ij is accumulated by rank ij mod nproc from b(i,j) = i+j with x = 10, and
#    every rank checks the whole array against its local copy (reference:
#    rel 1e-13; here exact: every element is accumulated once into 0);
#    float/double complex variants (test.F:1567-1622, 2204-2259) and int;
#  * test.F:700-725 overlapping accumulate: every rank adds 1.0 at (n/2, n/2),
#    rank 0 checks nproc (reference |d| <= 1e-10; exact here);
#  * ngatest_src/ndim_NGA_ACC.src for ndim 1..7 (the commented, smaller n set of
#    ngatest.def): fill with val, then MAXLOOP times accumulate alpha = val times
#    a random sub-range (random_range, ndim_util_comm.src:1-22) of rank
#    nproc-1-me's block from the same position of a full local array, comparing
#    the patch before/after (reference 1e-2; exact here, acc.h expression order).
GA_TYPES = {1001: np.int32, 1003: np.float32, 1004: np.float64, 1007: np.complex128}


def acc_expect(a, b, alpha):
    """a + alpha*b in the order of acc.h:46-49 / 119-143 (no FMA, int wraps)."""
    if np.iscomplexobj(a):
        re = a.real + (b.real * alpha.real - b.imag * alpha.imag)
        im = a.imag + (b.real * alpha.imag + b.imag * alpha.real)
        return re + 1j * im
    if a.dtype.kind == "i":
        return (a.astype(np.int64) + np.int64(alpha) * b.astype(np.int64)).astype(np.uint32).view(np.int32)
    return a + a.dtype.type(alpha) * b


def typed_scalar(t, v):
    if t == 1001:
        return ctypes.c_int(int(v))
    if t == 1003:
        return ctypes.c_float(v)
    if t == 1004:
        return ctypes.c_double(v)
    return (ctypes.c_double * 2)(v.real, v.imag)


def ga_ref_test(L, rank, size):
    ia = ga_amd_int_array()
    assert L.GA_Initialize() == 0
    P = ctypes.c_void_p
    # ---- test.F:596-725
    n = 100
    inc = (n - 1) // 20 + 1
    for t in (1004, 1007, 1003, 1001):
        dt = GA_TYPES[t]
        g = L.NGA_Create(t, 2, ia([n, n]), b"a", None)
        assert g > 0
        L.GA_Zero(g)
        L.GA_Sync()
        jj, ii = np.meshgrid(np.arange(1, n + 1), np.arange(1, n + 1), indexing="ij")
        b = (ii + jj).astype(dt)                       # C b[j][i] = Fortran b(i, j) = i + j
        if t == 1007:
            b = b + 1j * (ii - 2 * jj)
        x = {1001: 10, 1003: 10.0, 1004: 10.0, 1007: complex(10.0, -0.5)}[t]
        alpha = typed_scalar(t, x)
        a = np.zeros((n, n), dtype=dt)
        ij = 0
        for j in range(1, n + 1, inc):
            for i in range(1, n + 1, inc):
                ilo, ihi = i, min(i + inc - 1, n)
                if ihi == n - 1:
                    ihi = n
                jlo, jhi = j, min(j + inc - 1, n)
                if jhi == n - 1:
                    jhi = n
                if ij % size == rank:
                    L.NGA_Acc(g, ia([jlo - 1, ilo - 1]), ia([jhi - 1, ihi - 1]),
                              P(b.ctypes.data + b.itemsize * ((jlo - 1) * n + ilo - 1)), ia([n]), ctypes.byref(alpha))
                ij += 1
                sl = (slice(jlo - 1, jhi), slice(ilo - 1, ihi))
                a[sl] = acc_expect(a[sl], b[sl], x)
        L.GA_Sync()
        got = np.zeros((n, n), dtype=dt)
        L.NGA_Get(g, ia([0, 0]), ia([n - 1, n - 1]), P(got.ctypes.data), ia([n]))
        assert np.array_equal(got, a), f"test.F disjoint ga_acc type {t}"
        L.GA_Sync()
        L.GA_Destroy(g)
    say(rank, "test.F disjoint ga_acc (dbl, dcpl, float, int) ok")
    g = L.NGA_Create(1004, 2, ia([n, n]), b"b", None)
    L.GA_Zero(g)
    one = ctypes.c_double(1.0)
    e = np.ones(1)
    L.NGA_Acc(g, ia([n // 2 - 1, n // 2 - 1]), ia([n // 2 - 1, n // 2 - 1]), P(e.ctypes.data), ia([1]),
              ctypes.byref(one))
    L.GA_Sync()
    if rank == 0:
        v = np.zeros(1)
        L.NGA_Get(g, ia([n // 2 - 1, n // 2 - 1]), ia([n // 2 - 1, n // 2 - 1]), P(v.ctypes.data), ia([1]))
        assert v[0] == float(size), ("overlapping ga_acc", v[0], size)
    L.GA_Sync()
    L.GA_Destroy(g)
    say(rank, "test.F overlapping ga_acc ok")
    # ---- ndim_NGA_ACC.src
    n_of = {1: 2000, 2: 100, 3: 20, 4: 10, 5: 5, 6: 4, 7: 3}
    rng = np.random.default_rng(77 + rank)
    for t in (1001, 1004, 1007):
        dt = GA_TYPES[t]
        for ndim in range(1, 8):
            nn = n_of[ndim]
            dims = [nn] * ndim
            g = L.NGA_Create(t, ndim, ia(dims), b"a", None)
            assert g > 0
            val = {1001: rank * 2 + 3, 1004: 0.5 + rank * 0.25, 1007: complex(0.5 + rank, -0.25)}[t]
            # ga_fill(g_a, val): every rank puts val into its own block
            blo, bhi = (ctypes.c_int * ndim)(), (ctypes.c_int * ndim)()
            L.NGA_Distribution(g, rank, blo, bhi)
            if all(bhi[k] >= blo[k] for k in range(ndim)):
                ext = [bhi[k] - blo[k] + 1 for k in range(ndim)]
                f = np.full(ext, val, dtype=dt)
                L.NGA_Put(g, blo, bhi, P(f.ctypes.data), ia(ext[1:]))
            L.GA_Sync()
            proc = size - 1 - rank
            lop, hip = (ctypes.c_int * ndim)(), (ctypes.c_int * ndim)()
            L.NGA_Distribution(g, proc, lop, hip)
            has = all(hip[k] >= lop[k] for k in range(ndim))
            total = int(np.prod(dims))
            if t == 1001:
                b = rng.integers(-1000, 1000, total).astype(np.int32).reshape(dims)
            else:
                b = (rng.random(total) * 2 - 1).reshape(dims).astype(dt)
                if t == 1007:
                    b = b + 1j * (rng.random(total) - 0.5).reshape(dims)
            alpha = typed_scalar(t, val)
            ld = ia([nn] * (ndim - 1))
            for loop in range(20):
                lo, hi = [], []
                for k in range(ndim):               # random_range(lop, hip, lo, hi)
                    rg = hip[k] - lop[k] + 1
                    l_ = lop[k] + int(rng.random() * rg) + 1
                    h_ = hip[k] - (int(rng.random() * rg) + 1)
                    if h_ < l_:
                        l_, h_ = h_, l_
                    lo.append(max(l_, lop[k]))
                    hi.append(min(h_, hip[k]))
                ok = has and all(hi[k] >= lo[k] for k in range(ndim))
                L.GA_Sync()
                ext = [hi[k] - lo[k] + 1 for k in range(ndim)] if ok else []
                sl = tuple(slice(lo[k], hi[k] + 1) for k in range(ndim)) if ok else ()
                if ok:
                    before = np.zeros(ext, dtype=dt)
                    L.NGA_Get(g, ia(lo), ia(hi), P(before.ctypes.data), ia(ext[1:]))
                L.GA_Sync()
                if ok:
                    off = sum(lo[k] * int(np.prod(dims[k + 1:])) for k in range(ndim))
                    L.NGA_Acc(g, ia(lo), ia(hi), P(b.ctypes.data + b.itemsize * off), ld, ctypes.byref(alpha))
                L.GA_Sync()
                if ok:
                    after = np.zeros(ext, dtype=dt)
                    L.NGA_Get(g, ia(lo), ia(hi), P(after.ctypes.data), ia(ext[1:]))
                    want = acc_expect(before, b[sl], val)
                    assert np.array_equal(after, want), ("ndim_NGA_ACC", t, ndim, loop, lo, hi)
            L.GA_Sync()
            L.GA_Destroy(g)
    say(rank, "ndim_NGA_ACC (int, dbl, dcpl; ndim 1..7) ok")
    L.GA_Terminate()


def ga_amd_int_array():
    import ga_amd
    return ga_amd.int_array



# ---------------------------------------------------------------------------
# comex/testing/test.c test_vector (1240-1386) and test_vector_acc (1394-1491),
# restated.  test_vector: a random patch of a host 50x50 array goes to rank
# nproc-1-me's 51x51 array as two comex_putv calls (lower triangle incl. the
# diagonal: one descriptor per column of decreasing length; upper triangle: one
# per column), then comes back whole with one comex_getv of `cols` runs into
# another random position; exact.  test_vector_acc: every rank accumulates the
# even and then the odd elements of a[i] = i (ELEMS = 200) into rank 0 with
# alpha 0.1, one single-element run each, TIMES*nproc times; rank 0's array is
# then a * alpha*TIMES*nproc*nproc at rel 1e-4 (exact on one rank against the
# sequential sum).
def test_vector_ref(L, rank, size, loop=60):
    import ga_amd
    assert ga_amd.comex_init() == 0
    rng = np.random.default_rng(4321 + rank)
    M = 50
    dA, dB = [M, M], [M + 1, M + 1]
    b = ga_amd.comex_malloc(8 * dB[0] * dB[1], size)
    a = td_init_dims(dA)
    c = np.zeros_like(a)
    ga_amd.comex_barrier()
    proc = size - 1 - rank
    A, C = a.ctypes.data, c.ctypes.data
    for _ in range(loop):
        loA, hiA = td_get_range(rng, dA)
        loB, hiB = td_new_range(rng, dB, loA, hiA)
        loC, hiC = td_new_range(rng, dA, loA, hiA)
        cols, rows = hiA[1] - loA[1] + 1, hiA[0] - loA[0] + 1
        mrc = min(cols, rows)
        descs = []
        for i in range(mrc):               # lower triangle incl. diagonal
            s_ = A + 8 * td_index([loA[0] + i, loA[1] + i], dA)
            d_ = b[proc] + 8 * td_index([loB[0] + i, loB[1] + i], dB)
            descs.append(([s_], [d_], (rows - i) * 8))
        assert ga_amd.comex_putv(descs, proc) == 0
        descs = []
        for i in range(1, cols):           # upper triangle
            s_ = A + 8 * td_index([loA[0], loA[1] + i], dA)
            d_ = b[proc] + 8 * td_index([loB[0], loB[1] + i], dB)
            descs.append(([s_], [d_], min(i, rows) * 8))
        if cols - 1:
            assert ga_amd.comex_putv(descs, proc) == 0
        srcs = [b[proc] + 8 * td_index([loB[0], loB[1] + i], dB) for i in range(cols)]
        dsts = [C + 8 * td_index([loC[0], loC[1] + i], dA) for i in range(cols)]
        assert ga_amd.comex_getv([(srcs, dsts, rows * 8)], proc) == 0
        assert np.array_equal(td_patch(a, loA, hiA, dA), td_patch(c, loC, hiC, dA)), (loA, hiA)
    ga_amd.comex_barrier()
    assert ga_amd.comex_free(b[rank]) == 0
    say(rank, "test_vector ok")
    # ---- test_vector_acc
    ELEMS, TIMES, alpha = 200, 20, 0.1
    # diagnostics only (TEST_VEC_RANK_ALPHA=1): rank r uses alpha*(1+r), so a miss names its rank
    rank_alpha = os.environ.get("TEST_VEC_RANK_ALPHA") == "1"
    my_alpha = alpha * (1 + rank) if rank_alpha else alpha
    b = ga_amd.comex_malloc(8 * ELEMS, size)
    L.gaamd_memset(ctypes.c_void_p(b[rank]), 0, 8 * ELEMS)
    ga_amd.sync()
    a = np.arange(ELEMS, dtype=np.float64)
    A = a.ctypes.data
    ga_amd.comex_barrier()
    routes0, owned0 = ga_amd.route_counts(), ga_amd.owner_counts()
    # diagnostics only (TEST_VEC_SKIP_LOCAL=1): rank 0 does not accumulate into itself
    skip_local = os.environ.get("TEST_VEC_SKIP_LOCAL") == "1" and size > 1
    for _ in range(TIMES * size):
        for par in (0, 1):
            if skip_local and rank == 0:
                continue
            idx = range(par, ELEMS, 2)
            descs = [([A + 8 * j for j in idx], [b[0] + 8 * j for j in idx], 8)]
            assert ga_amd.comex_accv(38, my_alpha, descs, 0) == 0
    ga_amd.comex_fence_all()
    routes = {k: v - routes0[k] for k, v in ga_amd.route_counts().items()}
    say(rank, f"test_vector_acc routes {routes}")
    ga_amd.comex_barrier()
    owned = {k: v - owned0[k] for k, v in ga_amd.owner_counts().items()}
    cc = np.zeros(ELEMS)
    assert L.comex_get(ctypes.c_void_p(b[0]), ctypes.c_void_p(cc.ctypes.data), 8 * ELEMS, 0, 0) == 0
    senders = range(1, size) if skip_local else range(size)
    want = a * (alpha * TIMES * size * (sum(1 + r for r in senders) if rank_alpha else len(senders)))
    if not np.allclose(cc, want, rtol=1e-4, atol=0):
        bad = np.nonzero(~np.isclose(cc, want, rtol=1e-4, atol=0))[0]
        msg = f"test_vector_acc: {bad.size} elements off: " + ", ".join(
            f"[{j}] got {cc[j]!r} want {want[j]!r} (diff/(alpha*a) {(cc[j] - want[j]) / (alpha * a[j]) if a[j] else 0:+.3f})"
            for j in bad[:4])
        # diagnosis: read again after a pause -- a late update means completion was
        # reported early, a permanent miss means an update was lost
        import time
        time.sleep(0.5)
        again = np.zeros(ELEMS)
        assert L.comex_get(ctypes.c_void_p(b[0]), ctypes.c_void_p(again.ctypes.data), 8 * ELEMS, 0, 0) == 0
        ga_amd.comex_fence_all()
        healed = np.allclose(again, want, rtol=1e-4, atol=0)
        raise AssertionError(msg + f"; after 0.5 s: {'correct (late update)' if healed else 'still off (lost update)'}"
                             f"; owner applied {owned}")
    if rank == 0:
        # every remote request was applied as the io-vector request it was posted as
        # (a request once fell through to the packed-strided branch of the owner's
        # inbox loop and lost its whole contribution)
        remote = TIMES * size * 2 * (size - 1)
        assert owned == {"packed": 0, "iov": remote, "rmw": 0, "direct_src": 0}, owned
    if size == 1 and not rank_alpha:
        seq = np.zeros(ELEMS)
        for _ in range(TIMES):
            seq = seq + a * alpha
        assert np.array_equal(cc, seq)
    ga_amd.comex_barrier()
    assert ga_amd.comex_free(b[rank]) == 0
    say(rank, "test_vector_acc ok")
    ga_amd.comex_finalize()


def td_init_dims(dims):                 # init() for arbitrary dims, test.c:217-239
    n = int(np.prod(dims))
    i = np.arange(n)
    val = np.zeros(n)
    field = 1.0
    for d in dims:
        val += field * (i % d)
        i = i // d
        field *= 100.0
    return val



# ---------------------------------------------------------------------------
# armci/testing/test.c test_acc (896-976), restated through the ARMCI API
# (ARMCI_Malloc, ARMCI_AccS, ARMCI_AllFence, ARMCI_Barrier, ARMCI_GetS): a
# 2^ndim patch at the origin of a host array, alpha 0.1, accumulated TIMES*nproc
# times into the far corner of the ranks' arrays in a permuted proc order
# (GetPermutedProcList, test.c:993), then each rank gets its corner back and
# compares with a * alpha*TIMES*nproc at rel 1e-4 (exact on one rank against the
# sequential sum).  Odd ndim use ARMCI_NbAccS + ARMCI_WaitAll instead.
def armci_test_acc_ref(L, rank, size, times=10):
    import ga_amd
    assert L.ARMCI_Init() == 0
    P = ctypes.c_void_p
    alpha = ctypes.c_double(0.1)
    rng = np.random.default_rng(rank)
    for ndim in range(1, 8):
        dA, dB = TD_DIMS_A[:ndim], TD_DIMS_B[:ndim]
        sA, sB = td_strides(ndim)
        loA, loB = [0] * ndim, [d - 2 for d in dB]
        count = [2 * 8] + [2] * (ndim - 1)
        ptrs = (ctypes.c_void_p * size)()
        nbytes = 8 * int(np.prod(dB))
        assert L.ARMCI_Malloc(ptrs, nbytes) == 0
        L.gaamd_memset(ctypes.c_void_p(ptrs[rank]), 0, nbytes)
        ga_amd.sync()
        a = td_init(ndim)
        c = np.zeros_like(a)
        plist = list(range(size))
        for i in range(size):                  # random swapping, test.c:1013-1017
            j = int(rng.integers(size))
            plist[i], plist[j] = plist[j], plist[i]
        i1, i2 = td_index(loA, dA), td_index(loB, dB)
        L.ARMCI_AllFence()
        L.ARMCI_Barrier()
        for i in range(times * size):
            proc = plist[i % size]
            args = (P(a.ctypes.data + 8 * i1), ga_amd.int_array(sA), P(ptrs[proc] + 8 * i2), ga_amd.int_array(sB),
                    ga_amd.int_array(count), ndim - 1, proc)
            if ndim % 2:
                h = ctypes.c_int(0)
                assert L.ARMCI_NbAccS(38, ctypes.byref(alpha), *args, ctypes.byref(h)) == 0
            else:
                assert L.ARMCI_AccS(38, ctypes.byref(alpha), *args) == 0
        if ndim % 2:
            assert L.ARMCI_WaitAll() == 0
        L.ARMCI_AllFence()
        L.ARMCI_Barrier()
        assert L.ARMCI_GetS(P(ptrs[rank] + 8 * i2), ga_amd.int_array(sB), P(c.ctypes.data + 8 * i1),
                            ga_amd.int_array(sA), ga_amd.int_array(count), ndim - 1, rank) == 0
        hi = [1] * ndim
        got, base = td_patch(c, loA, hi, dA), td_patch(a, loA, hi, dA)
        want = base * (0.1 * times * size)
        assert np.allclose(got, want, rtol=1e-4, atol=0), (ndim, np.max(np.abs(got - want)))
        if size == 1:
            seq = np.zeros_like(base)
            for _ in range(times):
                seq = seq + base * 0.1
            assert np.array_equal(got, seq), ndim
        L.ARMCI_Barrier()
        assert L.ARMCI_Free(ctypes.c_void_p(ptrs[rank])) == 0
    say(rank, "armci test_acc ndim 1..7 ok")
    L.ARMCI_Finalize()



# ---------------------------------------------------------------------------
# remote io-vector accumulates at GA scatter-acc sizes: every rank sends one
# comex_accv of n single-float pairs to every rank (itself included) into the
# zone of the target's segment reserved for this source, destinations random in
# the zone (many repeats); sources in HBM on even ranks, in pageable host memory
# on odd ranks.  One source per zone, so the bits depend only on that source's
# pair order: each target replays every source's pairs in order (np.add.at is
# unbuffered, float32 multiply then add as acc.h) and compares bit for bit.
SCAT_N, SCAT_ZONE = 20000, 3000


def scat_pairs(src_rank, dst_rank):
    rng = np.random.default_rng(1000 * src_rank + dst_rank)
    idx = rng.integers(0, SCAT_ZONE, SCAT_N)
    vals = (rng.random(SCAT_N) * 2 - 1).astype(np.float32)
    return idx, vals


def scatter_remote_test(L, rank, size):
    import ga_amd
    FLT, alpha = 39, np.float32(0.7071067811865476)
    assert ga_amd.comex_init() == 0
    zone_b = SCAT_ZONE * 4
    seg = ga_amd.comex_malloc(zone_b * size, size)
    init = (np.arange(SCAT_ZONE * size) % 97).astype(np.float32) * np.float32(0.25)
    L.gaamd_memcpy(ctypes.c_void_p(seg[rank]), init.ctypes.data_as(ctypes.c_void_p), init.nbytes)
    ga_amd.sync()
    ga_amd.comex_barrier()
    keep = []
    for t in list(range(rank + 1, size)) + list(range(0, rank + 1)):
        idx, vals = scat_pairs(rank, t)
        if rank % 2 == 0:
            vb = ga_amd.DeviceBuffer(vals.nbytes)
            vb.upload(vals)
            sbase = vb.ptr
            keep.append(vb)
        else:
            sbase = vals.ctypes.data
            keep.append(vals)
        src = (np.uint64(sbase) + 4 * np.arange(SCAT_N, dtype=np.uint64)).astype(np.uint64)
        dst = (np.uint64(seg[t] + zone_b * rank) + 4 * idx.astype(np.uint64)).astype(np.uint64)
        g = ga_amd.GIOV()
        g.src = ctypes.cast(ctypes.c_void_p(src.ctypes.data), ctypes.POINTER(ctypes.c_void_p))
        g.dst = ctypes.cast(ctypes.c_void_p(dst.ctypes.data), ctypes.POINTER(ctypes.c_void_p))
        g.count, g.bytes = SCAT_N, 4
        ks, sp = ga_amd.scale_buffer(FLT, float(alpha))
        assert L.comex_accv(FLT, sp, ctypes.byref(g), 1, t, 0) == 0
        keep.append((src, dst))
    ga_amd.comex_fence_all()
    ga_amd.comex_barrier()
    got = np.zeros(SCAT_ZONE * size, dtype=np.float32)
    L.gaamd_memcpy(got.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(seg[rank]), got.nbytes)
    want = init.copy()
    for s_ in range(size):
        idx, vals = scat_pairs(s_, rank)
        z = want[SCAT_ZONE * s_:SCAT_ZONE * (s_ + 1)]
        np.add.at(z, idx, alpha * vals)
    bad = np.flatnonzero(got.view(np.uint32) != want.view(np.uint32))
    assert bad.size == 0, f"rank {rank}: {bad.size} elements differ, first zone {bad[0] // SCAT_ZONE}"
    ga_amd.comex_barrier()
    for b in keep:
        if isinstance(b, ga_amd.DeviceBuffer):
            b.free()
    assert ga_amd.comex_free(seg[rank]) == 0
    say(rank, "remote scatter-acc ok")
    ga_amd.comex_finalize()



# ---------------------------------------------------------------------------
# ngatest_src/ndim_NGA_SCATTER_ACC.src and ndim_NGA_GATHER.src restated (C API,
# row-major subscripts): for ndim 1..7, every rank draws m = total/100 distinct
# random elements from its own slice of the linear index space (me*total/nproc
# onwards, so the slices of different ranks never collide but cross owner
# blocks), scatter-accumulates random values with alpha = rand(me*2+1), and
# checks every element against v*alpha + (value before) read back with
# NGA_Get (reference 1e-5; exact here); then gathers the same elements and
# compares with single-element gets.  int, double, double complex.
def ngatest_gs(L, rank, size):
    ia = ga_amd_int_array()
    P = ctypes.c_void_p
    assert L.GA_Initialize() == 0
    n_of = {1: 2000, 2: 100, 3: 20, 4: 10, 5: 5, 6: 4, 7: 3}
    rng = np.random.default_rng(300 + rank)
    for t in (1001, 1004, 1007):
        dt = GA_TYPES[t]
        for ndim in range(1, 8):
            dims = [n_of[ndim]] * ndim
            total = int(np.prod(dims))
            g = L.NGA_Create(t, ndim, ia(dims), b"a", None)
            assert g > 0
            L.GA_Zero(g)
            m = max(1, total // 100)
            lo_i, span = rank * total // size, max(1, total // size)
            alpha = {1001: rank * 2 + 1, 1004: 0.25 + 0.5 * rank, 1007: complex(0.5, 0.25 * rank - 0.5)}[t]
            for loop in range(3):
                L.GA_Sync()
                lin = lo_i + rng.choice(min(span, total - lo_i), size=min(m, span), replace=False)
                k = len(lin)
                subs = np.array(np.unravel_index(lin, dims)).T.astype(np.int32).copy()   # k x ndim, C order
                if t == 1001:
                    v = rng.integers(-50, 50, k).astype(np.int32)
                else:
                    v = (rng.random(k) * 2 - 1).astype(dt)
                    if t == 1007:
                        v = v + 1j * (rng.random(k) - 0.5)
                before = np.zeros(k, dtype=dt)
                for i in range(k):
                    sub = ia(subs[i].tolist())
                    L.NGA_Get(g, sub, sub, P(before.ctypes.data + i * before.itemsize), ia([1] * (ndim - 1)))
                want = acc_expect(before, v, alpha)
                L.GA_Sync()
                al = typed_scalar(t, alpha)
                L.NGA_Scatter_acc_flat(g, P(v.ctypes.data), subs.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), k,
                                       ctypes.byref(al))
                L.GA_Sync()
                after = np.zeros(k, dtype=dt)
                for i in range(k):
                    sub = ia(subs[i].tolist())
                    L.NGA_Get(g, sub, sub, P(after.ctypes.data + i * after.itemsize), ia([1] * (ndim - 1)))
                assert np.array_equal(after, want), ("NGA_SCATTER_ACC", t, ndim, loop)
                gat = np.zeros(k, dtype=dt)
                L.NGA_Gather_flat(g, P(gat.ctypes.data), subs.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), k)
                assert np.array_equal(gat, after), ("NGA_GATHER", t, ndim, loop)
            L.GA_Sync()
            L.GA_Destroy(g)
    say(rank, "ndim_NGA_SCATTER_ACC / ndim_NGA_GATHER (int, dbl, dcpl; ndim 1..7) ok")
    L.GA_Terminate()


def random_remote_descriptors_test(L, rank, size):
    """Seeded random strided descriptors (tests/test_gpu_fuzz.py's generator: every op,
    0..7 stride levels, rows of 1..8 Ki elements, padded / overlapping / zero strides,
    offsets below the natural alignment) from rank 0 into rank 1's segment: accumulates
    and puts, blocking and non-blocking, from a plain device buffer, from rank 0's own
    segment (the direct-source route when the owner is another GPU), from pageable and
    from pinned host memory; and gets back from a region nobody writes.  One writer, so
    program order decides every byte: rank 1 replays the same sequence with the oracle
    and compares its segment exactly; rank 0 checks each get."""
    import ga_amd
    import cases as C
    from oracle import Oracle
    from test_gpu_fuzz import OPS, phased_fill, random_alpha, random_case
    from helpers import same_bits_nan_aware, first_mismatch
    ora = Oracle()
    assert ga_amd.comex_init() == 0
    owner = 1 % size
    REG = 4 << 20
    nreg = len(OPS) + 2                    # one region per op, one for puts, one for gets
    PUT, GET = len(OPS), len(OPS) + 1
    seg = ga_amd.comex_malloc(REG * nreg, size)
    srcseg = ga_amd.comex_malloc(REG, size)
    init = [phased_fill(op, REG, 0, 900 + i) for i, op in enumerate(OPS)]
    init += [np.random.default_rng(77).integers(0, 256, REG, dtype=np.uint8) for _ in range(2)]
    if rank == owner:
        for i, a in enumerate(init):
            assert L.gaamd_memcpy(ctypes.c_void_p(seg[owner] + i * REG), a.ctypes.data_as(ctypes.c_void_p), REG) == 0
    ga_amd.comex_barrier()
    rng = np.random.default_rng(int(os.environ.get("RDESC_SEED", "3")))
    ncase = int(os.environ.get("RDESC_CASES", "150"))

    def fits(c):
        s_hi = c["so"] + C.span(c["ss"], c["count"], c["levels"])[1]
        d_hi = c["do"] + C.span(c["ds"], c["count"], c["levels"])[1]
        return s_hi <= REG and d_hi <= REG

    def draw(op):
        while True:
            c = random_case(rng, op)
            c["alias"] = False
            if fits(c):
                return c

    plan = []
    for k in range(ncase):
        op = OPS[k % len(OPS)]
        c = draw(op)
        c["kind"] = ("acc", "acc", "put", "get")[int(rng.integers(0, 4))]
        c["src_kind"] = ("dev", "seg", "host", "pinned")[k % 4]
        c["nb"] = bool(rng.random() < 0.4)
        if c["kind"] != "acc":   # byte copies: whole rows of any length
            c["count"] = [c["count"][0] + int(rng.integers(0, 8))] + c["count"][1:]
            if not fits(c):
                c["kind"] = "acc"
                c["count"][0] = c["count"][0] // C.ESZ[op] * C.ESZ[op]
        plan.append(c)
    if rank == 0:
        handles, keep = [], []
        dev = ga_amd.DeviceBuffer(REG)
        pin = ga_amd.DeviceBuffer(REG, host=True)
        for k, c in enumerate(plan):
            op, count, levels = c["op"], c["count"], c["levels"]
            s_hi = c["so"] + C.span(c["ss"], count, levels)[1]
            if c["kind"] == "get":
                # owner's GET region (src side, strides ds) into a local buffer (strides ss)
                d_hi = c["do"] + C.span(c["ds"], count, levels)[1]
                local = np.random.default_rng(k).integers(0, 256, max(16, s_hi), dtype=np.uint8)
                lb = ga_amd.DeviceBuffer(local.size)
                lb.upload(local)
                assert ga_amd.comex_gets(seg[owner] + GET * REG + c["do"], c["ds"], lb.ptr + c["so"], c["ss"], count,
                                         levels, owner) == 0
                assert ga_amd.comex_fence_all() == 0
                want = local.copy()
                ora.puts(init[GET], c["do"], c["ds"], want, c["so"], c["ss"], count, levels)
                got = lb.download(np.uint8, local.size)
                assert np.array_equal(got, want), ("get", k, c)
                lb.free()
                continue
            src = phased_fill(op, max(16, s_hi), c["so"], 3000 + k)
            if c["src_kind"] == "dev":
                assert L.gaamd_memcpy(ctypes.c_void_p(dev.ptr), src.ctypes.data_as(ctypes.c_void_p), src.size) == 0
                sp = dev.ptr
            elif c["src_kind"] == "seg":
                assert L.gaamd_memcpy(ctypes.c_void_p(srcseg[rank]), src.ctypes.data_as(ctypes.c_void_p),
                                      src.size) == 0
                sp = srcseg[rank]
            elif c["src_kind"] == "pinned":
                ctypes.memmove(pin.ptr, src.ctypes.data, src.size)
                sp = pin.ptr
            else:
                sp = src.ctypes.data
            if c["kind"] == "acc":
                alpha = c["alpha"]
                dst = seg[owner] + OPS.index(op) * REG + c["do"]
                if c["nb"]:
                    rc, h = ga_amd.comex_nbaccs(op, alpha, sp + c["so"], c["ss"], dst, c["ds"], count, levels, owner)
                    assert rc == 0
                    assert ga_amd.comex_wait(h) == 0   # the source buffer is reused by the next case
                else:
                    assert ga_amd.comex_accs(op, alpha, sp + c["so"], c["ss"], dst, c["ds"], count, levels,
                                             owner) == 0
            else:
                assert ga_amd.comex_puts(sp + c["so"], c["ss"], seg[owner] + PUT * REG + c["do"], c["ds"], count,
                                         levels, owner) == 0
            keep.append(src)
        assert ga_amd.comex_fence_all() == 0
        dev.free()
        pin.free()
        say(rank, f"{ncase} random descriptors issued")
    ga_amd.comex_barrier()
    if rank == owner:
        want = [a.copy() for a in init]
        for k, c in enumerate(plan):
            if c["kind"] == "get":
                continue
            op, count, levels = c["op"], c["count"], c["levels"]
            s_hi = c["so"] + C.span(c["ss"], count, levels)[1]
            src = phased_fill(op, max(16, s_hi), c["so"], 3000 + k)
            if c["kind"] == "acc":
                ora.accs(op, c["alpha"], src, c["so"], c["ss"], want[OPS.index(op)], c["do"], c["ds"], count, levels)
            else:
                ora.puts(src, c["so"], c["ss"], want[PUT], c["do"], c["ds"], count, levels)
        for i in range(nreg):
            got = np.empty(REG, dtype=np.uint8)
            assert L.gaamd_memcpy(got.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(seg[owner] + i * REG), REG) == 0
            op = OPS[i] if i < len(OPS) else 0
            if i < len(OPS):
                assert same_bits_nan_aware(got, want[i], op), (C.NAMES[op], first_mismatch(got, want[i], op))
            else:
                assert np.array_equal(got, want[i]), ("put" if i == PUT else "get", i)
        say(rank, "segment equals the replayed sequence")
    ga_amd.comex_barrier()
    ga_amd.comex_free(srcseg[rank])
    ga_amd.comex_free(seg[rank])


if __name__ == "__main__":
    main()
