"""Worker for the multi-process tests (one rank per process).

Modes:
  boot-env   : built-in node-shm bootstrap from RANK/WORLD_SIZE; bootstrap
               self-test only (no GPU).
  boot-gloo  : torch.distributed gloo as the bootstrap hooks; self-test only.
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
    mode = sys.argv[1]
    rank, size = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import ga_amd
    L = ga_amd.lib()
    if mode in ("boot-gloo", "remote-gloo"):
        ag, bar = torch_hooks(rank, size)
        keep = (ag, bar)  # noqa: F841
        assert L.gaamd_set_bootstrap(rank, size, rank, ctypes.cast(ag, ctypes.c_void_p),
                                     ctypes.cast(bar, ctypes.c_void_p), None) == 0
    if mode.startswith("boot"):
        assert L.gaamd_bootstrap_selftest(5) == 0
        assert L.gaamd_rank() == rank and L.gaamd_size() == size
        print(f"RANK {rank} OK", flush=True)
        return
    remote_test(L, rank, size)
    print(f"RANK {rank} OK", flush=True)


def remote_test(L, rank, size):
    import ga_amd
    from oracle import Oracle
    ora = Oracle()
    DBL = 38
    assert ga_amd.comex_init() == 0
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

    # remote strided get of the previous rank's patch
    out = np.zeros((90, 120), dtype=np.float64)
    assert ga_amd.comex_gets(seg[prv] + (7 + 11 * ld) * 8, [ld * 8], out.ctypes.data, [120 * 8], count, 1,
                             prv) == 0
    ga_amd.comex_fence_all()
    pb = (np.arange(ld * ncol, dtype=np.float64) % 1000 + 1000 * prv).reshape(ncol, ld)
    exp = pb[11:101, 7:127] + total * src[:, :120]
    assert np.array_equal(out, exp), f"rank {rank}: remote get mismatch"

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

    ga_amd.comex_barrier()
    assert ga_amd.comex_free(seg[rank]) == 0
    ga_amd.comex_finalize()


if __name__ == "__main__":
    main()
