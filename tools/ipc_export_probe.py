"""Which sequence makes hipIpcGetMemHandle refuse a fresh allocation?

VERDICT r2 item 2: the runtime refused ("invalid argument"), once in 6 two-rank
C5 runs, to export a fresh 64 MiB segment whose base and size were exactly the
allocation's; comex_malloc then retried with another block.  This probe drives
two processes on one GPU (the exporter A, the importer B, /opt/rocm's HIP
runtime, dmabuf IPC) through the candidate sequences, each many times, and
counts refusals:

  reuse_after_close  A exports X, B opens + closes, A frees X and allocates the
                     same size (same address) and exports again
  free_while_open    A frees X while B still maps it, reallocates, exports
  import_va_reuse    B opens A's block at VA V, closes it, then B allocates the
                     same size (the runtime may hand out V again) and exports
  export_twice       A exports the same block twice
  mixed_sizes        interleaved 64 MiB / 1 GiB blocks, the bench's C5 pattern
                     (1 GiB GA blocks and sources, then a 64 MiB check GA)
  fd_growth          open file descriptors of the exporter after each export and
                     each free, and of the importer after each open and close
                     (dmabuf IPC: an export is a file descriptor)
  fd_limit           the exporter's RLIMIT_NOFILE lowered to a few descriptors above
                     its current count: does running out of descriptors make
                     hipIpcGetMemHandle refuse, and with which error

Usage: python tools/ipc_export_probe.py [rounds]  -> one JSON line per scenario.
"""
import ctypes
import json
import multiprocessing as mp
import os
import sys

HIP = "/opt/rocm/lib/libamdhip64.so"


class Handle(ctypes.Structure):   # hipIpcMemHandle_t: 64 bytes, passed BY VALUE to hipIpcOpenMemHandle
    _fields_ = [("reserved", ctypes.c_char * 64)]


def hip():
    L = ctypes.CDLL(HIP)
    L.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    L.hipFree.argtypes = [ctypes.c_void_p]
    L.hipIpcGetMemHandle.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    L.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), Handle, ctypes.c_uint]
    L.hipIpcCloseMemHandle.argtypes = [ctypes.c_void_p]
    L.hipSetDevice.argtypes = [ctypes.c_int]
    L.hipGetErrorString.restype = ctypes.c_char_p
    L.hipDeviceSynchronize.argtypes = []
    assert L.hipSetDevice(0) == 0
    return L


def alloc(L, n):
    p = ctypes.c_void_p()
    rc = L.hipMalloc(ctypes.byref(p), n)
    assert rc == 0, rc
    return p.value


def export(L, p):
    h = ctypes.create_string_buffer(64)
    rc = L.hipIpcGetMemHandle(h, ctypes.c_void_p(p))
    return rc, h.raw


def open_h(L, raw):
    p = ctypes.c_void_p()
    h = Handle()
    ctypes.memmove(ctypes.addressof(h), raw, 64)
    rc = L.hipIpcOpenMemHandle(ctypes.byref(p), h, 1)
    return rc, p.value


def nfds():
    return len(os.listdir("/proc/self/fd"))


def worker(role, q_in, q_out, rounds):
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    L = hip()
    MB = 1 << 20
    res = {}
    while True:
        cmd = q_in.get()
        if cmd is None:
            break
        name, args = cmd
        out = {}
        if role == "A":
            if name == "reuse_after_close" or name == "free_while_open":
                size = args
                p = alloc(L, size)
                rc, raw = export(L, p)
                q_out.put(("handle", rc, raw, p))
                q_in.get()                      # B has opened (and closed, for reuse_after_close)
                assert L.hipFree(ctypes.c_void_p(p)) == 0
                p2 = alloc(L, size)
                rc2, _ = export(L, p2)
                q_out.put(("second", rc2, p2 == p))
                q_in.get()                      # B closed (free_while_open)
                rc3, _ = export(L, p2)
                q_out.put(("third", rc3))
                assert L.hipFree(ctypes.c_void_p(p2)) == 0
            elif name == "import_va_reuse":
                size = args
                p = alloc(L, size)
                rc, raw = export(L, p)
                q_out.put(("handle", rc, raw, p))
                q_in.get()                      # B done
                assert L.hipFree(ctypes.c_void_p(p)) == 0
                q_out.put(("freed",))
            elif name == "export_twice":
                p = alloc(L, args)
                rc1, raw1 = export(L, p)
                rc2, raw2 = export(L, p)
                q_out.put(("twice", rc1, rc2, raw1 == raw2))
                assert L.hipFree(ctypes.c_void_p(p)) == 0
            elif name == "fd_growth":
                trace = []
                for i in range(args):
                    f0 = nfds()
                    p = alloc(L, 64 * MB)
                    rc, raw = export(L, p)
                    f1 = nfds()
                    q_out.put(("handle", rc, raw, p))
                    q_in.get()                  # B opened and closed it
                    assert L.hipFree(ctypes.c_void_p(p)) == 0
                    trace.append((f0, f1, nfds(), rc))
                q_out.put(("fd_growth", trace))
            elif name == "fd_limit":
                import resource
                soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
                base = nfds()
                resource.setrlimit(resource.RLIMIT_NOFILE, (base + 6, hard))
                got, ps = [], []
                for i in range(24):
                    try:
                        p = alloc(L, 64 * MB)
                    except AssertionError:
                        got.append(("alloc_refused", nfds()))
                        break
                    ps.append(p)
                    rc, _ = export(L, p)
                    got.append((rc, L.hipGetErrorString(rc).decode() if rc else "", nfds()))
                    if rc:
                        break
                resource.setrlimit(resource.RLIMIT_NOFILE, (soft, hard))
                # the same export after the limit is restored
                rc_after = export(L, ps[-1])[0] if ps else None
                for p in ps:
                    L.hipFree(ctypes.c_void_p(p))
                q_out.put(("fd_limit", base, soft, hard, got, rc_after))
            elif name == "mixed":
                sizes = args
                ps = []
                rcs = []
                for s in sizes:
                    p = alloc(L, s)
                    rc, raw = export(L, p)
                    rcs.append(rc)
                    ps.append((p, raw))
                q_out.put(("mixed", rcs, [raw for _, raw in ps]))
                q_in.get()                      # B opened and closed all
                for p, _ in ps:
                    assert L.hipFree(ctypes.c_void_p(p)) == 0
                q_out.put(("freed",))
        else:   # B: the importer
            if name in ("reuse_after_close", "free_while_open"):
                _, rc, raw, p = q_in.get()
                orc, v = open_h(L, raw)
                if name == "reuse_after_close":
                    L.hipIpcCloseMemHandle(ctypes.c_void_p(v))
                q_out.put(("opened", orc))
                q_in.get()                      # A exported the second block
                if name == "free_while_open":
                    L.hipIpcCloseMemHandle(ctypes.c_void_p(v))
                q_out.put(("closed",))
            elif name == "import_va_reuse":
                _, rc, raw, p = q_in.get()
                orc, v = open_h(L, raw)
                L.hipIpcCloseMemHandle(ctypes.c_void_p(v))
                mine = alloc(L, args)
                erc, _ = export(L, mine)
                assert L.hipFree(ctypes.c_void_p(mine)) == 0
                q_out.put(("import_va_reuse", orc, mine == v, erc))
            elif name == "fd_growth":
                trace = []
                for i in range(args):
                    _, rc, raw, p = q_in.get()
                    f0 = nfds()
                    orc, v = open_h(L, raw)
                    f1 = nfds()
                    L.hipIpcCloseMemHandle(ctypes.c_void_p(v))
                    trace.append((f0, f1, nfds(), orc))
                    q_out.put(("opened",))
                q_out.put(("fd_growth_b", trace))
            elif name == "mixed":
                _, rcs, raws = q_in.get()
                vs = []
                for raw in raws:
                    orc, v = open_h(L, raw)
                    vs.append(v)
                for v in vs:
                    L.hipIpcCloseMemHandle(ctypes.c_void_p(v))
                # now allocate + export blocks of the same sizes here (the importer side
                # becoming an exporter, as a rank does at the next comex_malloc)
                erc = []
                same = 0
                for raw, v in zip(raws, vs):
                    pass
                for s in args:
                    p = alloc(L, s)
                    if p in vs:
                        same += 1
                    erc.append(export(L, p)[0])
                    L.hipFree(ctypes.c_void_p(p))
                q_out.put(("mixed_b", erc, same))
        q_out.put(("done",))


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    ctx = mp.get_context("spawn")
    qa_in, qa_out, qb_in, qb_out = ctx.Queue(), ctx.Queue(), ctx.Queue(), ctx.Queue()
    A = ctx.Process(target=worker, args=("A", qa_in, qa_out, rounds))
    B = ctx.Process(target=worker, args=("B", qb_in, qb_out, rounds))
    A.start()
    B.start()
    MB = 1 << 20
    results = {}

    def run_pair(name, arg, steps):
        qa_in.put((name, arg))
        qb_in.put((name, arg))
        return steps()

    # reuse_after_close / free_while_open
    for name in ("reuse_after_close", "free_while_open"):
        stats = {"rounds": 0, "first_export_refused": 0, "second_export_refused": 0, "same_address": 0,
                 "third_export_refused": 0, "open_failed": 0}
        for size in [64 * MB] * rounds + [1024 * MB] * max(1, rounds // 4):
            qa_in.put((name, size))
            qb_in.put((name, size))
            h = qa_out.get()
            stats["first_export_refused"] += h[1] != 0
            qb_in.put(h)
            o = qb_out.get()
            stats["open_failed"] += o[1] != 0
            qa_in.put("go")
            sec = qa_out.get()
            stats["second_export_refused"] += sec[1] != 0
            stats["same_address"] += bool(sec[2])
            qb_in.put("go")
            qb_out.get()
            qa_in.put("go")
            third = qa_out.get()
            stats["third_export_refused"] += third[1] != 0
            assert qa_out.get()[0] == "done" and qb_out.get()[0] == "done"
            stats["rounds"] += 1
        results[name] = stats
    # import_va_reuse
    stats = {"rounds": 0, "open_failed": 0, "importer_got_same_va": 0, "export_refused": 0,
             "export_refused_at_same_va": 0}
    for size in [64 * MB] * rounds + [1024 * MB] * max(1, rounds // 4):
        qa_in.put(("import_va_reuse", size))
        qb_in.put(("import_va_reuse", size))
        h = qa_out.get()
        qb_in.put(h)
        r = qb_out.get()
        stats["open_failed"] += r[1] != 0
        stats["importer_got_same_va"] += bool(r[2])
        stats["export_refused"] += r[3] != 0
        stats["export_refused_at_same_va"] += (r[3] != 0) and bool(r[2])
        qa_in.put("go")
        qa_out.get()
        assert qa_out.get()[0] == "done" and qb_out.get()[0] == "done"
        stats["rounds"] += 1
    results["import_va_reuse"] = stats
    # export_twice
    stats = {"rounds": 0, "first_refused": 0, "second_refused": 0, "same_handle": 0}
    for _ in range(max(1, rounds // 4)):
        qa_in.put(("export_twice", 64 * MB))
        qb_in.put(("noop", 0))
        t = qa_out.get()
        stats["first_refused"] += t[1] != 0
        stats["second_refused"] += t[2] != 0
        stats["same_handle"] += bool(t[3])
        assert qa_out.get()[0] == "done" and qb_out.get()[0] == "done"
        stats["rounds"] += 1
    results["export_twice"] = stats
    # mixed sizes (the bench's C5 then check-GA pattern)
    stats = {"rounds": 0, "a_refused": 0, "b_refused": 0, "b_same_va": 0}
    sizes = [1024 * MB, 1024 * MB, 64 * MB, 256 * MB, 64 * MB]
    for _ in range(max(1, rounds // 2)):
        qa_in.put(("mixed", sizes))
        qb_in.put(("mixed", sizes))
        m = qa_out.get()
        stats["a_refused"] += sum(1 for x in m[1] if x)
        qb_in.put(m)
        b = qb_out.get()
        stats["b_refused"] += sum(1 for x in b[1] if x)
        stats["b_same_va"] += b[2]
        qa_in.put("go")
        qa_out.get()
        assert qa_out.get()[0] == "done" and qb_out.get()[0] == "done"
        stats["rounds"] += 1
    results["mixed_sizes"] = stats
    # descriptors per export / open, and after free / close
    nfd = max(4, rounds)
    qa_in.put(("fd_growth", nfd))
    qb_in.put(("fd_growth", nfd))
    for _ in range(nfd):
        qb_in.put(qa_out.get())
        qb_out.get()
        qa_in.put("go")
    ta = qa_out.get()[1]
    tb = qb_out.get()[1]
    assert qa_out.get()[0] == "done" and qb_out.get()[0] == "done"
    results["fd_growth"] = {"rounds": nfd, "exporter_fds_before_export_after_export_after_free": ta[:4] + ta[-2:],
                            "exporter_fd_leak_per_round": (ta[-1][2] - ta[0][0]) / nfd,
                            "importer_fds_before_open_after_open_after_close": tb[:4] + tb[-2:],
                            "importer_fd_leak_per_round": (tb[-1][2] - tb[0][0]) / nfd}
    qa_in.put(("fd_limit", 0))
    qb_in.put(("noop", 0))
    fl = qa_out.get()
    assert qa_out.get()[0] == "done" and qb_out.get()[0] == "done"
    results["fd_limit"] = {"fds_at_start": fl[1], "nofile_soft": fl[2], "nofile_hard": fl[3],
                           "exports_rc_errstr_fds": fl[4], "export_after_limit_restored_rc": fl[5]}
    qa_in.put(None)
    qb_in.put(None)
    A.join(60)
    B.join(60)
    for k, v in results.items():
        print(json.dumps({"scenario": k, **v}), flush=True)


if __name__ == "__main__":
    main()
