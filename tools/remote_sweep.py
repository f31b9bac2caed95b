#!/usr/bin/env python3
"""Remote accumulate by message size, two ranks (self-spawned; on one GPU they share
the card): rank 0 accumulates a 2-D f64 patch (rows of min(size, 16 KiB), leading
dimension 2 x row) from a plain device buffer into rank 1's segment, as
comex/testing/perf_strided.c does between two processes:
    latency   : comex_accs + comex_fence_proc per operation (remote completion)
    pipelined : `iters` comex_nbaccs back to back, waits, one fence at the end
One JSON line per size on rank 0's stdout, with the route each took.  Compare
COMEX_AMD_ONE_PASS_MIN settings (the one-pass route's floor) or COMEX_AMD_ONE_PASS=0.
Tuning evidence, not product code."""
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    # --ranks N --all-to-one: every rank but 0 accumulates into rank 0 at once (contention
    # for one owner's memory), rank 0 reports the slowest rank's pipelined time
    nranks = 2
    all_to_one = False
    argv = sys.argv[1:]
    if "--ranks" in argv:
        k = argv.index("--ranks")
        nranks = int(argv[k + 1])
        del argv[k:k + 2]
    if "--all-to-one" in argv:
        argv.remove("--all-to-one")
        all_to_one = True
    if "RANK" not in os.environ:
        import socket
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = str(s.getsockname()[1])
        s.close()
        procs = [subprocess.Popen([sys.executable, "-u", __file__] + sys.argv[1:],
                                  env=dict(os.environ, RANK=str(r), WORLD_SIZE=str(nranks), LOCAL_RANK=str(r),
                                           MASTER_ADDR="127.0.0.1", MASTER_PORT=port, COMEX_AMD_JOBID="rs" + port),
                                  stdout=None if r == 0 else subprocess.DEVNULL)
                 for r in range(nranks)]
        sys.exit(max(p.wait() for p in procs))
    import ga_amd
    rank = int(os.environ["RANK"])
    assert ga_amd.comex_init() == 0
    L = ga_amd.lib()
    size_w = int(os.environ["WORLD_SIZE"])
    cap = 64 << 20
    seg = ga_amd.comex_malloc(2 * cap, size_w)
    src = ga_amd.DeviceBuffer(2 * cap)
    L.gaamd_memset(src.ptr, 0, 2 * cap)
    L.gaamd_memset(seg[rank], 0, 2 * cap)
    ga_amd.sync()
    ga_amd.comex_barrier()
    sizes = [int(x) for x in (argv or [str(8 << 10), str(64 << 10), str(256 << 10), str(1 << 20),
                                       str(4 << 20), str(16 << 20)])]
    if all_to_one:
        import ctypes
        for size in sizes:
            row = min(size, 16384)
            rows = size // row
            count, stride, levels = [row, rows], [2 * row], (1 if rows > 1 else 0)
            iters = 200 if size <= (1 << 20) else 50
            ga_amd.comex_barrier()
            t0 = time.perf_counter()
            if rank != 0:
                hs = []
                for _ in range(iters):
                    rc, h = ga_amd.comex_nbaccs(38, 0.5, src.ptr, stride, seg[0], stride, count, levels, 0)
                    hs.append(h)
                    if len(hs) > 32:
                        ga_amd.comex_wait(hs.pop(0))
                for h in hs:
                    ga_amd.comex_wait(h)
                L.comex_fence_proc(0, 0)
            mine = (ctypes.c_double * 1)(time.perf_counter() - t0)
            ga_amd.comex_barrier()
            L.armci_msg_dgop(mine, 1, b"max")   # the slowest requester
            if rank == 0:
                print(json.dumps({"mode": "all_to_one", "ranks": size_w, "size": size,
                                  "us_per_op_slowest": round(mine[0] / iters * 1e6, 2),
                                  "job_GBps_alg": round(3 * size * iters * (size_w - 1) / mine[0] / 1e9, 1),
                                  "one_pass_min": os.environ.get("COMEX_AMD_ONE_PASS_MIN", "default"),
                                  "one_pass": os.environ.get("COMEX_AMD_ONE_PASS", "1")}), flush=True)
        sizes = []
    if rank == 0:
        for size in sizes:
            row = min(size, 16384)
            rows = size // row
            count = [row, rows]
            stride = [2 * row]
            levels = 1 if rows > 1 else 0
            iters = 400 if size <= (1 << 20) else 100
            r0 = ga_amd.route_counts()
            for _ in range(20):
                ga_amd.comex_accs(38, 0.5, src.ptr, stride, seg[1], stride, count, levels, 1)
            L.comex_fence_proc(1, 0)
            lat = []
            for _ in range(iters):
                t0 = time.perf_counter()
                ga_amd.comex_accs(38, 0.5, src.ptr, stride, seg[1], stride, count, levels, 1)
                L.comex_fence_proc(1, 0)
                lat.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            hs = []
            for _ in range(iters):
                rc, h = ga_amd.comex_nbaccs(38, 0.5, src.ptr, stride, seg[1], stride, count, levels, 1)
                hs.append(h)
                if len(hs) > 32:
                    ga_amd.comex_wait(hs.pop(0))
            for h in hs:
                ga_amd.comex_wait(h)
            L.comex_fence_proc(1, 0)
            pipe = (time.perf_counter() - t0) / iters
            r1 = ga_amd.route_counts()
            print(json.dumps({"size": size, "latency_us_median": round(statistics.median(lat) * 1e6, 2),
                              "pipelined_us_per_op": round(pipe * 1e6, 2),
                              "pipelined_GBps_alg": round(3 * size / pipe / 1e9, 1),
                              "routes": {k: r1[k] - r0[k] for k in r1},
                              "one_pass_min": os.environ.get("COMEX_AMD_ONE_PASS_MIN", "default")}), flush=True)
    ga_amd.comex_barrier()
    src.free()
    assert ga_amd.comex_free(seg[rank]) == 0
    ga_amd.comex_finalize()


if __name__ == "__main__":
    main()
