#!/usr/bin/env python3
"""bench.py -- device-resident strided f64 accumulate through the ComEx C ABI.

Metric (BASELINE.json): GiB/s device-resident 2-D strided f64 accumulate,
64 MiB patch; % HBM peak.

A "step" is one comex_nbaccs call (include/comex.h; reference comex_nbaccs,
comex/src-mpi-pr/comex.c:1998-2027 -> nb_accs 6890) applying dst += alpha*src
over the workload's patch, both sides resident in HBM; the handles are waited
on (comex_wait, one 64 steps back) and comex_wait_all closes the timed region,
so every step's kernel has finished inside it.  (A blocking comex_accs returns
only after its kernel finished -- local completion, SURVEY.md 8(b) -- so a
stream of them pays one host round trip per step: --api blocking measures that.)
Default workload "H": count = {2048*8 B, 4096 rows}, src & dst leading
dimension 8192 doubles (65 536 B) -- 64 MiB of payload, 192 MiB of algorithmic
HBM traffic (src read + dst read + dst write, 24 B per element).  Steps rotate
over --sets independent buffer sets (default 8 x 512 MiB) so the 256 MiB
Infinity Cache cannot serve the working set.  Before the timed region the same
step runs for --warmup steps and then for at least --warmup-ms of wall time,
so the K timed steps do not start on a cold (clock-ramping) GPU.

value = whole-job algorithmic traffic GiB/s = ranks * steps * bytes / max-over-
ranks wall time of the K timed steps (barrier + synchronize on both sides, no
timing events inside: their marker packets between kernels cost ~0.6 us per
step, tools/edge_probe.py).  roofline.achieved = the same algorithmic bytes per
launch / the average launch duration, from HIP events recorded at both ends of
every library stream around K more launches of the same step right after the
value region (per-launch event pairs slowed the kernels by ~8 %,
profiles/r01/gapprobe_H.json), so it includes the kernel-boundary gap.  The library runs independent accumulates on two HIP
streams (ga_amd/csrc/sched.cpp), so consecutive launches overlap at their
edges: the rocprofv3 --kernel-trace summary of the same command is committed
under profiles/, and the per-launch time it agrees with is the merged busy time
of the dispatches / dispatches (tools/kernel_union.py), not AverageNs, which
counts shared time twice.  roofline.traffic = HBM bytes per launch from
rocprofv3 FETCH_SIZE/WRITE_SIZE passes of the same workload (tools/pmc_traffic.py,
profiles/pmc_latest.json) -- collected in separate profiled runs, not this one
(roofline.traffic_source says so).  cpu_baseline = the reference's own _acc
(oracle/_ref, compiled from comex/src-common/acc.h) driven per row by the
restated nb_accs odometer (comex.c:6936-6961) on P host threads, each on its
own slab of the same workload, over a bounded sample (P = 1 .. 16 reported).

Multi-GPU: one process per GPU.  Under torch.distributed.run (RANK/WORLD_SIZE
set) every process is one rank; with --gpus N > 1 and no WORLD_SIZE, bench.py
starts the N rank processes itself (before any HIP call) and forwards rank 0's
line.  Every rank accumulates into its own partition (GA owner-aligned
patches) with no data-path collective -> "scaling": "weak".
torch.distributed (gloo, CPU) only carries the bootstrap allgather/barrier and
the max-over-ranks reduction.  At N > 1 the line also carries C5 (GA_Acc into a
block-distributed 32768^2 f64 GA): M1 (every rank its own
block) and M2 (every rank the whole array: (p-1)/p of it through the remote
path over xGMI), with per-GPU HBM fraction and per-GPU xGMI bytes/s, and an
exactness check of the exchange on both remote routes: on a 4096^2 GA before any
timed C5 step (c5.exchange_precheck) and at the configured size after them
(c5.exchange_check).
"""
import argparse
import ctypes
import gc
import json
import os
import socket
import subprocess
import sys
import time
from collections import deque

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident 2-D strided f64 accumulate, 64 MiB patch; % HBM peak"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E, MI355X_MICROARCH.md chip table (8.0 TB/s)
# xGMI: 7 links per MI355X at 153.6 GB/s each counting both directions (the task
# brief's "7 links x ~153 GB/s"; MI355X_MICROARCH.md has no xGMI figure), so
# 76.8 GB/s per link per direction.  An owner pulling its peers' contributions
# (M2) is bound by the links INTO it: min(7, p - 1) x 76.8 GB/s.
XGMI_LINKS = 7
XGMI_LINK_GBS_PER_DIRECTION = 76.8
DBL, DCP = 38, 41

WORKLOADS = {
    # name: (op, count, src_stride, dst_stride, description)
    "H": (DBL, [2048 * 8, 4096], [8192 * 8], [8192 * 8],
          "2-D f64 2048x4096 patch, ld 8192 (64 MiB payload)"),
    "H8200": (DBL, [2048 * 8, 4096], [8200 * 8], [8200 * 8],
              "2-D f64 2048x4096 patch, ld 8200 (64 MiB payload)"),
    "C2": (DBL, [64 << 20], [], [], "1-D contiguous f64, 64 MiB"),
    "C3": (DBL, [4096 * 8, 4096], [8192 * 8], [8192 * 8], "2-D f64 4096x4096 patch, ld 8192 (128 MiB)"),
    "C4": (DCP, [4096, 256, 256], [4096, 1048576], [4224, 1115136],
           "3-D double-complex 256^3 patch, dst in 264x264x256 (256 MiB)"),
}
# C5: GA_Acc into a block-distributed 32768^2 f64 array (GA's REGULAR
# distribution, NGA_Create).  M1 (default): every rank NGA_Acc's its own block
# from a device-resident local buffer (owner-aligned, no exchange).  --exchange
# (M2): every rank NGA_Acc's the WHOLE array, so (p-1)/p of its patch goes to
# the other owners (pack -> owner's unpack-acc over xGMI).  SURVEY.md 8(d) C5.
GA_DIMS = [32768, 32768]
C_DBL = 1004
ESZ = {DBL: 8, DCP: 16}
SCALE = {DBL: 0.7071067811865476, DCP: 0.6 - 0.8j}


def span_bytes(count, strides):
    hi = count[0]
    for j, s in enumerate(strides):
        hi += s * (count[j + 1] - 1)
    return hi


def patch_bytes(count):
    n = 1
    for c in count:
        n *= c
    return n


# ---------------------------------------------------------------- distributed
class Dist:
    def __init__(self, n_gpus):
        self.rank = int(os.environ.get("RANK", "0"))
        self.size = int(os.environ.get("WORLD_SIZE", "1"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        self.pg = None
        if self.size > 1:
            import torch
            import torch.distributed as td
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # gloo prints "[Gloo] Rank r is connected to ..." on stdout while it connects:
            # send fd 1 to stderr meanwhile so stdout carries only the one JSON line
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                td.init_process_group("gloo", rank=self.rank, world_size=self.size)
                td.barrier()
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(saved)
            self.torch, self.td = torch, td
        if n_gpus != self.size and self.rank == 0:
            print(f"warning: --gpus {n_gpus} but WORLD_SIZE {self.size}", file=sys.stderr)

    def hooks(self):
        """bootstrap allgather/barrier for gaamd_set_bootstrap (replaces MPI_Allgather)."""
        import ga_amd
        torch, td = self.torch, self.td

        def allgather(send, recv, nbytes, ctx):
            buf = torch.frombuffer(bytearray(ctypes.string_at(send, nbytes)), dtype=torch.uint8)
            out = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(self.size)]
            td.all_gather(out, buf)
            cat = torch.cat(out).numpy()   # keep alive across the memmove
            ctypes.memmove(recv, cat.ctypes.data, nbytes * self.size)
            return 0

        def barrier(ctx):
            td.barrier()
            return 0

        self._ag = ga_amd.ALLGATHER_FN(allgather)
        self._bar = ga_amd.BARRIER_FN(barrier)
        return self._ag, self._bar

    def max(self, x):
        if self.size == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64)
        self.td.all_reduce(t, op=self.td.ReduceOp.MAX)
        return float(t.item())

    def barrier(self):
        if self.size > 1:
            self.td.barrier()


# ---------------------------------------------------------------- GPU leg
def bootstrap(L, dist):
    if dist.size > 1:
        ag, bar = dist.hooks()
        rc = L.gaamd_set_bootstrap(dist.rank, dist.size, dist.local_rank, ctypes.cast(ag, ctypes.c_void_p),
                                   ctypes.cast(bar, ctypes.c_void_p), None)
        assert rc == 0, rc


class Handles:
    """Non-blocking step handles: at most `depth` outstanding (comex_wait on the
    oldest, which has long finished when the GPU keeps up), all drained by
    comex_wait_all at the end of a region."""

    def __init__(self, L, depth=64):
        self.L, self.depth, self.q = L, depth, deque()

    def new(self):
        h = ctypes.c_int(-1)
        self.q.append(h)
        if len(self.q) > self.depth:
            assert self.L.comex_wait(ctypes.byref(self.q.popleft())) == 0
        return ctypes.byref(h)

    def drain(self):
        assert self.L.comex_wait_all(0) == 0
        self.q.clear()


def warm(step, args, first=0):
    """W warm-up steps, then more of the same step until --warmup-ms have passed
    (outside the timed region: a cold process reads 5-10 % low for its first
    milliseconds).  Returns the index of the next step."""
    i = first
    for _ in range(args.warmup):
        step(i)
        i += 1
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.warmup_ms / 1e3:
        step(i)
        i += 1
    return i


def event_region(L, run, steps, first):
    """The roofline's per-launch time: the same `steps` steps once more, right
    after the value region, bracketed by one HIP event per library stream at each
    end (first start to last end over all streams).  Kept out of the value region:
    marker packets between kernels cost ~0.6 us per step there (tools/edge_probe.py,
    profiles/r02/edge_probe.jsonl).  Returns (ms, index of the next step)."""
    n = L.gaamd_num_streams()
    streams = [L.gaamd_stream_at(i) for i in range(n)]
    ev0 = [L.gaamd_event_create() for _ in streams]
    ev1 = [L.gaamd_event_create() for _ in streams]
    for e, st in zip(ev0, streams):
        L.gaamd_event_record(e, st)
    for i in range(steps):
        run(first + i)
    for e, st in zip(ev1, streams):
        L.gaamd_event_record(e, st)
    assert L.comex_wait_all(0) == 0
    ms = max(L.gaamd_event_elapsed_ms(a, b) for a in ev0 for b in ev1)
    for e in ev0 + ev1:
        L.gaamd_event_destroy(e)
    return ms, first + steps


def run_ga(args, dist, exchange=None, steps=None, warmup_ms=None, terminate=True):
    """C5: NGA_Acc (include/ga.h; reference capi.c:2079 -> ngai_acc_common,
    global/src/onesided.c:1334) on a 32768^2 f64 GA.  NGA_Acc is GA's blocking
    call: every owner but the last through ARMCI_NbAccS, the last ARMCI_AccS
    (onesided.c:1421-1438)."""
    import ga_amd
    L = ga_amd.lib()
    if not L.comex_initialized():
        bootstrap(L, dist)
    assert L.GA_Initialize() == 0
    routes0 = ga_amd.route_counts()     # this measurement's routes (warm-up included), not the process's
    ia = ga_amd.int_array
    dims = [args.ga_dims, args.ga_dims] if args.ga_dims else GA_DIMS
    exchange = (args.exchange if exchange is None else exchange) and dist.size > 1
    steps = args.steps if steps is None else steps
    g = L.NGA_Create(C_DBL, 2, ia(dims), b"C5", None)
    assert g > 0
    blo, bhi = (ctypes.c_int * 2)(), (ctypes.c_int * 2)()
    L.NGA_Distribution(g, dist.rank, blo, bhi)
    lo, hi = ([0, 0], [dims[0] - 1, dims[1] - 1]) if exchange else (list(blo), list(bhi))
    rows, cols = hi[0] - lo[0] + 1, hi[1] - lo[1] + 1
    payload = rows * cols * 8
    if args.src_seg:   # the local buffer in this rank's segment: the direct-source route
        src_seg = ga_amd.comex_malloc(payload, dist.size)
        src, src_ptr = None, src_seg[dist.rank]
    else:
        src_seg, src = None, ga_amd.DeviceBuffer(payload)
        src_ptr = src.ptr
    ga_amd.fill(src_ptr, rows * cols, 0, 0x5EED0000 + dist.rank)
    # the local block: fill through NGA_Access (its HBM address)
    ptr, ld = ctypes.c_void_p(), (ctypes.c_int * 1)()
    L.NGA_Access(g, blo, bhi, ctypes.byref(ptr), ld)
    block_bytes = (bhi[0] - blo[0] + 1) * (bhi[1] - blo[1] + 1) * 8
    ga_amd.fill(ptr.value, block_bytes // 8, 0, 0x5EED0001 + dist.rank)
    L.NGA_Release_update(g, blo, bhi)
    ga_amd.sync()
    L.GA_Sync()
    grid = (ctypes.c_int * 2)()
    L.GA_Get_proc_grid(g, grid)
    alpha = ctypes.c_double(SCALE[DBL])
    clo, chi, cld = ia(lo), ia(hi), ia([cols])
    def step(_i):
        L.NGA_Acc(g, clo, chi, ctypes.c_void_p(src_ptr), cld, ctypes.byref(alpha))
        if args.verbose:
            print(f"rank {dist.rank}: NGA_Acc done", file=sys.stderr, flush=True)

    saved = args.warmup_ms
    if warmup_ms is not None:
        args.warmup_ms = warmup_ms
    if args.verbose:
        print(f"rank {dist.rank}: GA created, src {'segment' if src_seg else 'buffer'}, warming", file=sys.stderr,
              flush=True)
    nxt = warm(step, args)
    args.warmup_ms = saved
    ga_amd.sync()
    L.GA_Sync()
    if args.verbose:
        print(f"rank {dist.rank}: warm-up done", file=sys.stderr, flush=True)
    launch = ga_amd.last_launch()
    # value region: wall clock only (no marker packets between the steps)
    dist.barrier()
    ga_amd.sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(nxt + i)
    ga_amd.sync()
    if exchange:
        L.GA_Sync()                     # every owner has applied every contribution
    t1 = time.perf_counter()
    dist.barrier()
    elapsed = dist.max(t1 - t0)
    if exchange:
        avg_kernel_s = elapsed / steps   # the work runs on the owners' streams
    else:
        region_ms, _ = event_region(L, step, steps, nxt + steps)
        avg_kernel_s = dist.max(region_ms / 1e3 / steps)
    routes = {k: v - routes0[k] for k, v in ga_amd.route_counts().items()}
    topology = ga_amd.device_topology()
    if src is not None:
        src.free()
    L.GA_Sync()
    if src_seg is not None:
        ga_amd.comex_free(src_seg[dist.rank])
    L.GA_Destroy(g)
    if terminate:
        L.GA_Terminate()
    desc = (f"GA_Acc, {dims[0]}x{dims[1]} f64 GA on a {grid[0]}x{grid[1]} grid, "
            + ("every rank the whole array (M2)" if exchange else f"own {rows}x{cols} block (M1)"))
    return dict(op=DBL, desc=desc, payload=payload, alg_bytes=3 * payload, elems=rows * cols, elapsed=elapsed,
                avg_kernel_s=avg_kernel_s, launch=launch, streams=L.gaamd_num_streams(), exchange=exchange,
                steps=steps, block_bytes=block_bytes, array_bytes=dims[0] * dims[1] * 8, routes=routes,
                topology=topology)


def run_gpu(args, dist, finalize=True):
    import ga_amd
    L = ga_amd.lib()
    if args.workload == "C5":
        return run_ga(args, dist, terminate=finalize)
    bootstrap(L, dist)
    assert ga_amd.comex_init() == 0
    for kv in args.tune or []:
        k, v = kv.split("=")
        ga_amd.set_tuning(k, int(v))

    op, count, sstr, dstr, desc = WORKLOADS[args.workload]
    esz = ESZ[op]
    levels = len(count) - 1
    sbytes, dbytes = span_bytes(count, sstr), span_bytes(count, dstr)
    payload = patch_bytes(count)
    elems = payload // esz
    xfer = getattr(args, "xfer", "acc")
    # src read + dst read + dst write; a strided put/get reads and writes once
    alg_bytes = 3 * payload if xfer == "acc" else 2 * payload
    type_code = 0                      # f64 reals (dcpl = 2 f64 each)

    # --sets independent (src, dst) pairs; rotate so the MALL cannot hold them.
    # --exchange: dst are comex_malloc segments and rank r accumulates into rank
    # r+1's (the remote path, pack -> owner's unpack-acc).
    exchange = args.exchange and dist.size > 1
    target = (dist.rank + 1) % dist.size if exchange else dist.rank
    # --self-packed (N=1): accumulates to this rank take the packed route (pack ->
    # staging -> progress thread unpack-acc), forced as COMEX_ENABLE_ACC_SELF=0 /
    # COMEX_ENABLE_ACC_SMP=0 force it in the reference (comex.c:450-471)
    self_packed = args.self_packed and not exchange
    seg_dst = exchange or self_packed      # the packed and direct routes need a registered dst
    sets, segs, src_segs = [], [], []
    for i in range(args.sets):
        if args.src_seg:                   # the source patch in this rank's own segment
            sseg = ga_amd.comex_malloc(sbytes, dist.size)
            s = None
            src_segs.append(sseg)
            sptr = sseg[dist.rank]
        elif args.host_src:                # pinned host memory: GA's local (MA) buffer
            s = ga_amd.DeviceBuffer(sbytes, host=True)
            sptr = s.ptr
        else:
            s = ga_amd.DeviceBuffer(sbytes)
            sptr = s.ptr
        ga_amd.fill(sptr, sbytes // 8, type_code, 0x5EED0000 + dist.rank)
        if seg_dst:
            seg = ga_amd.comex_malloc(dbytes, dist.size)
            ga_amd.fill(seg[dist.rank], dbytes // 8, type_code, 0x5EED0001 + dist.rank + 977 * i)
            segs.append(seg)
            sets.append((s, None, sptr))
        else:
            d = ga_amd.DeviceBuffer(dbytes)
            ga_amd.fill(d.ptr, dbytes // 8, type_code, 0x5EED0001 + dist.rank + 977 * i)
            sets.append((s, d, sptr))
    ga_amd.sync()
    if seg_dst or args.src_seg:
        L.comex_barrier(0)

    keep, sp = ga_amd.scale_buffer(op, SCALE[op])
    ss, ds, cnt = ga_amd.int_array(sstr), ga_amd.int_array(dstr), ga_amd.int_array(count)
    if seg_dst:
        ptrs = [(ctypes.c_void_p(sp), ctypes.c_void_p(seg[target])) for (_, _, sp), seg in zip(sets, segs)]
    else:
        ptrs = [(ctypes.c_void_p(sp), ctypes.c_void_p(d.ptr)) for _, d, sp in sets]
    pipeline = args.pipeline and not exchange
    packed = [ga_amd.DeviceBuffer(payload) for _ in sets] if pipeline else []
    hd = Handles(L)
    nb = args.api == "nb"

    def step(i):
        sp_, dp_ = ptrs[i % len(ptrs)]
        if pipeline:
            # the remote path's two kernels back to back on one GPU: pack (comex.c:1267)
            # then the owner's unpack-acc (comex.c:4238-4268)
            pk = ctypes.c_void_p(packed[i % len(packed)].ptr)
            rc = L.gaamd_pack(sp_, ss, cnt, levels, pk, None) or \
                L.gaamd_unpack_acc(op, sp, pk, dp_, ds, cnt, levels, None)
        elif xfer == "put":             # comex_puts (comex.c:6342): local src -> the target's patch
            rc = (L.comex_nbputs(sp_, ss, dp_, ds, cnt, levels, target, 0, hd.new()) if nb else
                  L.comex_puts(sp_, ss, dp_, ds, cnt, levels, target, 0))
        elif xfer == "get":             # comex_gets (comex.c:6617): the target's patch -> local buffer
            rc = (L.comex_nbgets(dp_, ds, sp_, ss, cnt, levels, target, 0, hd.new()) if nb else
                  L.comex_gets(dp_, ds, sp_, ss, cnt, levels, target, 0))
        else:
            rc = (L.comex_nbaccs(op, sp, sp_, ss, dp_, ds, cnt, levels, target, 0, hd.new()) if nb else
                  L.comex_accs(op, sp, sp_, ss, dp_, ds, cnt, levels, target, 0))
        if rc:
            raise RuntimeError(f"step returned {rc}")

    nxt = warm(step, args)
    warmup_steps = nxt
    hd.drain()
    ga_amd.sync()
    launch = ga_amd.last_launch()

    # value region: barrier + sync on both sides, wall clock, no timing events; no
    # garbage collection inside it (as timeit): a collection pass there is host time
    # the GPU work does not need
    gc.disable()
    L.comex_barrier(0)
    dist.barrier()
    ga_amd.sync()
    # BENCH_STAMPS=1 (diagnostic runs only, never the driver's): the library's host
    # stamps (gaamd_diag "stamps", CLOCK_BOOTTIME) of the first call and of the closing wait,
    # read after the region, for tools/region_edges.py to place on a kernel trace
    stamps_on = os.environ.get("BENCH_STAMPS") == "1"
    st_buf = (ctypes.c_ulonglong * 8)()

    def value_region(first):
        first_stamps = None
        if stamps_on:
            L.gaamd_diag(b"stamps", 1, None, 0)
        b0 = time.clock_gettime_ns(time.CLOCK_BOOTTIME)
        t0 = time.perf_counter()
        step(first)
        t_first = time.perf_counter()
        if stamps_on:
            L.gaamd_diag(b"stamps", -1, st_buf, 8)
            first_stamps = list(st_buf[:5])
        for i in range(1, args.steps):
            step(first + i)
        t_enq = time.perf_counter()
        # every step's kernel has finished: comex_wait_all synchronises every library
        # stream (hipStreamSynchronize each), i.e. all GPU work of this rank
        bw = time.clock_gettime_ns(time.CLOCK_BOOTTIME)
        hd.drain()
        if seg_dst:
            L.comex_fence_all(0)            # remote completion: the owner has applied every request
        t1 = time.perf_counter()
        b1 = time.clock_gettime_ns(time.CLOCK_BOOTTIME)
        # boottime_ns: the region's ends on the clock rocprofv3 stamps kernels with,
        # so a profiled run can place the first kernel's start and the last one's end
        prof = {"first_call_us": round((t_first - t0) * 1e6, 1),
                "enqueue_all_us": round((t_enq - t0) * 1e6, 1), "total_us": round((t1 - t0) * 1e6, 1),
                "boottime_ns": [b0, b1]}
        if stamps_on:
            L.gaamd_diag(b"stamps", 0, st_buf, 8)
            prof["stamps_ns"] = {"region_start": b0, "first_call": first_stamps, "wait_call_py": bw,
                                 "wait": list(st_buf[5:8]), "region_end": b1}
        return t1 - t0, prof

    elapsed, region_profile = value_region(nxt)
    gc.enable()
    dist.barrier()
    elapsed = dist.max(elapsed)
    nxt += args.steps
    # diagnostics only (BENCH_DIAG_REGIONS=n): n more regions shaped exactly like
    # the value region, to show its spread; `value` stays the first region
    diag = []
    for _ in range(int(os.environ.get("BENCH_DIAG_REGIONS", "0"))):
        L.comex_barrier(0)
        dist.barrier()
        ga_amd.sync()
        e, prof = value_region(nxt)
        nxt += args.steps
        diag.append(dict(prof, us_per_step=round(e / args.steps * 1e6, 2)))
    if seg_dst:
        avg_kernel_s = elapsed / args.steps   # the work runs on the owners' streams / progress thread
    else:
        # roofline: the same K steps again inside per-stream HIP events
        region_ms, nxt = event_region(L, step, args.steps, nxt)
        avg_kernel_s = dist.max(region_ms / 1e3 / args.steps)
    blocking = None
    if nb and xfer == "acc" and not pipeline and not exchange and not seg_dst:
        # the blocking API beside the headline: the same K steps through
        # comex_accs, each returning after its kernel -- a host round trip per step,
        # the call GA's NGA_Acc makes for its last owner (onesided.c:1421-1438)
        # the call through a prototype-free function object with every argument already a
        # ctypes object: no per-argument conversion in the loop (ctypes' argtypes path cost
        # ~2-3 us of Python per call, 5-7 % of a 38 us step, that a C caller -- GA --
        # never pays; tools/blocking_lib_probe.cpp times the same call from C)
        raw = ctypes.CDLL(ga_amd._lib.LIB_PATH).comex_accs
        raw.restype = ctypes.c_int
        c_op, c_lv, c_tg, c_zero = ctypes.c_int(op), ctypes.c_int(levels), ctypes.c_int(target), ctypes.c_int(0)
        bargs = [(c_op, sp, sp_, ss, dp_, ds, cnt, c_lv, c_tg, c_zero) for sp_, dp_ in ptrs]
        for i in range(args.warmup):   # W untimed calls, as every timed region here has
            if raw(*bargs[(nxt + i) % len(bargs)]):
                raise RuntimeError("blocking warm-up step failed")
        nxt += args.warmup
        L.comex_barrier(0)
        dist.barrier()
        ga_amd.sync()
        tb = time.perf_counter()
        for i in range(args.steps):
            if raw(*bargs[(nxt + i) % len(bargs)]):
                raise RuntimeError("blocking step failed")
        tb = dist.max(time.perf_counter() - tb)
        nxt += args.steps
        # the same K blocking calls issued from C (gaamd_time_blocking_accs): what GA's C /
        # Fortran NGA_Acc -> ARMCI_AccS sees, without the interpreter's per-call cost
        srcs = (ctypes.c_void_p * len(ptrs))(*[p_[0].value for p_ in ptrs])
        dsts = (ctypes.c_void_p * len(ptrs))(*[p_[1].value for p_ in ptrs])
        # W untimed calls of the C loop first, as every timed region here has a warm-up
        if args.warmup and not L.gaamd_time_blocking_accs(op, sp, srcs, ss, dsts, ds, cnt, levels, target, len(ptrs),
                                                          args.warmup):
            raise RuntimeError("blocking warm-up (C loop) failed")
        L.comex_barrier(0)
        dist.barrier()
        ga_amd.sync()
        ncall = max(args.steps, 100)   # at least 100 calls: a 20-call mean is one slow call away from noise
        ns = L.gaamd_time_blocking_accs(op, sp, srcs, ss, dsts, ds, cnt, levels, target, len(ptrs), ncall)
        if not ns:
            raise RuntimeError("blocking step (C loop) failed")
        tc = dist.max(ns * 1e-9) * args.steps / ncall   # per K steps, as the Python figure
        blocking = {"api": "comex_accs per step (blocking: returns after its kernel)",
                    "value": round(dist.size * alg_bytes * args.steps / tb / 2 ** 30, 2),
                    "hbm_peak_frac": round(alg_bytes * args.steps / tb / (HBM_PEAK_GBS * 1e9), 4),
                    "ms_per_step": round(tb / args.steps * 1e3, 4),
                    "caller": "Python (ctypes, one call per step)",
                    "c_caller": {"value": round(dist.size * alg_bytes * args.steps / tc / 2 ** 30, 2),
                                 "hbm_peak_frac": round(alg_bytes * args.steps / tc / (HBM_PEAK_GBS * 1e9), 4),
                                 "ms_per_step": round(tc / args.steps * 1e3, 4),
                                 "calls": ncall,
                                 "how": "the same calls from a C loop (libga_amd_diag.so gaamd_time_blocking_accs, over the public comex_accs)"}}

    res = dict(op=op, desc=desc, payload=payload, alg_bytes=alg_bytes, elems=elems, elapsed=elapsed,
               avg_kernel_s=avg_kernel_s, launch=launch, streams=L.gaamd_num_streams(), pipeline=pipeline,
               xfer=xfer, warmup_steps=warmup_steps, region_profile=region_profile, diag_regions=diag,
               blocking=blocking)
    for b in packed:
        b.free()
    if (dist.size == 1 and not args.no_host and xfer == "acc" and not pipeline and not self_packed
            and args.api == "nb"):
        res["host"] = host_inclusive(L, ga_amd, op, count, sstr, dstr, levels, sbytes, dbytes, payload, alg_bytes)
    routes = ga_amd.route_counts()
    for s, d, _ in sets:
        if s is not None:
            s.free()
        if d is not None:
            d.free()
    if segs or src_segs:
        L.comex_barrier(0)
        for seg in segs + src_segs:
            ga_amd.comex_free(seg[dist.rank])
    res["exchange"] = exchange
    res["self_packed"] = self_packed
    res["routes"] = routes
    res["topology"] = ga_amd.device_topology()
    if finalize:
        ga_amd.comex_finalize()
    return res


def c5_extras(args, dist, wd=None):
    """N > 1: C5 in the same job -- M1, every rank NGA_Acc's its
    own block (owner-aligned, HBM-bound), and M2, every rank NGA_Acc's the whole
    array, (p-1)/p of it through the remote path (pack into exported staging HBM,
    the owner's unpack-acc reading it over xGMI).  Few steps: these are reported
    beside the headline, not as `value`."""
    out = {}
    # every cross-GPU operation FIRST: remote strided acc of every
    # type, put and get with seeded random descriptors, accv/putv/getv, rmw, between
    # rank pairs, exact by closed form (ga_amd/xcheck.py, no oracle), the routes it
    # exercised summed over the ranks; a MISMATCH is rerun at once under the
    # conservative publication mode and classified
    if not args.no_xcheck:
        if wd is not None:
            wd.phase = "xdev_check"
        from ga_amd.xcheck import xdev_check_diagnosed
        try:
            out["xdev_check"] = xdev_check_diagnosed(dist.rank, dist.size, budget_s=args.xcheck_s)
        except Exception as e:   # a failed call is a finding, not a lost line (the watchdog covers a hang)
            out["xdev_check"] = {"result": "ERROR", "rank": dist.rank, "error": repr(e)[:500]}
    # the exchange's exactness on a small GA (4096^2, both routes) before any timed C5
    # step: on the first run over separate GPUs a visibility bug
    # reads as exchange_precheck MISMATCH, not as a plausible rate
    if wd is not None:
        wd.phase = "exchange_precheck"
    assert ga_amd_lib().GA_Initialize() == 0
    out["exchange_precheck"] = {route: exchange_check_diagnosed(dist, src_seg, n=4096) for route, src_seg in
                                (("buffer_src", False), ("segment_src", True))}
    saved = args.src_seg
    m2 = max(1, args.c5_steps // 2)
    for mode, exchange, steps, src_seg in (("M1", False, args.c5_steps, False), ("M2", True, m2, False),
                                           ("M2_src_in_segment", True, m2, True)):
        if args.verbose:
            print(f"rank {dist.rank}: C5 {mode} starts", file=sys.stderr, flush=True)
        if wd is not None:
            wd.phase = mode
        args.src_seg = src_seg
        r = run_ga(args, dist, exchange=exchange, steps=steps, warmup_ms=0.0, terminate=False)
        args.src_seg = saved
        p = dist.size
        t = r["elapsed"] / steps
        d = {"desc": r["desc"], "steps": steps, "ms_per_step": round(t * 1e3, 3),
             "GiB_per_s_job": round(p * r["alg_bytes"] / t / 2 ** 30, 1)}
        if exchange:
            # each owner receives (p-1) blocks' worth of its peers' contributions per step
            # (packed rows, or their sources read in place); they cross xGMI only when
            # the ranks sit on different GPUs (say which)
            inbound = (p - 1) * r["block_bytes"]
            rate = inbound / t / 1e9
            topo = r.get("topology") or {}
            gpus, per_gpu = topo.get("gpus_on_node", 1), topo.get("ranks_on_gpu", p)
            if gpus == p and topo.get("peer_loads") != "off":
                links = min(XGMI_LINKS, p - 1)
                peak = links * XGMI_LINK_GBS_PER_DIRECTION
                d["xgmi_GBps_per_gpu"] = round(rate, 1)
                d["roofline"] = {"bound": "xgmi", "achieved": round(rate, 1), "peak": round(peak, 1),
                                 "unit": "GB/s", "frac": round(rate / peak, 4),
                                 "peak_basis": f"{links} links into each owner x {XGMI_LINK_GBS_PER_DIRECTION} GB/s "
                                               "per direction (153.6 GB/s per link, both directions)",
                                 "achieved_basis": "(p-1) x owner block bytes per GPU per step / step time"}
            else:
                # ranks share GPUs: the peers' bytes are read from the same HBM, not over xGMI
                d["inter_rank_GBps_per_gpu"] = round(rate, 1)
                d["roofline"] = None
                d["xgmi_note"] = (f"{p} ranks on {gpus} GPU(s) ({per_gpu} per GPU): "
                                  + ("no byte crossed xGMI" if gpus == 1 else
                                     "part of the traffic stays on one GPU") + "; no xGMI roofline")
            d["devices_distinct"] = gpus
            d["note"] = ("whole-array accumulate by every rank; value counts 3 x payload of HBM-side traffic per rank; "
                         + ("the local buffer lies in the rank's comex segment: owners on other GPUs accumulate "
                            "straight from it (direct-source route, no pack); ranks sharing a GPU the one-pass route"
                            if src_seg else
                            "the local buffer is a plain device buffer: owners on other GPUs pack -> staging -> owner "
                            "unpack-acc; ranks sharing a GPU the one-pass route"))
            d["routes"] = r.get("routes")
        else:
            d["hbm_peak_frac_per_gpu"] = round(r["alg_bytes"] / t / (HBM_PEAK_GBS * 1e9), 4)
        out[mode] = d
    # the exactness check runs at the configured GA size, not a reduced one
    n_chk = args.ga_dims if args.ga_dims else GA_DIMS[0]
    if wd is not None:
        wd.phase = "exchange_check"
    out["exchange_check"] = {route: exchange_check_diagnosed(dist, src_seg, n=n_chk) for route, src_seg in
                             (("buffer_src", False), ("segment_src", True))}
    # diagnostics only (BENCH_CHECK_LOOPS=n): the exchange check n more times per route,
    # with the first mismatch's details (never the driver's runs)
    loops = int(os.environ.get("BENCH_CHECK_LOOPS", "0"))
    if loops:
        rep = {}
        for route, src_seg in (("buffer_src", False), ("segment_src", True)):
            bad, first = 0, None
            for _ in range(loops):
                r = c5_exchange_check(dist, src_seg, n=n_chk)
                if r["result"] != "exact":
                    bad += 1
                    first = first or r
            rep[route] = {"loops": loops, "mismatches": bad, "first_mismatch": first}
        out["exchange_check_loops"] = rep
    ga_amd_lib().GA_Terminate()
    return out


def exchange_check_diagnosed(dist, src_seg, n):
    """c5_exchange_check, and on MISMATCH once more in this process under the
    conservative publication mode (gaamd_diag "publish": a system-scope release on
    every library stream before every post and fence): a mismatch that clears is a
    visibility fault, one that persists a logic fault."""
    res = c5_exchange_check(dist, src_seg, n=n)
    if res["result"] == "exact":
        return res
    L = ga_amd_lib()
    old = (ctypes.c_ulonglong * 1)()
    L.gaamd_diag(b"publish", 1, old, 1)
    try:
        again = c5_exchange_check(dist, src_seg, n=n)
    finally:
        L.gaamd_diag(b"publish", int(old[0]), None, 0)
    res["conservative_rerun"] = again
    res["diagnosis"] = ("clears: visibility" if again["result"] == "exact" else "persists: logic")
    return res


def ga_amd_lib():
    import ga_amd
    return ga_amd.lib()


def c5_exchange_check(dist, src_seg, n=4096):
    """Cross-GPU exactness of the exchange (the driver's N > 1 run is the first on
    separate GPUs): every rank NGA_Acc's a whole n x n f64 GA from a source of the
    constant 2**rank (alpha 1, the array zeroed first), so every element must read
    exactly 2**p - 1 afterwards -- a lost, doubled or stale contribution shows as a
    wrong element and its value says whose.  The source is a plain device buffer
    (packed route to other GPUs, one-pass to ranks on the same GPU) or lies in the
    rank's segment (direct-source route to other GPUs, one-pass on the same GPU)."""
    import ga_amd
    L = ga_amd.lib()
    ia = ga_amd.int_array
    g = L.NGA_Create(C_DBL, 2, ia([n, n]), b"C5chk", None)
    assert g > 0
    L.GA_Zero(g)
    L.GA_Sync()
    nbytes = n * n * 8
    seg, buf = None, None
    if src_seg:
        seg = ga_amd.comex_malloc(nbytes, dist.size)
        ptr = seg[dist.rank]
    else:
        buf = ga_amd.DeviceBuffer(nbytes)
        ptr = buf.ptr
    ga_amd.fill_const(ptr, nbytes, float(2 ** dist.rank))   # on the GPU: no n^2 host array at 32768^2
    ga_amd.sync()
    routes0 = ga_amd.route_counts()
    alpha = ctypes.c_double(1.0)
    L.NGA_Acc(g, ia([0, 0]), ia([n - 1, n - 1]), ctypes.c_void_p(ptr), ia([n]), ctypes.byref(alpha))
    ga_amd.sync()
    L.GA_Sync()
    routes = {k: v - routes0[k] for k, v in ga_amd.route_counts().items()}
    blo, bhi = (ctypes.c_int * 2)(), (ctypes.c_int * 2)()
    L.NGA_Distribution(g, dist.rank, blo, bhi)
    rows, cols = bhi[0] - blo[0] + 1, bhi[1] - blo[1] + 1
    out = np.empty(rows * cols)
    L.NGA_Get(g, blo, bhi, out.ctypes.data_as(ctypes.c_void_p), ia([cols]))
    want = float(2 ** dist.size - 1)
    bad = int(np.count_nonzero(out != want))
    sample = None if not bad else float(out[np.nonzero(out != want)[0][0]])
    L.GA_Sync()
    if seg is not None:
        ga_amd.comex_free(seg[dist.rank])
    if buf is not None:
        buf.free()
    L.GA_Destroy(g)
    worst = int(dist.max(float(bad)))
    res = {"array": f"{n}x{n} f64", "expect_every_element": want, "wrong_elements_max_over_ranks": worst,
           "result": "exact" if worst == 0 else "MISMATCH", "routes_rank": routes}
    if worst:
        # which rank's block, and what its first wrong element reads (2^p - 1 minus a
        # missing contribution 2^k, or plus a doubled one, says whose)
        bad_rank = int(dist.max(float(dist.rank) if bad else -1.0))
        res["a_rank_with_wrong_elements"] = bad_rank
        res["its_wrong_elements"] = int(dist.max(float(bad) if dist.rank == bad_rank else -1.0))
        res["its_first_wrong_value"] = dist.max(sample if dist.rank == bad_rank else -1e300)
    return res


PCIE_GBS = 63.0   # PCIe Gen5 x16 per direction (MI355X_MICROARCH.md host link, spec)


def host_inclusive(L, ga_amd, op, count, sstr, dstr, levels, sbytes, dbytes, payload, alg_bytes, iters=5):
    """The path as north_star states it: it starts and ends in host memory (MA
    segments that feed MPI/OFI).  Reported beside `value`, never as it.  Each case
    one untimed call, then `iters` timed ones (median and best):
      staged_*     : hipMemcpy2D of the src and the dst PATCH host -> HBM (the rows of
                     the patch only, not the whole leading-dimension span), the same
                     strided accumulate kernel as the headline, hipMemcpy2D of the dst
                     patch HBM -> host: 3 x payload over PCIe, one direction at a time
      ga_host_src_*: comex_accs with src in host memory and dst in HBM -- GA's NGA_Acc
                     from a local (MA) buffer into a block the GPU owns (onesided.c:
                     1403-1438): the kernel reads the src patch over PCIe (pinned:
                     directly; pageable: the library registers its pages per call),
                     1 x payload over PCIe
      both_host_pinned: comex_accs with both sides in pinned host memory (zero-copy):
                     2 x payload read + 1 x payload written over PCIe
    rate = algorithmic bytes (3 x payload, as `value`) / time; roofline = the
    PCIe-bound time (PCIE_GBS per direction: H2D + D2H bytes when the copies take
    turns, the busier direction when a kernel moves both at once) / time."""
    out = {"unit": "GiB/s", "note": "host-inclusive rates beside value (never value); rate = 3 x payload / time",
           "pcie_peak_GBps_per_direction": PCIE_GBS,
           "pcie_peak_basis": "PCIe Gen5 x16, 63 GB/s per direction (MI355X_MICROARCH.md)"}
    keep, sp = ga_amd.scale_buffer(op, SCALE[op])
    ss, ds, cnt = ga_amd.int_array(sstr), ga_amd.int_array(dstr), ga_amd.int_array(count)
    dsrc, ddst = ga_amd.DeviceBuffer(sbytes), ga_amd.DeviceBuffer(dbytes)
    rows = payload // count[0]
    # a 2-D view of the patch for hipMemcpy2D: rows of count[0] bytes; 1-D patches one
    # row, 3-D ones (C4) need a contiguous outer level -- only 1/2-level patches here
    two_d = levels <= 1 or all(sstr[j] == sstr[j - 1] * count[j] and dstr[j] == dstr[j - 1] * count[j]
                               for j in range(1, levels))
    spitch = sstr[0] if levels else count[0]
    dpitch = dstr[0] if levels else count[0]

    def timed(fn):
        fn()
        ts = []
        for _ in range(iters):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return ts[len(ts) // 2], ts[0]

    def entry(t_med, t_best, h2d, d2h, overlapped, how):
        # the PCIe-bound time: one direction after the other for the staged copies,
        # both directions at once for a kernel reading and writing host memory
        peak_t = (max(h2d, d2h) if overlapped else h2d + d2h) / (PCIE_GBS * 1e9)
        return {"value": round(alg_bytes / t_med / 2 ** 30, 2), "best": round(alg_bytes / t_best / 2 ** 30, 2),
                "ms": round(t_med * 1e3, 3), "pcie_h2d_bytes": h2d, "pcie_d2h_bytes": d2h,
                "roofline": {"bound": "pcie", "achieved": round((h2d + d2h) / t_med / 1e9, 2),
                             "peak": PCIE_GBS * (2 if overlapped and h2d and d2h else 1), "unit": "GB/s",
                             "frac": round(peak_t / t_med, 4),
                             "basis": ("H2D and D2H concurrently, bound by the busier direction" if overlapped
                                       else "one direction at a time")},
                "how": how}

    for kind in ("pinned", "pageable"):
        if kind == "pinned":
            hs, hd = ga_amd.DeviceBuffer(sbytes, host=True), ga_amd.DeviceBuffer(dbytes, host=True)
            hsp, hdp = hs.ptr, hd.ptr
            L.gaamd_memset(ctypes.c_void_p(hsp), 1, sbytes)
            L.gaamd_memset(ctypes.c_void_p(hdp), 0, dbytes)
        else:
            hs_a, hd_a = np.ones(sbytes, np.uint8), np.zeros(dbytes, np.uint8)
            hsp, hdp = hs_a.ctypes.data, hd_a.ctypes.data
        if two_d:
            def staged():
                L.gaamd_memcpy2d(ctypes.c_void_p(dsrc.ptr), spitch, ctypes.c_void_p(hsp), spitch, count[0], rows)
                L.gaamd_memcpy2d(ctypes.c_void_p(ddst.ptr), dpitch, ctypes.c_void_p(hdp), dpitch, count[0], rows)
                if L.comex_accs(op, sp, ctypes.c_void_p(dsrc.ptr), ss, ctypes.c_void_p(ddst.ptr), ds, cnt, levels,
                                0, 0):
                    raise RuntimeError("staged accumulate failed")
                L.gaamd_memcpy2d(ctypes.c_void_p(hdp), dpitch, ctypes.c_void_p(ddst.ptr), dpitch, count[0], rows)
            out[f"staged_{kind}"] = entry(*timed(staged), 2 * payload, payload, False,
                                          f"hipMemcpy2D src+dst patch H2D ({kind}), strided accumulate kernel, "
                                          "hipMemcpy2D dst patch D2H")

        def host_src():
            if L.comex_accs(op, sp, ctypes.c_void_p(hsp), ss, ctypes.c_void_p(ddst.ptr), ds, cnt, levels, 0, 0):
                raise RuntimeError("host-source accumulate failed")
            L.comex_fence_all(0)
        out[f"ga_host_src_{kind}"] = entry(*timed(host_src), payload, 0, True,
                                           f"comex_accs, src patch in {kind} host memory, dst in HBM "
                                           "(GA's NGA_Acc from a local buffer, onesided.c:1403-1438)")
        if kind == "pinned":
            def both_host():
                if L.comex_accs(op, sp, ctypes.c_void_p(hsp), ss, ctypes.c_void_p(hdp), ds, cnt, levels, 0, 0):
                    raise RuntimeError("host accumulate failed")
                L.comex_fence_all(0)
            out["both_host_pinned"] = entry(*timed(both_host), 2 * payload, payload, True,
                                            "comex_accs, src and dst patch in pinned host memory (zero-copy kernel)")
            hs.free()
            hd.free()
    dsrc.free()
    ddst.free()
    return out


# ---------------------------------------------------------------- CPU leg
def run_cpu_baseline(workload, seconds, threads):
    """The reference's _acc per row (oracle/_ref), or the restatement if _ref is absent.
    SURVEY.md 8(d): P host workers, each on its own slab of the patch (oracle/mt_split.h),
    for P = 1, 2, 4, 8, 16 (up to `threads`: the GPU box's CPU share per GPU is 16); each
    as many full steps as fit in ~seconds/#P (at least 2).  `value` is the P = `threads`
    rate; every P is reported beside it.  Provenance: the reference's own _acc (acc.h,
    compiled into oracle/_ref) for the arithmetic, driven by the restated nb_accs
    odometer (comex.c:6936-6961) -- comex.c itself is not built here."""
    from oracle import Oracle, Ref, ref_available
    op, count, sstr, dstr, _ = WORKLOADS[workload]
    sbytes, dbytes = span_bytes(count, sstr), span_bytes(count, dstr)
    src = np.empty(sbytes, np.uint8)
    dst = np.empty(dbytes, np.uint8)
    o = Oracle()
    o.fill(src[: sbytes // 8 * 8].view(np.float64), 0x5EED0000)
    o.fill(dst[: dbytes // 8 * 8].view(np.float64), 0x5EED0001)
    if ref_available():
        impl, kind = Ref(), "reference"
    else:
        impl, kind = o, "port"
    levels = len(count) - 1
    rates, notes = {}, []
    ps = sorted({p for p in (1, 2, 4, 8, 16) if p <= threads} | {max(1, threads)})
    for p in ps:
        impl.accs_mt(op, SCALE[op], src, 0, sstr, dst, 0, dstr, count, levels, p)   # warm-up (page-in)
        n, t0 = 0, time.perf_counter()
        while True:
            impl.accs_mt(op, SCALE[op], src, 0, sstr, dst, 0, dstr, count, levels, p)
            n += 1
            el = time.perf_counter() - t0
            if (el >= seconds / len(ps) and n >= 2) or n >= 10000:
                break
        rates[p] = round(3 * patch_bytes(count) * n / el / 2 ** 30, 3)
        notes.append(f"P={p}: {n} full {workload} steps in {el:.1f} s")
    P = max(rates)
    # the progress-rank path (ACC_SMP=0): pack (comex.c:1267-1328) then
    # unpack-accumulate (4238-4268) on one core -- the restatement (oracle), as comex.c
    # itself is not built here; no MPI copy in between, so an upper bound for that path
    packed = None
    o.accs_packed(op, SCALE[op], src, 0, sstr, dst, 0, dstr, count, levels)   # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        o.accs_packed(op, SCALE[op], src, 0, sstr, dst, 0, dstr, count, levels)
        n += 1
        el = time.perf_counter() - t0
        if (el >= seconds / (len(ps) + 1) and n >= 2) or n >= 10000:
            break
    packed = {"value": round(3 * patch_bytes(count) * n / el / 2 ** 30, 3), "unit": "GiB/s", "cores": 1,
              "kind": "port", "sample": f"{n} full {workload} steps in {el:.1f} s: oracle pack + unpack-acc "
                                        "(comex.c:1267-1328, 4238-4268), one core, no MPI transfer"}
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": rates[P], "unit": "GiB/s", "cores": P, "kind": kind, "single_core_value": rates[1],
            "provenance": ("reference _acc (comex/src-common/acc.h compiled into oracle/_ref) + restated odometer "
                           "(comex.c:6936-6961)") if kind == "reference" else "oracle restatement (oracle/comex_oracle.c)",
            "by_workers": {str(k): v for k, v in sorted(rates.items())},
            "packed_path_single_core": packed,
            "host": {"cpu": model, "nproc": os.cpu_count()},
            "sample": "; ".join(notes) + "; P host threads each on its own slab of the patch (outer level); "
                      + ("reference comex/src-common/acc.h _acc (HAVE_BLAS=0, gcc -O2) per row, "
                         "odometer of comex.c:6936-6961" if kind == "reference" else "oracle restatement")}


def load_traffic(workload, launch_bytes):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if it is for
    this workload (profiles/pmc_latest.json, written by tools/pmc_traffic.py)."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if d.get("workload") == workload:
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def free_port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    return port


def spawn_ranks(n):
    """--gpus N > 1 without a launcher: start N rank processes of this script
    (one per GPU, LOCAL_RANK = GPU index) before this process touches HIP, wait
    for all, forward rank 0's stdout line; exit status = the worst rank's."""
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    # a rank that dies leaves the others blocked in a collective: stop them all then
    rcs = [None] * n
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        if any(rc not in (None, 0) for rc in rcs):
            for p in procs:
                if p.poll() is None:
                    p.kill()
            rcs = [p.wait() for p in procs]
            break
        time.sleep(0.05)
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--warmup-ms", type=float, default=500.0,
                    help="after --warmup steps, keep warming with the same step for this long (outside the timing)")
    ap.add_argument("--api", default="nb", choices=["nb", "blocking"],
                    help="nb: comex_nbaccs steps (handles waited 64 back, comex_wait_all at the end); "
                         "blocking: comex_accs (returns after its kernel finished)")
    ap.add_argument("--workload", default="H", choices=sorted(WORKLOADS) + ["C5"])
    ap.add_argument("--sets", type=int, default=8, help="rotating buffer sets (MALL defeat)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="host workers of the CPU baseline (the GPU box's CPU share is 16 per GPU)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host", action="store_true",
                    help="N=1: skip the host-inclusive block (patch H2D/D2H and host-source rates)")
    ap.add_argument("--exchange", action="store_true",
                    help="N>1: rank r accumulates into rank r+1's partition (remote path, SURVEY 8(d) M2)")
    ap.add_argument("--streams", type=int, default=0,
                    help="library HIP streams (COMEX_AMD_STREAMS; 0 = the library default: 2, or 1 when ranks share the GPU)")
    ap.add_argument("--self-packed", action="store_true",
                    help="N=1: force the packed route for accumulates to self (COMEX_ENABLE_ACC_SELF/SMP=0)")
    ap.add_argument("--src-seg", action="store_true",
                    help="sources in this rank's comex_malloc segment (the direct-source route for --exchange)")
    ap.add_argument("--host-src", action="store_true",
                    help="sources in pinned host memory (GA's local MA buffer); with --exchange: remote "
                         "accumulates from a host source")
    ap.add_argument("--pipeline", action="store_true",
                    help="step = pack + unpack-acc (the remote path's two kernels) instead of the fused acc")
    ap.add_argument("--xfer", default="acc", choices=["acc", "put", "get"],
                    help="operation per step: strided accumulate (the metric), or strided put / get")
    ap.add_argument("--tune", action="append", help="key=value tuning knob (gaamd_set_tuning)")
    ap.add_argument("--ga-dims", type=int, default=0, help="C5: square GA of this size instead of 32768^2")
    ap.add_argument("--c5-steps", type=int, default=4, help="N>1: timed C5 M1 steps (M2: half as many)")
    ap.add_argument("--no-extras", action="store_true", help="N>1: skip the C5 M1/M2 measurements")
    ap.add_argument("--no-xcheck", action="store_true", help="N>1: skip the cross-GPU self-check (xdev_check)")
    ap.add_argument("--xcheck-s", type=float, default=30.0,
                    help="N>1: seconds after which the cross-GPU self-check stops after its current round")
    ap.add_argument("--extras-timeout", type=float, default=300.0,
                    help="N>1: seconds the C5 extras may take before the headline line is printed without them")
    ap.add_argument("--verbose", action="store_true", help="progress lines on stderr")
    args = ap.parse_args()
    if os.environ.get("BENCH_STACK_DUMP_S"):   # diagnostics: where a hung rank is stuck
        import faulthandler
        faulthandler.dump_traceback_later(int(os.environ["BENCH_STACK_DUMP_S"]), exit=False)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    # Load libga_amd (and with it /opt/rocm's HIP runtime) before torch: torch's
    # wheel bundles its own libamdhip64 with the same SONAME, and whichever loads
    # first serves the library.  The bundled runtime hangs in hipIpcOpenMemHandle
    # of a 2 GiB segment while a 1 GiB one is mapped (tools/malloc_repro.py,
    # profiles/r02/README.md); /opt/rocm's does not.
    import ga_amd
    ga_amd.lib()
    if args.streams:
        os.environ["COMEX_AMD_STREAMS"] = str(args.streams)
    if args.self_packed:   # read once at comex_init
        for k in ("COMEX_ENABLE_ACC_SELF", "COMEX_ENABLE_ACC_SMP"):
            os.environ[k] = "0"

    dist = Dist(args.gpus)
    extras_on = dist.size > 1 and not args.no_extras and args.workload != "C5"
    r = run_gpu(args, dist, finalize=not extras_on)
    # the headline line is complete before the extras start: should the extras (the
    # first cross-GPU exchange of a job) not finish, the watchdog still prints it
    line = make_line(args, dist, r, ga_amd) if dist.rank == 0 else None
    if extras_on:
        wd = ExtrasWatchdog(args.extras_timeout, dist.rank, line)
        # the C5 exchange needs every same-node peer mapped by IPC; a rank that could not
        # map one would abort there, so the extras are skipped (by every rank) instead
        unmapped = int(dist.max(float(ga_amd.lib().gaamd_peers_unmapped())))
        if unmapped:
            ga_amd.lib().comex_finalize()
            c5 = {"skipped": f"a rank could not map {unmapped} same-node peer(s) by IPC at comex_init"}
        else:
            c5 = c5_extras(args, dist, wd)
        if not wd.cancel():
            time.sleep(3600)   # the watchdog owns the line and the exit status
        if line is not None:
            line["c5"] = c5
    if line is not None:
        print(json.dumps(line), flush=True)


EXTRAS_TIMEOUT_STATUS = 3


class ExtrasWatchdog:
    """N > 1: the C5 extras run after the headline is measured.  If they have not
    finished after `seconds` (a hang in an exchange no one-GPU box could rehearse),
    rank 0 prints the headline line with the extras marked as timed out, every rank
    dumps its Python stacks to stderr and the job ends with status
    EXTRAS_TIMEOUT_STATUS (3): the headline was measured and is reported, and the
    hang is a failure the caller sees, not a success with a note.
    The line is printed exactly once: cancel() and fire() settle it under a lock."""

    def __init__(self, seconds, rank, line):
        import threading
        self.phase = "start"
        self.rank, self.line = rank, line
        self.lock = threading.Lock()
        self.settled = False
        self.t = threading.Timer(seconds, self.fire, args=(seconds,))
        self.t.daemon = True
        self.t.start()

    def fire(self, seconds):
        import faulthandler
        with self.lock:
            if self.settled:        # the extras finished first: main prints the line
                return
            self.settled = True
            print(f"rank {self.rank}: C5 extras still in phase {self.phase!r} after {seconds:.0f} s; stacks:",
                  file=sys.stderr, flush=True)
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
            if self.line is not None:
                self.line["c5"] = {"timed_out": f"C5 extras did not finish within {seconds:.0f} s "
                                                f"(phase {self.phase!r} on rank 0); the headline above was "
                                                "measured before they started"}
                print(json.dumps(self.line), flush=True)
            os._exit(EXTRAS_TIMEOUT_STATUS)

    def cancel(self):
        """True: the extras finished in time and the caller prints the line; False:
        the watchdog fired (and is ending the process)."""
        with self.lock:
            self.t.cancel()
            if self.settled:
                return False
            self.settled = True
            return True


def make_line(args, dist, r, ga_amd):
    n = dist.size
    alg = r["alg_bytes"]
    value = n * args.steps * alg / r["elapsed"] / 2 ** 30
    achieved = alg / r["avg_kernel_s"] / 1e9
    traffic = load_traffic(args.workload, alg) if r.get("xfer", "acc") == "acc" else None
    cpu = None
    if not args.no_cpu and n == 1 and args.workload != "C5" and r.get("xfer", "acc") == "acc":
        cpu = run_cpu_baseline(args.workload, args.cpu_seconds, args.cpu_threads)
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_note": (f"{r.get('warmup_steps', args.warmup)} untimed steps: --warmup {args.warmup}, then the "
                        f"same step until {args.warmup_ms:.0f} ms had passed"),
        "ms_per_step": round(r["elapsed"] / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64" if r["op"] == DBL else "c128",
        "data": ("synthetic (splitmix64, SURVEY.md 8(d)); %s, %d rotating buffer sets"
                 % ("src in pinned host memory, dst in HBM" if args.host_src else "device-resident src+dst",
                    args.sets)),
        "config": {"workload": args.workload, "patch": r["desc"], "payload_bytes": r["payload"],
                   "algorithmic_bytes_per_step": alg,
                   "parallelism": (("GA_Acc of the whole array by every rank: remote owners apply the "
                                    "contributions (over xGMI when the ranks sit on different GPUs)"
                                    if args.workload == "C5" else
                                    f"exchange x{n}: rank r -> rank r+1 through the owner's route "
                                    "(over xGMI when the ranks sit on different GPUs)")
                                   if r["exchange"] else f"owner-aligned x{n} (no collective)"),
                   "kernel": r["launch"]},
        "payload_GiB_per_s": round(value / (3 if r.get("xfer", "acc") == "acc" else 2), 2),
        "hbm_peak_frac": round(value * 2 ** 30 / (dist.size * HBM_PEAK_GBS * 1e9), 4),   # per GPU
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic,
                     "traffic_source": ("profiles/pmc_latest.json: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of "
                                        "this workload's kernel (tools/pmc_traffic.py, gfx950 FETCH_SIZE x2), "
                                        "collected in separate profiled runs, not this one") if traffic else None,
                     "kernel_ms_avg": round(r["avg_kernel_s"] * 1e3, 4),
                     "timing": ("HIP events at both ends of every library stream around K more launches of the "
                                "same step right after the value region (first start to last end) / K"),
                     "frac_kind": ("event-pair figure: an HIP event pair per library stream around K extra launches; "
                                   "the rocprofv3 summaries under profiles/ give the per-launch AverageNs on one "
                                   "stream and the merged busy time per dispatch on the default two streams, which "
                                   "bracket it"),
                     "streams": r["streams"],
                     "rocprof_check": ("consecutive launches overlap on the library streams: compare kernel_ms_avg "
                                       "with the merged busy time per dispatch of the rocprofv3 kernel trace "
                                       "(tools/kernel_union.py), not with AverageNs"
                                       if r["streams"] > 1 else "compare kernel_ms_avg with rocprofv3 AverageNs")},
        "cpu_baseline": cpu,
        "api": ("comex_nbaccs per step, handles waited 64 back + comex_wait_all" if args.api == "nb"
                else "comex_accs per step (blocking: returns after its kernel)"),
    }
    line["hip_runtime"] = ga_amd.lib().gaamd_hip_runtime().decode()
    topo = r.get("topology")
    if n > 1 and topo:
        # how the ranks sat on the node's GPUs (a one-GPU rehearsal must not
        # read as an xGMI run), the C5 entries say the same per measurement
        line["topology"] = dict(topo, ranks=n)
        if topo["ranks_on_gpu"] > 1:
            line["roofline"]["note"] = (f"{topo['ranks_on_gpu']} ranks share each GPU: a rank's kernel time "
                                        "includes the other ranks' traffic on the same HBM")
    if n > 1:
        line["cpu_baseline_note"] = "the CPU baseline is measured at N = 1 only (rank 0), per the bench contract"
    if r.get("region_profile"):
        line["value_region"] = r["region_profile"]   # host-clock marks inside the timed region
    if r.get("diag_regions"):
        line["diag_regions"] = r["diag_regions"]
    if r.get("blocking"):
        line["blocking_api"] = r["blocking"]   # same K steps through the blocking call, after the value region
    if r.get("xfer", "acc") != "acc":
        line["metric"] = f"GiB/s device-resident strided f64 {r['xfer']} (comex_{r['xfer']}s), not the headline metric"
        line["config"]["step"] = f"comex_{r['xfer']}s of the patch; algorithmic bytes = 2 x payload (read + write)"
    if r.get("pipeline"):
        # two kernels per step on one stream: pack moves 2x payload, unpack-acc 3x
        moved = 5 * r["payload"]
        line["config"]["step"] = "gaamd_pack + gaamd_unpack_acc on one stream (pack-buffer traffic not credited in value)"
        line["roofline"]["achieved"] = round(moved / r["avg_kernel_s"] / 1e9, 1)
        line["roofline"]["frac"] = round(moved / r["avg_kernel_s"] / 1e9 / HBM_PEAK_GBS, 4)
        line["roofline"]["traffic"] = None
        line["roofline"]["timing"] = "bytes both kernels move (5 x payload) / (event-pair region / steps)"
    if r.get("routes") and (r["exchange"] or r.get("self_packed") or args.src_seg):
        line["routes"] = r["routes"]
    if r.get("self_packed"):
        line["metric"] = "GiB/s strided f64 accumulate to self through the packed route (not the headline metric)"
        line["config"]["step"] = ("comex_nbaccs to self with COMEX_ENABLE_ACC_SELF=0 / COMEX_ENABLE_ACC_SMP=0: pack -> "
                                  "staging -> progress thread unpack-acc; value credits 3 x payload per step")
        line["roofline"] = None
        line["moved_GBps"] = round(5 * r["payload"] * args.steps / r["elapsed"] / 1e9, 1)
    if r["exchange"]:
        # the kernels run on the owners' streams: no single-kernel roofline; the
        # per-step time is the whole exchange (pack, hand-off, unpack-acc)
        line["roofline"] = None
        line["exchange_achieved_GBps_per_rank"] = round(achieved, 1)
    if "host" in r:
        line["host_inclusive"] = r["host"]
    return line


if __name__ == "__main__":
    main()
