"""world_size-2 multi-process coverage.

CPU (no GPU): the rank bootstrap both ways the runtime supports -- the built-in
node shared-memory rendezvous (RANK/WORLD_SIZE from the environment) and
torch.distributed gloo as the allgather/barrier hooks.
GPU: two ranks on one MI355X exercise comex_malloc + IPC mapping, the remote
accumulate through the owner's progress thread, and remote put/get.
"""
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _progress_file(mode):
    """On a gpurun box (GRAFT_REPO_ROOT set) the ranks' output is also appended, line
    by line, to gpurun_out/progress/<mode>.log as it comes: a long multi-rank test
    then shows activity (the box takes 3 silent minutes for a hang)."""
    root = os.environ.get("GRAFT_REPO_ROOT")
    if not root:
        return None
    d = os.path.join(root, "gpurun_out", "progress")
    os.makedirs(d, exist_ok=True)
    return open(os.path.join(d, f"{mode}.log"), "a", buffering=1)


def launch(mode, n=2, timeout=240, nodes=None, extra_env=None):
    """nodes: node id of every rank (COMEX_AMD_NODE), None = all on this host."""
    import threading
    import time
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, COMEX_AMD_JOBID=f"t{port}", COMEX_AMD_STAGING_MB="16",
                   TEST_STACK_DUMP_S=str(max(10, timeout - 15)))
        if nodes is not None:
            env["COMEX_AMD_NODE"] = str(nodes[r])
            env["TEST_NODES"] = ",".join(str(x) for x in nodes)
            env["COMEX_AMD_WIRE_ADDR"] = "127.0.0.1"
        env.update(extra_env or {})
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "mp_worker.py"), mode], cwd=ROOT, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    prog = _progress_file(mode)
    outs = [[] for _ in procs]

    def drain(r, p):
        for line in p.stdout:
            outs[r].append(line)
            if prog:
                prog.write(f"[{time.strftime('%H:%M:%S')} rank {r}] {line}")

    readers = [threading.Thread(target=drain, args=(r, p), daemon=True) for r, p in enumerate(procs)]
    for t in readers:
        t.start()
    deadline = time.monotonic() + timeout
    try:
        for p in procs:
            p.wait(timeout=max(1.0, deadline - time.monotonic()))
    except subprocess.TimeoutExpired:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for t in readers:
            t.join(5)
        tails = [f"--- rank {r} ---\n" + "".join(o)[-2000:] for r, o in enumerate(outs)]
        raise AssertionError(f"{mode}: ranks did not finish in {timeout} s\n" + "\n".join(tails))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for t in readers:
        t.join(10)
    if prog:
        prog.close()
    res = [(p.returncode, "".join(o)) for p, o in zip(procs, outs)]
    for r, (rc, out) in enumerate(res):
        assert rc == 0 and f"RANK {r} OK" in out, f"rank {r} rc={rc}\n{out[-3000:]}"
    return [out for _, out in res]


def test_bootstrap_env_shm_two_ranks():
    launch("boot-env")


def test_bootstrap_torch_gloo_two_ranks():
    launch("boot-gloo")


def test_bootstrap_env_shm_four_ranks():
    launch("boot-env", n=4)


@pytest.mark.parametrize("n", [2, 5])
def test_vmm_descriptor_exchange_cpu(n):
    """The vmm allocator's descriptor exchange (vmm.cpp: per-process datagram sockets,
    SCM_RIGHTS, messages keyed by (rank, allocation number)) on the CPU: every rank
    passes a memfd per round to every other and reads the ones it received back."""
    launch("boot-fdx", n=n)


@pytest.mark.parametrize("nodes", [[0, 1], [0, 0, 1, 1], [1, 0, 1, 2]])
def test_bootstrap_several_nodes_and_wire(nodes):
    """Per-node shm + cross-node collectives through the hooks + TCP PING frames."""
    launch("boot-nodes", n=len(nodes), nodes=nodes)


@pytest.mark.gpu
def test_remote_acc_put_get_two_ranks_one_gpu():
    launch("remote", n=2, timeout=120)


@pytest.mark.gpu
def test_remote_put_then_acc_same_patch_no_fence():
    """A non-blocking put then an accumulate into the same remote patch with no
    fence: the accumulate lands after the put (advisor finding, comex.cpp)."""
    launch("order", n=2, timeout=120)


@pytest.mark.gpu
def test_remote_across_devices():
    """One rank per MI355X of the box (2..8): each opens the others' segments and
    staging by IPC on other devices; remote acc/put/get/accv/getv/putv over xGMI
    (peer memory read with system-scope loads, puts applied by the owner), the
    put/acc ordering case, random strided descriptors between two GPUs (every op,
    overlapping and sub-aligned rows, all source kinds), and the full-size C5 exchange check (32768^2 f64 GA,
    M1 + M2 on both routes, exact).  Needs a multi-GPU box (skipped on one)."""
    import ga_amd
    ndev = ga_amd.lib().gaamd_device_count()
    if ndev < 2:
        pytest.skip("one GPU visible: the cross-device case needs a multi-GPU node")
    n = min(ndev, 8)
    launch("remote", n=n, timeout=180, extra_env={"TEST_DISTINCT_DEVICES": "1"})
    launch("order", n=n, timeout=180)
    launch("rdesc", n=2, timeout=170)   # random descriptors from GPU 0 into GPU 1's segment
    launch("xcheck", n=n, timeout=240)  # the bench's cross-GPU self-check, every rank pair shift
    launch("c5full", n=n, timeout=420, extra_env={"COMEX_AMD_STAGING_MB": "256", "TEST_DISTINCT_DEVICES": "1"})


@pytest.mark.gpu
@pytest.mark.parametrize("mode,n", [("remote", 2), ("remote", 3), ("order", 2), ("directsrc", 3), ("c1", 2),
                                    ("stress", 3), ("scatremote", 3)])
def test_cross_device_path_forced_on_one_gpu(mode, n):
    """COMEX_AMD_PEER_LOADS=all treats every other rank's memory as another GPU's
    (the path test_remote_across_devices takes on a multi-GPU node): the owner
    reads peer staging / segments with system-scope loads, on its pull streams,
    pulling ordered chunks and io-vector requests into local scratch first; puts
    and putv into peer memory go through the owner; gets/getv read with
    system-scope loads.  Same exact checks as the ordinary runs."""
    env = {"COMEX_AMD_PEER_LOADS": "all"}
    if mode == "stress":
        env["COMEX_AMD_STAGING_MB"] = "1"
    launch(mode, n=n, timeout=180, extra_env=env)


@pytest.mark.gpu
def test_cross_device_c5_exchange_forced_on_one_gpu():
    """The C5 exchange (M1 + M2, both routes, exact) on 4 ranks with every other
    rank's memory treated as another GPU's (COMEX_AMD_PEER_LOADS=all), 8192^2 GA."""
    launch("c5full", n=4, timeout=240, extra_env={"COMEX_AMD_PEER_LOADS": "all", "TEST_C5_N": "8192"})


@pytest.mark.gpu
def test_remote_three_ranks_gloo_hooks():
    launch("remote-gloo", n=3, timeout=120)


@pytest.mark.gpu
@pytest.mark.parametrize("nodes", [[0, 1], [0, 0, 1, 1]])
def test_remote_across_nodes_wire(nodes):
    """Ranks on different (simulated) nodes: acc/put/get/accv/getv/putv through the
    MPI-PR message protocol over TCP (wire.cpp); [0,0,1,1] mixes IPC and wire."""
    launch("remote-gloo", n=len(nodes), timeout=120, nodes=nodes)


@pytest.mark.gpu
def test_remote_across_nodes_wire_small_chunks():
    """Payloads cut into many row-range frames (1 MiB pinned chunks)."""
    launch("remote-gloo", n=2, timeout=120, nodes=[0, 1], extra_env={"COMEX_AMD_WIRE_MB": "1"})


@pytest.mark.gpu
def test_ga_layer_across_nodes():
    launch("ga-gloo", n=3, timeout=120, nodes=[0, 0, 1])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 4])
def test_ga_layer_nga_acc(n):
    """NGA_Create/NGA_Acc/NGA_Put/NGA_Get/NGA_Access over n ranks on one GPU."""
    launch("ga", n=n, timeout=120)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,n,nodes,staging", [("stress", 3, None, "1"), ("stress-gloo", 4, None, "16"),
                                                  ("stress-gloo", 3, [0, 0, 1], "1")])
def test_stress_random_programs(mode, n, nodes, staging):
    """Seeded random programs of remote/local accumulates (blocking, non-blocking,
    host or HBM source, 1-D..3-D, io-vector), puts, gets and fences on every rank
    at once; each rank checks its segment against all ranks' programs replayed
    (integer-valued f64: exact in any order).  A 1 MiB staging ring forces
    row-range chunking; nodes [0,0,1] mixes IPC and the wire protocol."""
    launch(mode, n=n, timeout=150, nodes=nodes, extra_env={"COMEX_AMD_STAGING_MB": staging})


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["same-gpu", "cross-device", "cross-device-1MiB-staging", "packed", "wire"])
def test_random_remote_descriptors(variant):
    """Seeded random strided descriptors (every op, 0..7 levels, overlapping and zero
    strides, offsets below the natural alignment) accumulated, put and got between
    two ranks on every route: the one-pass route (same GPU), the packed and direct-
    source routes with every peer treated as another GPU (also with a 1 MiB staging
    ring, so rows travel as row ranges), the packed route forced by the reference's
    SMP toggles, and the wire protocol between simulated nodes.  One writer: the
    owner's segment must equal the oracle replaying the sequence, byte for byte."""
    base = int(os.environ.get("RDESC_SEED", "3"))   # soak runs set another base
    env = {"same-gpu": {"RDESC_SEED": str(base)},
           "cross-device": {"COMEX_AMD_PEER_LOADS": "all", "RDESC_SEED": str(base)},
           "cross-device-1MiB-staging": {"COMEX_AMD_PEER_LOADS": "all", "COMEX_AMD_STAGING_MB": "1",
                                         "RDESC_SEED": str(base + 1)},
           "packed": {"COMEX_ENABLE_ACC_SMP": "0", "COMEX_ENABLE_PUT_SMP": "0", "RDESC_SEED": str(base + 2)},
           "wire": {"RDESC_SEED": str(base + 3)}}[variant]
    if variant == "wire":
        launch("rdesc-gloo", n=2, timeout=170, nodes=[0, 1], extra_env=env)
    else:
        launch("rdesc", n=2, timeout=170, extra_env=env)


@pytest.mark.gpu
@pytest.mark.parametrize("n,seed", [(3, "0"), (4, "5"), (4, "11"), (3, "17")])
def test_stress_random_programs_one_pass_everywhere(n, seed):
    """The same random programs with the one-pass route taken by every device-source
    accumulate into a rank of this GPU, however small (COMEX_AMD_ONE_PASS_MIN=1):
    hundreds of memory-lock hand-offs per rank between requesters and owners that
    accumulate into their own segments, on-demand completion marks, non-blocking
    waits and fences interleaved with puts and gets -- exact."""
    launch("stress", n=n, timeout=150, extra_env={"COMEX_AMD_ONE_PASS_MIN": "1", "STRESS_SEED": seed,
                                                  "STRESS_OPS": "800"})


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 3])
def test_comex_test_acc_restated(n):
    """comex/testing/test.c test_acc + test_cplx_acc (1028-1235) for ndim 1..7:
    TIMES*nproc accumulates of a host patch (alpha 0.1 / (0, 0.1)) into the far
    corner of every rank's array, checked at the reference's rel 1e-4 (exactly
    on one rank, where the order is fixed)."""
    launch("testacc", n=n, timeout=150)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 3])
def test_comex_test_dim_restated(n):
    """comex/testing/test.c test_dim (526-609) + test_nbdim (667-802) for ndim
    1..7: random strided patches of a host array put into rank proc's array and
    got back into another random position, exact comparison; blocking to
    nproc-1-me, then all ndim non-blocking to get_next_RRproc's targets."""
    launch("testdim", n=n, timeout=150)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 3, 4])
def test_ga_reference_acc_tests_restated(n):
    """global/testing/test.F:596-725 (disjoint and overlapping ga_acc; double,
    double complex, float and int) and ngatest_src/ndim_NGA_ACC.src (random
    sub-ranges of another rank's block, ndim 1..7; int, double, double complex)
    on n ranks, exact against acc.h's expression order."""
    launch("garef", n=n, timeout=150)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 3])
def test_comex_test_vector_restated(n):
    """comex/testing/test.c test_vector (1240-1386: triangular comex_putv pieces of
    a random 2-D patch, comex_getv of the whole patch, exact) and test_vector_acc
    (1394-1491: even/odd single-element comex_accv runs from every rank into rank
    0, TIMES*nproc times, rel 1e-4; exact on one rank)."""
    launch("testvec", n=n, timeout=150)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 3])
def test_armci_test_acc_restated(n):
    """armci/testing/test.c test_acc (896-976) through ARMCI_Malloc/ARMCI_AccS
    (ARMCI_NbAccS + ARMCI_WaitAll for odd ndim)/ARMCI_AllFence/ARMCI_GetS, ndim
    1..7, rel 1e-4 as the reference (exact on one rank)."""
    launch("armciacc", n=n, timeout=150)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,n,nodes", [("scatremote", 1, None), ("scatremote", 3, None),
                                          ("scatremote-gloo", 3, [0, 0, 1])])
def test_remote_scatter_acc_large(mode, n, nodes):
    """comex_accv of 20 000 single-float pairs from every rank to every rank, many
    repeated destinations, sources in HBM (even ranks) or pageable host memory (odd
    ranks): the owner orders repeats on its GPU (launch_iov_runs) and host sources
    are gathered into one upload; bit-exact against each source's pairs replayed in
    order.  nodes [0,0,1] sends the third rank's traffic over the wire protocol."""
    launch(mode, n=n, timeout=150, nodes=nodes)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 3])
def test_ga_ndim_scatter_acc_gather_restated(n):
    """global/testing/ngatest_src/ndim_NGA_SCATTER_ACC.src + ndim_NGA_GATHER.src:
    distinct random elements per rank (crossing owner blocks), scatter-acc then
    per-element get, gather vs get; ndim 1..7, int/double/double complex, exact."""
    launch("ngags", n=n, timeout=150)


@pytest.mark.gpu
@pytest.mark.parametrize("n,nodes", [(1, None), (2, None), (3, None), (3, [0, 0, 1]), (2, [0, 1])])
def test_armci_message_groups_rmw_mutexes(n, nodes):
    """message.c / groups.c / rmw / mutexes / values / flags / domains / Memget /
    armci_read/write_strided over n ranks; with `nodes` the cross-node cases go
    through the wire protocol's FETCH_AND_ADD / SWAP / LOCK / UNLOCK frames."""
    launch("armcimisc-gloo" if nodes else "armcimisc", n=n, timeout=120, nodes=nodes)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2])
def test_packed_route_forced_by_comex_enable_toggles(n):
    """COMEX_ENABLE_{ACC,PUT}_{SELF,SMP}=0 (comex.c:438-471): accumulates and
    puts to this rank, and same-node puts, take the packed route (pack ->
    staging -> progress thread unpack) as the reference's tests force it; the
    whole remote suite still matches the oracle.  With n=1 every operation is to
    self, so the route is exercised on a single rank."""
    toggles = {"COMEX_ENABLE_ACC_SELF": "0", "COMEX_ENABLE_ACC_SMP": "0", "COMEX_ENABLE_PUT_SELF": "0",
               "COMEX_ENABLE_PUT_SMP": "0", "COMEX_AMD_VERBOSE": "1"}
    outs = launch("remote", n=n, timeout=120, extra_env=toggles)
    assert "acc to self packed, put to self packed, same-node put packed" in outs[0], outs[0][-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2])
def test_reference_route_toggles_packed_iov_get(n):
    """The rest of the reference's route toggles (comex.c:413-573): with SELF/SMP off
    for accumulates, puts and gets, COMEX_ENABLE_{ACC,PUT,GET}_PACKED=0 sends every
    strided operation row by row as contiguous ones (nb_accs 6918-6961),
    COMEX_ENABLE_{ACC,PUT,GET}_IOV=0 every io-vector pair by pair (nb_accv 7342-7351),
    and gets go through the owner (nb_get's OP_GET, 6188-6214: the owner packs into the
    requester's staging).  The whole remote suite stays exact against the oracle,
    and each of the three routes ran (gaamd_toggle_counts)."""
    toggles = {k: "0" for k in ("COMEX_ENABLE_ACC_SELF", "COMEX_ENABLE_ACC_SMP", "COMEX_ENABLE_PUT_SELF",
                                "COMEX_ENABLE_PUT_SMP", "COMEX_ENABLE_GET_SELF", "COMEX_ENABLE_GET_SMP",
                                "COMEX_ENABLE_ACC_PACKED", "COMEX_ENABLE_PUT_PACKED", "COMEX_ENABLE_GET_PACKED",
                                "COMEX_ENABLE_ACC_IOV", "COMEX_ENABLE_PUT_IOV", "COMEX_ENABLE_GET_IOV")}
    toggles["TEST_EXPECT_TOGGLES"] = "1"
    outs = launch("remote", n=n, timeout=180, extra_env=toggles)
    assert "toggle routes" in outs[0], outs[0][-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("n,one_pass", [(2, "1"), (4, "1"), (3, "0")])
def test_one_pass_same_gpu_exchange(n, one_pass):
    """Ranks sharing this GPU accumulate from plain device buffers into every
    rank's block (their own included), blocking and non-blocking, concurrently:
    the one-pass route under the owners' memory locks must lose no update (exact
    integer sums); with COMEX_AMD_ONE_PASS=0 the same program on the packed route."""
    launch("onepass", n=n, timeout=180, extra_env={"COMEX_AMD_ONE_PASS": one_pass})


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 3])
def test_owner_host_source_self_acc_vs_one_pass_peers(n):
    """the owner accumulates into its own block from pageable host
    memory (host-side route, a join instead of sched_pick) while same-GPU peers
    accumulate >= 64 KiB device patches into the same elements on the one-pass route:
    the owner's launch takes its own memory lock as well, so no update is lost."""
    launch("hostself", n=n, timeout=150)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,n,extra", [("remote", 3, {}), ("onepass", 4, {}), ("directsrc", 3, {}),
                                          ("segcache", 3, {"COMEX_AMD_SEGMENT_CACHE_MB": "0"}), ("segcache", 3, {}),
                                          ("stress", 3, {"COMEX_AMD_STAGING_MB": "1"}),
                                          ("c5full", 8, {"COMEX_AMD_STAGING_MB": "256", "TEST_C5_N": "16384"}),
                                          ("c5full", 4, {"COMEX_AMD_PEER_LOADS": "all", "TEST_C5_N": "8192"})])
def test_vmm_segments(mode, n, extra):
    """HBM segments from the virtual-memory allocator
    (COMEX_AMD_SEGMENT_ALLOC=vmm, vmm.cpp) -- hipMemCreate + a dmabuf descriptor
    handed to the peers over a per-process socket (SCM_RIGHTS), keyed by owner rank
    and allocation number -- under the remote suite, the one-pass and
    direct-source routes, create/free cycles, random programs and C5 (one GPU, and
    with every peer treated as another GPU), all exact."""
    launch(mode, n=n, timeout=150, extra_env=dict(extra, COMEX_AMD_SEGMENT_ALLOC="vmm"))


@pytest.mark.gpu
@pytest.mark.parametrize("alloc,finalize,granule", [("ipc", True, None), ("vmm", True, None), ("ipc", False, None),
                                                    ("vmm", False, None), ("ipc", True, 17), ("vmm", True, 17)])
def test_stale_segment_replaced(alloc, finalize, granule):
    """The replacement path for a new segment whose peer mappings read other memory
    (the runtime defect of DESIGN.md section 6), forced on demand
    (gaamd_diag "stale_gen" = 2): the owner sets the block aside, allocates another, the
    exchange repeats, and every accumulate into the segments is exact, on both segment
    allocators; with comex_finalize and without (the exit hook then joins the idle
    progress thread: a process exiting with set-aside blocks once crashed there).
    granule: 64 MiB segments whose owners write a foreign tag into interior granule 17
    (34 MiB in) of the second one -- the whole-block check (k_seg_check, VERDICT r4
    item 4) must find it, not only a mismatch at the block's ends."""
    env = {"TEST_STALE_GEN": "2", "COMEX_AMD_SEGMENT_ALLOC": alloc,
           "STALEFIX_NO_FINALIZE": "0" if finalize else "1"}
    if granule is not None:
        env.update(TEST_STALE_GRANULE=str(granule), TEST_STALE_N=str(1 << 23))
    launch("stalefix", n=3, timeout=120, extra_env=env)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["remote", "hostseg-ga"])
def test_host_segments_three_ranks(mode):
    """COMEX_AMD_SEGMENT=host gives every rank a host segment (a
    POSIX shm object mapped and HIP-registered by every rank of the node, as the
    reference's _shm_create/_shm_attach), so GA's host-side local operations work with
    several ranks per node.  `remote`: the whole remote suite (acc/put/get/accv/getv/
    putv, a chunked remote accumulate) into host segments, exact vs the oracle;
    `hostseg-ga`: host writes through NGA_Access seen by the peers' NGA_Get, remote
    NGA_Acc checked on the host, and pnga_zero's NGA_Access + memset visible to all."""
    launch(mode, n=3, timeout=150, extra_env={"COMEX_AMD_SEGMENT": "host"})


@pytest.mark.gpu
@pytest.mark.parametrize("one_pass", ["1", "0"])
def test_config_c1_one_mib_remote_acc_two_ranks(one_pass):
    """BASELINE config C1: a 1-D contiguous f64 accumulate of 1 MiB from rank 0 to
    rank 1 and back (2 ranks, one GPU), the survey's synthetic data, bit-exact
    against the oracle; host, device and segment sources (packed, one-pass and
    direct-source routes; COMEX_AMD_ONE_PASS=0 sends the device source packed)."""
    launch("c1", n=2, timeout=120, extra_env={"COMEX_AMD_ONE_PASS": one_pass})


@pytest.mark.gpu
def test_config_c5_full_size_eight_ranks_one_gpu():
    """BASELINE config C5 at its stated size: NGA_Acc into a 32768^2 f64 GA on 8 ranks
    sharing this GPU -- M1 (own 1 GiB block) and M2 (every rank the whole 8 GiB
    array), checked exactly with the 2**rank scheme.  The owners
    share the GPU, so EVERY rank's M2 takes the one-pass route (its fused kernel
    writes each owner's block under the owner's memory lock) -- the worker asserts
    one_pass > 0 and no packed or direct-source request for every rank.  The routes
    an 8-GPU node takes are the next test."""
    launch("c5full", n=8, timeout=420, extra_env={"COMEX_AMD_STAGING_MB": "256"})


@pytest.mark.gpu
def test_config_c5_full_size_eight_ranks_cross_device_routes():
    """C5 at its stated size on the routes an 8-GPU node takes:
    32768^2 f64 GA, 8 ranks, every other rank's memory treated as another GPU's
    (COMEX_AMD_PEER_LOADS=all).  M2: even ranks accumulate the whole 8 GiB array from
    a plain device buffer -- the packed route: pack -> staging -> the owner pulls
    the chunk with system-scope loads on a pull stream of that source; odd ranks from
    their own segment -- the direct-source route: the owner's kernel reads the source
    in place with system-scope loads.  The worker asserts the route counts (packed
    only on even ranks, direct_src only on odd ones, no one-pass) and checks every
    element of every block exactly (2**8 - 1)."""
    launch("c5full", n=8, timeout=420, extra_env={"COMEX_AMD_STAGING_MB": "256", "COMEX_AMD_PEER_LOADS": "all"})


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2])
def test_direct_ops_on_self_after_packed_self_traffic(n):
    """COMEX_ENABLE_{ACC,PUT}_{SELF,SMP}=0: a put and an accumulate to this rank take
    the packed route; a get, an io-vector get and an rmw on the same bytes issued
    right after (no barrier, no fence) see them applied (the
    reference flushes first, comex.c:6073-6080, 6228-6235).  With ACC_SMP=0 a
    >= 1 MiB same-node accumulate from a segment takes the packed route too."""
    toggles = {"COMEX_ENABLE_ACC_SELF": "0", "COMEX_ENABLE_ACC_SMP": "0", "COMEX_ENABLE_PUT_SELF": "0",
               "COMEX_ENABLE_PUT_SMP": "0", "COMEX_AMD_STAGING_MB": "64"}
    launch("selforder", n=n, timeout=150, extra_env=toggles)


@pytest.mark.gpu
@pytest.mark.parametrize("n,one_pass", [(2, "0"), (3, "0"), (3, "1")])
def test_direct_source_remote_accumulate(n, one_pass):
    """Source in the caller's segment: the owner accumulates straight from it
    (no pack, no staging), bit-exact against the oracle; smaller patches keep
    the packed route.  An owner on the caller's GPU takes the
    one-pass route instead unless COMEX_AMD_ONE_PASS=0 (the ranks of this test
    share one GPU; with the route off they exercise the direct-source route, as
    owners on other GPUs do)."""
    launch("directsrc", n=n, timeout=120, extra_env={"COMEX_AMD_ONE_PASS": one_pass})


@pytest.mark.gpu
def test_bench_two_ranks_exchange_exact():
    """The driver's N > 1 invocation shape (bench.py --gpus 2 spawning its own ranks)
    ends with the C5 exchange check: every element of a 4096^2 GA accumulated by
    both ranks from constant sources must be exact on the packed and the
    direct-source route, and rank 0 prints one JSON line."""
    import json
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1",
                        "--warmup-ms", "0", "--no-cpu", "--ga-dims", "8192", "--c5-steps", "2"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    chk = line["c5"]["exchange_check"]
    assert chk["buffer_src"]["result"] == "exact" and chk["segment_src"]["result"] == "exact", chk
    assert chk["buffer_src"]["array"] == "8192x8192 f64", chk   # at --ga-dims, not a fixed 4096


@pytest.mark.gpu
def test_bench_extras_watchdog_keeps_headline():
    """If the N > 1 extras (the cross-GPU exchange) do not finish in time, rank 0
    still prints the headline line -- measured before the extras -- exactly once,
    with the extras marked as timed out, and the job ends with bench.py's
    EXTRAS_TIMEOUT_STATUS (3): a hang is a failure the caller sees."""
    import json
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1",
                        "--warmup-ms", "0", "--no-cpu", "--ga-dims", "8192", "--c5-steps", "2",
                        "--extras-timeout", "0.05"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 3 and len(lines) == 1, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert "timed_out" in line["c5"], line["c5"]


@pytest.mark.gpu
@pytest.mark.parametrize("n,cache", [(2, "16384"), (3, "16384"), (3, "0")])
def test_segment_cache_reuse(n, cache):
    """Freed segments are kept with their IPC export and serve the next comex_malloc of
    their size; remote accumulates into reused segments stay exact (and with the cache
    off, every segment is a fresh block)."""
    launch("segcache", n=n, timeout=120, extra_env={"COMEX_AMD_SEGMENT_CACHE_MB": cache})


@pytest.mark.gpu
@pytest.mark.parametrize("n,peer", [(2, "all"), (3, "all"), (2, "auto")])
def test_xdev_self_check(n, peer):
    """the self-check bench.py's N > 1 extras open with -- remote
    strided acc (every type) / put / get with random descriptors, accv / putv / getv,
    rmw, between rank pairs -- exact by closed form on one MI355X; with every peer
    treated as another GPU (PEER_LOADS=all) the packed, direct-source and system-scope
    get routes all ran (route counters summed over the ranks)."""
    outs = launch("xcheck", n=n, timeout=200, extra_env={"COMEX_AMD_PEER_LOADS": peer})
    assert any(l.startswith("XCHECK ") for l in outs[0].splitlines())


@pytest.mark.gpu
def test_xdev_self_check_classifies_a_dropped_chunk():
    """the owners drop every 7th packed chunk (gaamd_diag
    "drop_chunk"); the check reads MISMATCH, reruns in the same processes under the
    conservative publication mode, reads MISMATCH again and says "persists: logic"."""
    launch("xcheck", n=2, timeout=200, extra_env={"COMEX_AMD_PEER_LOADS": "all", "XCHECK_DROP": "7"})


@pytest.mark.gpu
@pytest.mark.parametrize("alloc", ["ipc", "vmm"])
def test_odd_size_segments(alloc):
    """segments of 2 MiB + 9..15 bytes and sizes that are not multiples of 8
    map on every peer without a replacement (granule tags kept clear of the end tag, the
    end tag on an aligned word), on both allocators."""
    launch("oddseg", n=2, timeout=120, extra_env={"COMEX_AMD_SEGMENT_ALLOC": alloc})


@pytest.mark.gpu
def test_vmm_window_used_up_is_a_clear_error():
    """the vmm allocator maps every block at a range never used before;
    when its private window [COMEX_AMD_VMM_VA_BASE, COMEX_AMD_VMM_VA_LIMIT) is used up
    the next comex_malloc aborts with a message naming the variables -- not a
    runtime-chosen range that may be one handed back earlier.  A 1 GiB window and
    64 MiB segments with the freed-block cache off: the first ~15 cycles run, then
    the error, well within the timeout."""
    code = ("import ctypes, ga_amd\n"
            "L = ga_amd.lib()\n"
            "out = (ctypes.c_ulonglong * 2)()\n"
            "assert ga_amd.comex_init() == 0\n"
            "for i in range(64):\n"
            "    seg = ga_amd.comex_malloc(64 << 20, 1)\n"
            "    assert ga_amd.comex_free(seg[0]) == 0\n"
            "    assert L.gaamd_diag(b'vmm_window', 0, out, 2) == 0\n"
            "    assert out[0] == (i + 1) * (66 << 20), (i, out[0])   # 64 MiB + the 2 MiB guard each\n"
            "    assert out[0] + out[1] == 1 << 30, (out[0], out[1])\n"
            "    print('cycle', i, 'window used', out[0], 'left', out[1], flush=True)\n"
            "print('no error after 64 cycles', flush=True)\n")
    env = dict(os.environ, COMEX_AMD_SEGMENT_ALLOC="vmm", COMEX_AMD_SEGMENT_CACHE_MB="0",
               COMEX_AMD_VMM_VA_BASE=hex(0x200000000000), COMEX_AMD_VMM_VA_LIMIT=hex(0x200000000000 + (1 << 30)))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0, r.stdout
    assert "private address window is used up" in r.stderr and "COMEX_AMD_VMM_VA_LIMIT" in r.stderr, r.stderr[-2000:]
    # the counter: 1 GiB // 66 MiB = 15 cycles ran, the 16th found the window used up
    cycles = [l for l in r.stdout.splitlines() if l.startswith("cycle ")]
    assert len(cycles) == (1 << 30) // (66 << 20), r.stdout[-2000:]
