#!/usr/bin/env python3
"""Two ranks on one GPU: comex_malloc of growing sizes (diagnosing a hang seen
in the C5 M2 source segment of 2 GiB).  Self-spawns when RANK is unset."""
import faulthandler
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    if "RANK" not in os.environ:
        import socket
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = str(s.getsockname()[1])
        s.close()
        procs = [subprocess.Popen([sys.executable, "-u", __file__] + sys.argv[1:],
                                  env=dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                                           MASTER_ADDR="127.0.0.1", MASTER_PORT=port, COMEX_AMD_JOBID="m" + port))
                 for r in range(2)]
        sys.exit(max(p.wait() for p in procs))
    faulthandler.dump_traceback_later(int(os.environ.get("REPRO_DUMP_S", "50")), exit=True)
    if os.environ.get("REPRO_TORCH") == "1":   # torch's own HIP runtime loaded first, as in bench.py N>1
        import torch  # noqa: F401
        import torch.distributed  # noqa: F401
    import ga_amd
    rank = int(os.environ["RANK"])
    assert ga_amd.comex_init() == 0
    keep = os.environ.get("REPRO_KEEP") == "1"     # keep every segment live (no free between sizes)
    live = []
    for gib in [float(x) for x in (sys.argv[1:] or ["1", "2", "3"])]:
        n = int(gib * (1 << 30))
        print(f"rank {rank}: malloc {gib} GiB", file=sys.stderr, flush=True)
        seg = ga_amd.comex_malloc(n, 2)
        print(f"rank {rank}: malloc {gib} GiB ok", file=sys.stderr, flush=True)
        ga_amd.comex_barrier()
        if keep:
            live.append(seg)
        else:
            assert ga_amd.comex_free(seg[rank]) == 0
    for seg in live:
        assert ga_amd.comex_free(seg[rank]) == 0
    ga_amd.comex_finalize()
    print(f"rank {rank}: OK", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
