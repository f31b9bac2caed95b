#!/usr/bin/env python3
"""One parametrised runner for the GPU evidence sessions (it replaces
the 57 one-off scripts rounds 4-6 kept under tools/sessions/, which stay in git history
up to commit 22cce4d).

    python3 tools/session.py RECIPE[,RECIPE...] [--tag DIR] [--list]

Each recipe is a list of steps; every step runs under its own `timeout -k 10 S` with its
stdout (and stderr) in gpurun_out/<tag>/<step>.<ext>, and the first step that fails ends
the session with status 10 + its index (a GPU step after a fault, abort or time limit is
never started: the gpurun rules).  Run on the GPU box as

    gpurun --timeout 1100 -- 'python3 tools/session.py final --tag r06final'

and copy what the judge should read from gpurun_out/<tag>/ to profiles/r0N/<tag>/.
"""
import argparse
import os
import subprocess
import sys
import time

PYTEST = "python3 -u -m pytest -x -v --timeout {t} --timeout-method thread -p no:cacheprovider"
DRIVER = "python3 bench.py --gpus 1 --steps 20 --warmup 5"


def _n_proxy(n, port):
    # the driver's N > 1 shape on this box's one GPU, every peer treated as another GPU
    return (f"env COMEX_AMD_PEER_LOADS=all python3 -m torch.distributed.run --nnodes=1 --nproc-per-node {n} "
            f"--master-addr 127.0.0.1 --master-port {port} bench.py --gpus {n} --steps 20 --warmup 5 --no-cpu")


# name -> [(step, timeout s, command, output extension)]
RECIPES = {
    "suite": [("gpu_suite", 900, PYTEST.format(t=240) + " -m gpu tests", "log")],
    "smoke": [("smoke", 180, "python3 -c 'import __graft_entry__ as g; g.smoke()'", "log")],
    "driver": [(f"bench_driver_{i}", 240, DRIVER, "json") for i in (1, 2, 3)],
    "bench": [("bench_H", 300, "python3 bench.py --no-host", "json"),
              ("bench_C5_n1", 300, "python3 bench.py --workload C5 --no-cpu", "json")],
    "configs": [(f"bench_{w}", 240, f"python3 bench.py --workload {w} --no-cpu --no-host", "json")
                for w in ("C2", "C3", "C4", "H8200")],
    "putget": [(f"{x}_H", 200, f"python3 bench.py --xfer {x} --steps 50 --warmup 5 --no-cpu --no-host", "json")
               for x in ("put", "get")],
    "evidence": [("evidence", 900, "bash tools/evidence.sh r06", "log")],
    "iov": [("iov_tests", 300, PYTEST.format(t=120) + " -m gpu tests/test_gpu_parity.py -k 'one_workgroup or partitions_large or accv "
                                                     "or getv or putv'", "log"),
            ("scatter_ab", 240, "python3 tools/scatter_bench.py --pairs 512,1024,2048,4096,8192,16384,32768,65536 "
                                "--steps 50 --ab --nb", "jsonl")],
    "iov_probe": [("probe_random", 300, "./tools/iov_lds_probe", "jsonl"),
                  ("probe_200slots", 300, "./tools/iov_lds_probe 200", "jsonl")],
    "iov_pmc": [("pmc_iov_1Mi", 300, "python3 tools/pmc_iov.py --pairs 1048576 --outdir gpurun_out/{tag}/pmc1mi",
                 "json"),
                ("pmc_iov_64Ki", 300, "python3 tools/pmc_iov.py --pairs 65536 --outdir gpurun_out/{tag}/pmc64ki",
                 "json")],
    "iov_trace": [("iov_trace", 200, "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/{tag}/iovprof "
                                     "-o iov -- python3 tools/scatter_bench.py --pairs 16384 --no-cpu --steps 200",
                   "jsonl")],
    "shape": [("shape_sweep", 240, "python3 tools/shape_sweep.py --rows 32,64,128,256,512,1024,2048,4096,16384",
               "jsonl"),
              ("short_rows_probe", 300, "./tools/short_rows_probe 40", "jsonl")],
    "xcheck": [("xcheck_tests", 600, PYTEST.format(t=220) + " -m gpu tests/test_multiproc.py -k xdev", "log"),
               ("n2_proxy", 400, _n_proxy(2, 29561), "json"),
               ("n8_proxy", 600, _n_proxy(8, 29562), "json")],
    "fuzz": [("fuzz", 600, "env GAAMD_FUZZ_SEED={seed} " + PYTEST.format(t=240) + " -m gpu tests/test_gpu_fuzz.py",
              "log")],
}
RECIPES["final"] = RECIPES["suite"] + RECIPES["smoke"] + RECIPES["driver"] + RECIPES["bench"] + RECIPES["evidence"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("recipes", nargs="?", default="")
    ap.add_argument("--tag", default=None, help="gpurun_out/<tag>/ (default: the recipe names)")
    ap.add_argument("--seed", default="6", help="fuzz: GAAMD_FUZZ_SEED")
    ap.add_argument("--list", action="store_true")
    args = ap.parse_args()
    if args.list or not args.recipes:
        for k, v in RECIPES.items():
            print(f"{k:10s} " + ", ".join(s[0] for s in v))
        return 0
    tag = args.tag or args.recipes.replace(",", "_")
    out = os.path.join("gpurun_out", tag)
    os.makedirs(out, exist_ok=True)
    os.environ.setdefault("TMPDIR", "/tmp")
    steps = [s for r in args.recipes.split(",") for s in RECIPES[r]]
    for k, (name, tmo, cmd, ext) in enumerate(steps):
        cmd = cmd.format(tag=tag, seed=args.seed)
        path = os.path.join(out, f"{name}.{ext}")
        err = path if ext == "log" else os.path.join(out, f"{name}.err")
        t0 = time.time()
        with open(path, "w") as fo, open(err, "a") if err != path else open(os.devnull, "w") as fe:
            rc = subprocess.call(f"timeout -k 10 {tmo} {cmd}", shell=True, stdout=fo,
                                 stderr=(fo if err == path else fe))
        print(f"[session] {name}: rc {rc} in {time.time() - t0:.0f} s -> {path}", flush=True)
        if rc != 0:
            return 10 + k
    return 0


if __name__ == "__main__":
    sys.exit(main())
