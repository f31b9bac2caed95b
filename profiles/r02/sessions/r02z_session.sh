#!/bin/bash
# round-2 GPU session z: evidence on the current tree -- GPU suite, the driver's
# invocation three times, rocprofv3 of it (1 and 2 streams), PMC HBM traffic of H
set -uo pipefail
O=gpurun_out/r02z
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$O/$name.err"; tail -5 "$O/$name.out"; exit $rc; fi
}
step suite 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider -rf
tail -3 "$O/suite.out"
step bench1 180 python3 bench.py --gpus 1 --steps 20 --warmup 5
step bench2 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
step bench3 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
for f in "$O"/bench*.out; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], round(d["value"]*2**30/8e12,4), d["roofline"]["frac"], d["value_region"]["total_us"])')"; done
step prof2 200 rocprofv3 --kernel-trace --stats -d "$O/prof2" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
step prof1 200 rocprofv3 --kernel-trace --stats -d "$O/prof1" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --streams 1
step pmc 300 python3 tools/pmc_traffic.py --workload H --tag r02 --outdir "$O/pmc"
cat "$O/pmc.out"
echo done
