#!/bin/bash
# round-2 GPU session k: per-shape bench lines (2 streams) and rocprofv3 kernel
# summaries (1 stream, so AverageNs is the per-launch time) for H8200, C2, C3, C4;
# strided put/get at H; the packed route to self
set -uo pipefail
O=gpurun_out/r02k
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
for W in H8200 C2 C3 C4; do
  step bench_$W 120 python3 bench.py --workload $W --steps 100 --warmup 5 --no-cpu
  step prof_$W 150 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof_$W" -o run -- python3 bench.py --workload $W --steps 100 --warmup 5 --no-cpu --streams 1
done
for X in put get; do
  step bench_$X 120 python3 bench.py --xfer $X --steps 100 --warmup 5 --no-cpu
done
step selfpacked 120 python3 bench.py --self-packed --steps 100 --warmup 5 --no-cpu
step prof_selfpacked 150 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof_selfpacked" -o run -- python3 bench.py --self-packed --steps 100 --warmup 5 --no-cpu
echo done
