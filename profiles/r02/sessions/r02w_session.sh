#!/bin/bash
# round-2 GPU session w: whole GPU suite, the driver's bench invocation, the
# 2-rank rehearsal with C5 extras, rocprof summaries (1 and 2 streams)
set -uo pipefail
O=gpurun_out/r02w
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step suite 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider -rf
tail -12 "$O/suite.out"
step bench_drv 180 python3 bench.py --gpus 1 --steps 20 --warmup 5
tail -c 400 "$O/bench_drv.out"
step bench_drv2 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
tail -c 600 "$O/bench_drv2.out"
step spawn2 300 env BENCH_STACK_DUMP_S=240 python3 -u bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --ga-dims 16384 --c5-steps 4 --verbose
cat "$O/spawn2.out"
step prof2 200 rocprofv3 --kernel-trace --stats -d "$O/prof2" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
step prof1 200 rocprofv3 --kernel-trace --stats -d "$O/prof1" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --streams 1
echo done
