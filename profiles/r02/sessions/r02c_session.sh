#!/bin/bash
# round-2 GPU session c: the new ARMCI surface test, the whole GPU suite, the
# driver's bench invocation (event-free value region) and its rocprof summary
set -uo pipefail
O=gpurun_out/r02c
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step misc 400 python -u -m pytest tests/test_multiproc.py -v -k "armci_message" --timeout 150 --timeout-method thread -p no:cacheprovider
tail -8 "$O/misc.out"
step suite 1000 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider -rf
tail -12 "$O/suite.out"
step bench_drv 180 python3 bench.py --gpus 1 --steps 20 --warmup 5
cat "$O/bench_drv.out"
step bench_drv_b 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
cat "$O/bench_drv_b.out"
step prof 240 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
echo done
