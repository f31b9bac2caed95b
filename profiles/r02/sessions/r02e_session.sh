#!/bin/bash
# round-2 GPU session e: ARMCI surface test again; isolate the 2-rank hang of
# session d (GA M2 with the source in a segment), with progress lines
set -uo pipefail
O=gpurun_out/r02e
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step misc 300 python -u -m pytest tests/test_multiproc.py -v -k "armci_message" --timeout 150 --timeout-method thread -p no:cacheprovider -rf
tail -8 "$O/misc.out"
step c5m2 150 python3 -u bench.py --gpus 2 --workload C5 --exchange --ga-dims 8192 --steps 4 --warmup 2 --no-cpu --verbose
tail -2 "$O/c5m2.out"
step c5m2seg 150 python3 -u bench.py --gpus 2 --workload C5 --exchange --src-seg --ga-dims 8192 --steps 4 --warmup 2 --no-cpu --verbose
tail -2 "$O/c5m2seg.out"
step spawn2 300 python3 -u bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --ga-dims 16384 --c5-steps 4 --verbose
cat "$O/spawn2.out"
echo done
