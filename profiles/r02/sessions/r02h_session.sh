#!/bin/bash
set -uo pipefail
O=gpurun_out/r02h
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step k_1_1 70 env REPRO_KEEP=1 python3 -u tools/malloc_repro.py 1 1
grep "rank" "$O/k_1_1.err" | tail -3
step k_05_2 70 env REPRO_KEEP=1 python3 -u tools/malloc_repro.py 0.5 2
grep "rank" "$O/k_05_2.err" | tail -3
step k_1_2 70 env REPRO_KEEP=1 python3 -u tools/malloc_repro.py 1 2
grep "rank" "$O/k_1_2.err" | tail -3
echo done
