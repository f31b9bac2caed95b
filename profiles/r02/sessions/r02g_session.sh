#!/bin/bash
set -uo pipefail
O=gpurun_out/r02g
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step repro 70 env COMEX_AMD_DEBUG=2 python3 -u tools/malloc_repro.py 1 2 3
grep -v "amdgpu.ids" "$O/repro.err" | tail -30
step m2seg16 90 env BENCH_STACK_DUMP_S=60 COMEX_AMD_DEBUG=2 python3 -u bench.py --gpus 2 --workload C5 --exchange --src-seg --ga-dims 16384 --steps 2 --warmup 1 --warmup-ms 0 --no-cpu --verbose
grep "comex_malloc\|rank" "$O/m2seg16.err" | grep -v "acc ->\|put ->\|get ->" | tail -30
echo done
