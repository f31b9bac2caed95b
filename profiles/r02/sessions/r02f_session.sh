#!/bin/bash
# round-2 GPU session f: where do the two intermittent hangs stop (stack dumps)
set -uo pipefail
O=gpurun_out/r02f
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
for i in 1 2 3; do
  step misc2_$i 200 python -u -m pytest tests/test_multiproc.py -v -k "armci_message and 2-None" --timeout 150 --timeout-method thread -p no:cacheprovider -rf
  tail -3 "$O/misc2_$i.out"
done
step spawn2 170 env BENCH_STACK_DUMP_S=120 python3 -u bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --ga-dims 16384 --c5-steps 4 --verbose
cat "$O/spawn2.out"
echo done
