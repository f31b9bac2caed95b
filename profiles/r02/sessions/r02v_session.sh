#!/bin/bash
# round-2 GPU session v: the inbox fix -- the vector-acc test repeated, then the
# multi-process suite
set -uo pipefail
O=gpurun_out/r02v
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$name rc=$rc"; exit $rc; fi
    echo "$name rc=$rc $(grep -ho '[0-9]* passed\|[0-9]* failed' "$O/$name.out" | tr '\n' ' ') $(grep -ho 'diff/(alpha\*a) [-+0-9.]*\|owner applied.*\|AssertionError: {.*' "$O/$name.out" | head -2)"
}
for i in $(seq 1 20); do
  step vec_$i 150 python -u -m pytest tests/test_multiproc.py -q -x -k "test_comex_test_vector_restated" --timeout 120 --timeout-method thread -p no:cacheprovider
done
step mp 600 python -u -m pytest tests/test_multiproc.py -q --timeout 150 --timeout-method thread -p no:cacheprovider -rf -m gpu
tail -5 "$O/mp.out"
echo done
