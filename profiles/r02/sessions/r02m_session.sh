#!/bin/bash
# round-2 GPU session m: the intermittent test_vector_acc miss (last element of a
# descriptor off by one contribution) -- default vs one library stream
set -uo pipefail
O=gpurun_out/r02m
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
for i in 1 2 3 4 5 6; do
  step vec_$i 120 python -u -m pytest tests/test_multiproc.py -q -k "test_comex_test_vector_restated" --timeout 100 --timeout-method thread -p no:cacheprovider
  grep "elements off\|passed\|failed" "$O/vec_$i.out" | tail -3
done
for i in 1 2 3 4 5 6; do
  step vec1s_$i 120 env COMEX_AMD_STREAMS=1 python -u -m pytest tests/test_multiproc.py -q -k "test_comex_test_vector_restated" --timeout 100 --timeout-method thread -p no:cacheprovider
  grep "elements off\|passed\|failed" "$O/vec1s_$i.out" | tail -3
done
echo done
