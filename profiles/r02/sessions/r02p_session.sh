#!/bin/bash
# round-2 GPU session p: the intermittent vector-acc miss -- how often, which rank,
# late or lost, and whether the owner sees the staging bytes the requester uploaded
set -uo pipefail
O=gpurun_out/r02p
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
for i in 1 2 3 4 5 6 7 8 9 10; do
  step vec_$i 150 env TEST_VEC_RANK_ALPHA=1 COMEX_AMD_CHECK_IOV=1 python -u -m pytest tests/test_multiproc.py -q -x -k "test_comex_test_vector_restated and not 1" --timeout 120 --timeout-method thread -p no:cacheprovider
  grep -ho "test_vector_acc: .*\|staging bytes differ.*\|[0-9]* passed.*\|[0-9]* failed.*" "$O/vec_$i.out" "$O/vec_$i.err" | cut -c1-400 | head -6
done
echo done
