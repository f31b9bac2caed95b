#!/bin/bash
# round-2 GPU session t: the vector-acc lost request -- rank 0 not accumulating into
# itself (only progress-thread kernels touch the array), and an all-XCD acquire kernel
# before each progress-thread launch
set -uo pipefail
O=gpurun_out/r02t
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$name rc=$rc"; exit $rc; fi
    echo "$name rc=$rc $(grep -ho '[0-9]* passed\|[0-9]* failed' "$O/$name.out" | tr '\n' ' ') $(grep -ho 'diff/(alpha\*a) [-+0-9.]*' "$O/$name.out" | head -1)"
}
for v in skiplocal acqk skiplocal_s1; do
  case $v in
    skiplocal) E="TEST_VEC_SKIP_LOCAL=1";;
    acqk) E="COMEX_AMD_DIAG_OWNER_PRESYNC=3";;
    skiplocal_s1) E="TEST_VEC_SKIP_LOCAL=1 COMEX_AMD_STREAMS=1";;
  esac
  for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
    step ${v}_$i 150 env $E TEST_VEC_RANK_ALPHA=1 python -u -m pytest tests/test_multiproc.py -q -x -k "test_comex_test_vector_restated and not 1" --timeout 120 --timeout-method thread -p no:cacheprovider
  done
done
echo done
