#!/bin/bash
# round-2 GPU session r: the vector-acc lost request -- one library stream, old
# progress back-off, owner-side delay, requester-side delay, owner sync
set -uo pipefail
O=gpurun_out/r02r
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$name rc=$rc"; exit $rc; fi
    echo "$name rc=$rc $(grep -ho '[0-9]* passed\|[0-9]* failed' "$O/$name.out" | tr '\n' ' ') $(grep -ho 'diff/(alpha\*a) [-+0-9.]*' "$O/$name.out" | head -1)"
}
for v in base s1 spin0 odelay rdelay osync; do
  case $v in
    base) E="X=1";;
    s1) E="COMEX_AMD_STREAMS=1";;
    spin0) E="COMEX_AMD_PROGRESS_SPIN_US=0";;
    odelay) E="COMEX_AMD_DIAG_OWNER_DELAY_US=100";;
    rdelay) E="COMEX_AMD_DIAG_REQ_DELAY_US=100";;
    osync) E="COMEX_AMD_DIAG_OWNER_SYNC=1";;
  esac
  for i in 1 2 3 4 5 6 7 8; do
    step ${v}_$i 150 env $E TEST_VEC_RANK_ALPHA=1 python -u -m pytest tests/test_multiproc.py -q -x -k "test_comex_test_vector_restated and not 1" --timeout 120 --timeout-method thread -p no:cacheprovider
  done
done
echo done
