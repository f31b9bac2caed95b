#!/bin/bash
# round-2 GPU session s: the vector-acc lost request -- owner syncs before its launch
# (stream / device), system-scope acquire in the owner's kernel, requester waits for
# each request's completion
set -uo pipefail
O=gpurun_out/r02s
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$name rc=$rc"; exit $rc; fi
    echo "$name rc=$rc $(grep -ho '[0-9]* passed\|[0-9]* failed' "$O/$name.out" | tr '\n' ' ') $(grep -ho 'diff/(alpha\*a) [-+0-9.]*' "$O/$name.out" | head -1)"
}
for v in base presync devsync sysacq reqwait; do
  case $v in
    base) E="X=1";;
    presync) E="COMEX_AMD_DIAG_OWNER_PRESYNC=1";;
    devsync) E="COMEX_AMD_DIAG_OWNER_PRESYNC=2";;
    sysacq) E="COMEX_AMD_DIAG_OWNER_SYSACQ=1";;
    reqwait) E="COMEX_AMD_DIAG_REQ_WAIT=1";;
  esac
  for i in 1 2 3 4 5 6 7 8 9 10; do
    step ${v}_$i 150 env $E TEST_VEC_RANK_ALPHA=1 python -u -m pytest tests/test_multiproc.py -q -x -k "test_comex_test_vector_restated and not 1" --timeout 120 --timeout-method thread -p no:cacheprovider
  done
done
echo done
