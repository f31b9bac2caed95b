#!/bin/bash
# round-2 GPU session o: bisect the vector-acc lost update -- delays on either side
set -uo pipefail
O=gpurun_out/r02o
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
for v in base osync lsync; do
  for i in 1 2 3 4 5 6 7 8; do
    case $v in
      base) E="";;
      osync) E="COMEX_AMD_DIAG_OWNER_SYNC=1";;
      lsync) E="COMEX_AMD_PROGRESS_SPIN_US=0";;
    esac
    step ${v}_$i 150 env $E TEST_VEC_RANK_ALPHA=1 COMEX_AMD_STREAMS=1 python -u -m pytest tests/test_multiproc.py -q -x -k "test_comex_test_vector_restated and not 1" --timeout 120 --timeout-method thread -p no:cacheprovider
    grep -o "test_vector_acc: [0-9]* elements off: \[[0-9]*\] got [^)]*) want [^)]*) (diff/(alpha\*a) [-+0-9.]*" "$O/${v}_$i.out" | head -1
  done
done
echo done
