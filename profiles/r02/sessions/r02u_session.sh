#!/bin/bash
# round-2 GPU session u: the vector-acc lost request, traced in the owner's kernel
# (source read vs staging, destination read vs the last value written there)
set -uo pipefail
O=gpurun_out/r02u
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$name rc=$rc"; exit $rc; fi
    echo "$name rc=$rc $(grep -ho '[0-9]* passed\|[0-9]* failed' "$O/$name.out" | tr '\n' ' ') $(grep -ho 'diff/(alpha\*a) [-+0-9.]*' "$O/$name.out" | head -1)"
    grep -ho "\[ga_amd [0-9]*\] trace.*\|owner applied.*\|routes {.*" "$O/$name.out" "$O/$name.err" | head -8
}
for v in trace; do
  case $v in
    trace) E="COMEX_AMD_DIAG_TRACE=1 TEST_VEC_SKIP_LOCAL=1";;
    trace_s1) E="COMEX_AMD_DIAG_TRACE=1 TEST_VEC_SKIP_LOCAL=1 COMEX_AMD_STREAMS=1";;
  esac
  for i in $(seq 1 16); do
    step ${v}_$i 150 env $E TEST_VEC_RANK_ALPHA=1 python -u -m pytest tests/test_multiproc.py -q -x -k "test_comex_test_vector_restated and not 1" --timeout 120 --timeout-method thread -p no:cacheprovider -s
  done
done
echo done
