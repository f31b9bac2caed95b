#!/bin/bash
# round-2 GPU session n: which rank's contribution the vector-acc miss loses,
# and whether it arrives late (completion reported early) or never (lost update)
set -uo pipefail
O=gpurun_out/r02n
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
for i in 1 2 3 4 5 6 7 8; do
  step vec_$i 150 env TEST_VEC_RANK_ALPHA=1 COMEX_AMD_STREAMS=1 COMEX_AMD_CHECK_IOV=1 python -u -m pytest tests/test_multiproc.py -q -x -k "test_comex_test_vector_restated and not 1" --timeout 120 --timeout-method thread -p no:cacheprovider
  grep -o "test_vector_acc: .*\|staging bytes differ.*" "$O/vec_$i.out" | head -4 | cut -c1-300
done
echo done
