#!/bin/bash
# round-2 GPU session ad: flakiness check -- the multi-process GPU tests three times
set -uo pipefail
O=gpurun_out/r02ad
mkdir -p "$O"
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 500 python -u -m pytest tests/test_multiproc.py tests/test_gpu_semantics.py -q --timeout 150 --timeout-method thread -p no:cacheprovider -rf -m gpu > "$O/mp_$i.out" 2> "$O/mp_$i.err"
  rc=$?
  echo "mp_$i rc=$rc $(tail -1 $O/mp_$i.out)"
  grep "^FAILED" "$O/mp_$i.out" | head
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
echo done
