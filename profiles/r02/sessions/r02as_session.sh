#!/bin/bash
# round-2 GPU session as: the whole GPU suite with 1 and 4 library streams (scheduler
# robustness beyond the default 2)
set -uo pipefail
O=gpurun_out/r02as
mkdir -p "$O"
export TMPDIR=/tmp
for ns in 4 1; do
  timeout -k 10 600 env COMEX_AMD_STREAMS=$ns python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider -rf > "$O/suite_$ns.out" 2> "$O/suite_$ns.err"
  rc=$?
  echo "streams=$ns rc=$rc $(tail -1 $O/suite_$ns.out)"
  grep "^FAILED" "$O/suite_$ns.out" | head -8 | cut -c1-250
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
echo done
