#!/bin/bash
# round-2 GPU session aq: stress campaign, longer programs, 1/2/4 library streams
set -uo pipefail
O=gpurun_out/r02aq
mkdir -p "$O"
export TMPDIR=/tmp
for streams in 2 1 4; do
for seed in 11 12 13 14 15; do
  timeout -k 10 400 env COMEX_AMD_STREAMS=$streams STRESS_SEED=$seed STRESS_OPS=3000 python -u -m pytest tests/test_multiproc.py -q -k "test_stress_random_programs" --timeout 300 --timeout-method thread -p no:cacheprovider -rf > "$O/s_${streams}_$seed.out" 2> "$O/s_${streams}_$seed.err"
  rc=$?
  echo "streams=$streams seed=$seed rc=$rc $(tail -1 $O/s_${streams}_$seed.out)"
  grep -h "^FAILED\|differ\|Error" "$O/s_${streams}_$seed.out" | head -4 | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
done
echo done
