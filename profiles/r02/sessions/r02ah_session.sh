#!/bin/bash
# round-2 GPU session ah: the 2-rank self-spawned line with C5 extras, repeated
# (one earlier run: hipIpcGetMemHandle of a segment failed with invalid argument)
set -uo pipefail
O=gpurun_out/r02ah
mkdir -p "$O"
export TMPDIR=/tmp
for i in 1 2 3 4 5 6; do
  timeout -k 10 150 python3 -u bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --ga-dims 16384 --c5-steps 4 > "$O/spawn2_$i.out" 2> "$O/spawn2_$i.err"
  rc=$?
  echo "spawn2_$i rc=$rc"
  grep -h "hipIpcGetMemHandle\|fatal" "$O/spawn2_$i.err" | head -5
  grep '^{' "$O/spawn2_$i.out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['c5']['exchange_check']['packed']['result']), json.dumps(d['c5']['exchange_check']['direct_src']['result']))"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo done
