#!/bin/bash
# round-2 GPU session y: N = 2 and 3 self-spawned on one GPU with the C5 exchange check
set -uo pipefail
O=gpurun_out/r02y
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$O/$name.err"; exit $rc; fi
}
step spawn2 300 python3 -u bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --ga-dims 16384 --c5-steps 4
step spawn3 300 python3 -u bench.py --gpus 3 --steps 20 --warmup 5 --no-cpu --ga-dims 12288 --c5-steps 2
for f in spawn2 spawn3; do grep '^{' "$O/$f.out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], json.dumps(d['c5']))"; done
echo done
