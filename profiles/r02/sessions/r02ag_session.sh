#!/bin/bash
# round-2 GPU session ag: round-end check on the current tree -- smoke, GPU suite,
# the driver's invocation, a 2-rank self-spawned line with the C5 extras
set -uo pipefail
O=gpurun_out/r02ag
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$O/$name.err"; tail -5 "$O/$name.out"; exit $rc; fi
}
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
tail -2 "$O/smoke.out"
step suite 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider -rf
tail -2 "$O/suite.out"
step bench 180 python3 bench.py --gpus 1 --steps 20 --warmup 5
step spawn2 300 python3 -u bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --ga-dims 16384 --c5-steps 4
for f in bench spawn2; do grep '^{' "$O/$f.out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], round(d['value']*2**30/8e12/d['n_gpus'],4), d['roofline']['frac'], (d.get('c5') or {}).get('exchange_check'))"; done
echo done
