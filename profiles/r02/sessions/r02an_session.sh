#!/bin/bash
# round-2 GPU session an: refresh of the secondary lines on the final tree -- C5 at N=1,
# host-inclusive rates, GA gemm
set -uo pipefail
O=gpurun_out/r02an
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$O/$name.err"; exit $rc; fi
}
step c5 240 python3 bench.py --workload C5 --steps 10 --warmup 3 --no-cpu
grep '^{' "$O/c5.out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5', d['value'], round(d['value']*2**30/8e12,4), d['roofline']['frac'])"
step host 300 python3 bench.py --steps 10 --warmup 3 --no-cpu --host-rates
grep '^{' "$O/host.out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('host', json.dumps(d.get('host'))[:900])"
echo done
