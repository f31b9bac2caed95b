#!/bin/bash
# round-2 GPU session ab: packed-route chunking -- COMEX_AMD_RING_CHUNKS 1/2/4/8 on the
# packed route to self (N=1), the 2-rank exchange and C5 M2 (2 ranks, one GPU)
set -uo pipefail
O=gpurun_out/r02ab
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$O/$name.err"; exit $rc; fi
}
for rep in 1 2; do
for c in 1 2 4 8; do
  step self_${c}_$rep 120 env COMEX_AMD_RING_CHUNKS=$c python3 bench.py --self-packed --steps 50 --warmup 5 --no-cpu
  step ex2_${c}_$rep 150 env COMEX_AMD_RING_CHUNKS=$c python3 bench.py --gpus 2 --exchange --steps 30 --warmup 5 --no-cpu --no-extras
done
done
for c in 1 4; do
  step c5_${c} 300 env COMEX_AMD_RING_CHUNKS=$c python3 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu --ga-dims 16384 --c5-steps 4
done
for f in "$O"/self_*.out "$O"/ex2_*.out; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
for f in "$O"/c5_*.out; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["c5"]; print(c["M2"]["ms_per_step"], c["M2_src_in_segment"]["ms_per_step"], c["exchange_check"]["packed"]["result"])')"; done
echo done
