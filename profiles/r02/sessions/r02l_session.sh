#!/bin/bash
# round-2 GPU session l: progress-thread polling change -- packed route to self,
# 2-rank exchange (packed, direct-source) before/after (COMEX_AMD_PROGRESS_SPIN_US=0
# restores the old back-off), and the multi-process suite
set -uo pipefail
O=gpurun_out/r02l
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
for spin in 2000 0; do
  step selfpacked_$spin 120 env COMEX_AMD_PROGRESS_SPIN_US=$spin python3 bench.py --self-packed --steps 100 --warmup 5 --no-cpu
  step ex2_$spin 150 env COMEX_AMD_PROGRESS_SPIN_US=$spin python3 bench.py --gpus 2 --exchange --steps 50 --warmup 5 --no-cpu --no-extras
  step ex2seg_$spin 150 env COMEX_AMD_PROGRESS_SPIN_US=$spin python3 bench.py --gpus 2 --exchange --src-seg --steps 50 --warmup 5 --no-cpu --no-extras
done
for f in "$O"/*.out; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
step mp 600 python -u -m pytest tests/test_multiproc.py -q --timeout 150 --timeout-method thread -p no:cacheprovider -rf -m gpu
tail -5 "$O/mp.out"
echo done
