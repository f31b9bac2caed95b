#!/bin/bash
# round-2 GPU session d: ARMCI surface, COMEX_ENABLE toggles, direct-source
# route; value-region spread; packed route on one rank; 2-rank exchange with and
# without the source in a segment
set -uo pipefail
O=gpurun_out/r02d
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step mp 600 python -u -m pytest tests/test_multiproc.py tests/test_legacy_acc.py -v -k "armci_message or packed_route or direct_source or gpu_legacy" --timeout 150 --timeout-method thread -p no:cacheprovider -rf
tail -15 "$O/mp.out"
step diag 180 env BENCH_DIAG_REGIONS=12 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
cat "$O/diag.out"
step selfpacked 180 python3 bench.py --gpus 1 --steps 50 --warmup 5 --no-cpu --self-packed
cat "$O/selfpacked.out"
step ex2 240 python3 bench.py --gpus 2 --exchange --steps 20 --warmup 5 --no-cpu --no-extras
cat "$O/ex2.out"
step ex2seg 240 python3 bench.py --gpus 2 --exchange --src-seg --steps 20 --warmup 5 --no-cpu --no-extras
cat "$O/ex2seg.out"
step spawn2 400 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --ga-dims 16384 --c5-steps 4
cat "$O/spawn2.out"
echo done
