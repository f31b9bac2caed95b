#!/bin/bash
# round-2 GPU session b: timed-region edge probe (host wait modes), the flaky
# 2-rank vector test repeated (default / one library stream), new semantics tests
set -uo pipefail
O=gpurun_out/r02b
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step sem 300 python -u -m pytest tests/test_gpu_semantics.py -q --timeout 120 --timeout-method thread -p no:cacheprovider -rA
tail -3 "$O/sem.out"
step edge_default 120 python3 tools/edge_probe.py
step edge_spin 120 env COMEX_AMD_WAIT=spin python3 tools/edge_probe.py
step edge_yield 120 env COMEX_AMD_WAIT=yield python3 tools/edge_probe.py
step edge_blocking 120 env COMEX_AMD_WAIT=blocking python3 tools/edge_probe.py
for i in 1 2 3 4; do
  step vec_$i 200 python -u -m pytest tests/test_multiproc.py -q -k "test_comex_test_vector_restated" --timeout 150 --timeout-method thread -p no:cacheprovider
done
for i in 1 2 3; do
  step vec1s_$i 200 env COMEX_AMD_STREAMS=1 python -u -m pytest tests/test_multiproc.py -q -k "test_comex_test_vector_restated" --timeout 150 --timeout-method thread -p no:cacheprovider
done
step order 200 python -u -m pytest tests/test_multiproc.py -q -k "put_then_acc" --timeout 150 --timeout-method thread -p no:cacheprovider
step bench_drv 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
step bench_drv_b 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
echo done
