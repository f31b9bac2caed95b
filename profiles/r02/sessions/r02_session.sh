#!/bin/bash
# tools/r02_session.sh -- round-2 GPU check: the parity suite, then the driver's
# bench invocation (and A/B variants of the timing), then rocprofv3 summaries.
# Each GPU step has its own time limit; a crash/timeout ends the script.  A plain
# test failure (pytest rc 1) does not stop the measurements.
set -uo pipefail
O=gpurun_out/r02
mkdir -p "$O"
export TMPDIR=/tmp
step() {   # step NAME TIMEOUT CMD...: run, record rc, stop on anything but 0/1
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step gpu_tests 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rA
tail -5 "$O/gpu_tests.out"
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step bench_drv1 180 python3 bench.py --gpus 1 --steps 20 --warmup 5
step bench_drv2 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
step bench_drv_nowarm 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --warmup-ms 0 --no-cpu
step bench_drv_blocking 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --api blocking --no-cpu
COMEX_AMD_BLOCKING_SYNC=0 step bench_drv_oldapi 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --api blocking --no-cpu
step bench_drv_1stream 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --tune streams=1
step bench_300 120 python3 bench.py --steps 300 --no-cpu
step bench_2000 120 python3 bench.py --steps 2000 --no-cpu
step bench_2000b 120 python3 bench.py --steps 2000 --no-cpu
step spawn2 240 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --ga-dims 16384
step prof1 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof1" -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --tune streams=1
step prof2 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof2" -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
echo done
