#!/bin/bash
# round-2 GPU session aa: where the value region's host edges go -- profiled runs of the
# driver's invocation with the region's boottime stamps, host waits polling (default)
# vs the runtime's synchronize (COMEX_AMD_HOST_WAIT=hip); then unprofiled A/B
set -uo pipefail
O=gpurun_out/r02aa
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$O/$name.err"; exit $rc; fi
}
step prof_poll 200 rocprofv3 --kernel-trace -d "$O/prof_poll" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
export COMEX_AMD_HOST_WAIT=hip
step prof_hip 200 rocprofv3 --kernel-trace -d "$O/prof_hip" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
unset COMEX_AMD_HOST_WAIT
for i in 1 2 3; do
  step bench_poll_$i 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
  step bench_hip_$i 180 env COMEX_AMD_HOST_WAIT=hip python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
done
for f in "$O"/bench_*.out; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], round(d["value"]*2**30/8e12,4), d["roofline"]["frac"], d["value_region"]["total_us"], d["value_region"]["first_call_us"])')"; done
echo done
