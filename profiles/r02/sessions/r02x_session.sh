#!/bin/bash
# round-2 GPU session x: the 2-D-grid direct kernel (grid2d) against k_rows2d --
# interleaved sweeps on the 2-D shapes, the driver's invocation A/B/A/B, the
# H-shape stand-alone probe for reference
set -uo pipefail
O=gpurun_out/r02x
mkdir -p "$O"
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$O/$name.err"; exit $rc; fi
}
step sweep_H 200 python3 tools/sweep.py --workload H --steps 40 --rounds 9 --variants "default;grid2d=1;streams=1;grid2d=1,streams=1"
cat "$O/sweep_H.out"
step sweep_C3 200 python3 tools/sweep.py --workload C3 --steps 40 --rounds 7 --variants "default;grid2d=1"
cat "$O/sweep_C3.out"
step sweep_H16k 200 python3 tools/sweep.py --workload H --rows 16384 --steps 20 --rounds 7 --variants "default;grid2d=1"
cat "$O/sweep_H16k.out"
for i in 1 2 3; do
  step bench_def_$i 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
  step bench_g2d_$i 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --tune grid2d=1
done
for f in "$O"/bench_*.out; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], round(d["value"]*2**30/8e12,4), d["roofline"]["frac"], d["value_region"]["total_us"])')"; done
step hprobe 120 ./tools/h_shape_probe
tail -8 "$O/hprobe.out"
echo done
