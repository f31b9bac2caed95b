#!/bin/bash
# round-2 GPU session ak: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG)
# (default) vs the stream of the latest launch first (COMEX_AMD_STREAM_PRIORITY=1)
set -uo pipefail
O=gpurun_out/r02at
mkdir -p "$O"
export TMPDIR=/tmp
for i in 1 2 3 4 5 6 7; do
  for v in 0 1; do
    timeout -k 10 150 env HIP_FORCE_DEV_KERNARG=$v python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > "$O/b_${v}_$i.out" 2> "$O/b_${v}_$i.err" || exit 1
    echo "devkernarg=$v run=$i $(grep '^{' $O/b_${v}_$i.out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], round(d["value"]*2**30/8e12,4), d["roofline"]["frac"], d["value_region"]["total_us"])')"
  done
done
echo done
