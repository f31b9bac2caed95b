#!/bin/bash
# round-2 GPU session ak: end-of-region sync order -- library streams in index order
# (default) vs the stream of the latest launch first (COMEX_AMD_SYNC_ORDER=1)
set -uo pipefail
O=gpurun_out/r02ak2
mkdir -p "$O"
export TMPDIR=/tmp
for i in 1 2 3 4 5 6 7; do
  for v in 0 1; do
    timeout -k 10 150 env COMEX_AMD_SYNC_ORDER=$v python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > "$O/b_${v}_$i.out" 2> "$O/b_${v}_$i.err" || exit 1
    echo "order=$v run=$i $(grep '^{' $O/b_${v}_$i.out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], round(d["value"]*2**30/8e12,4), d["roofline"]["frac"], d["value_region"]["total_us"])')"
  done
done
echo done
