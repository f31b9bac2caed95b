#!/bin/bash
# round-2 GPU session ar: rotated chunk order for remote accumulates -- correctness
# (multi-process suite, stress seeds, C5 exchange check) and the 2/3-rank C5 lines
set -uo pipefail
O=gpurun_out/r02ar
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_multiproc.py -q --timeout 150 --timeout-method thread -p no:cacheprovider -rf -m gpu > "$O/mp.out" 2> "$O/mp.err"
echo "mp rc=$? $(tail -1 $O/mp.out)"
grep "^FAILED" "$O/mp.out" | head
for seed in 21 22 23 24 25; do
  timeout -k 10 300 env STRESS_SEED=$seed STRESS_OPS=800 python -u -m pytest tests/test_multiproc.py -q -k "test_stress_random_programs" --timeout 250 --timeout-method thread -p no:cacheprovider > "$O/s_$seed.out" 2>&1
  echo "seed=$seed rc=$? $(tail -1 $O/s_$seed.out)"
done
for n in 2 3; do
  timeout -k 10 240 python3 -u bench.py --gpus $n --steps 10 --warmup 3 --no-cpu --ga-dims 12288 --c5-steps 4 > "$O/spawn$n.out" 2> "$O/spawn$n.err"
  echo "spawn$n rc=$? $(grep '^{' $O/spawn$n.out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["c5"]; print(c["M2"]["ms_per_step"], c["M2_src_in_segment"]["ms_per_step"], c["exchange_check"]["packed"]["result"], c["exchange_check"]["direct_src"]["result"])')"
done
echo done
