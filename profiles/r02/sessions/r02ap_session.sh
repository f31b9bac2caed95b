#!/bin/bash
# round-2 GPU session ap: stress campaign -- the seeded random multi-rank programs with
# other seeds and longer programs (latent ordering races like the inbox one)
set -uo pipefail
O=gpurun_out/r02ap
mkdir -p "$O"
export TMPDIR=/tmp
for seed in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 400 env STRESS_SEED=$seed STRESS_OPS=800 python -u -m pytest tests/test_multiproc.py -q -k "test_stress_random_programs" --timeout 300 --timeout-method thread -p no:cacheprovider -rf > "$O/s_$seed.out" 2> "$O/s_$seed.err"
  rc=$?
  echo "seed=$seed rc=$rc $(tail -1 $O/s_$seed.out)"
  grep -h "^FAILED\|differ\|Error" "$O/s_$seed.out" | head -4 | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
echo done
