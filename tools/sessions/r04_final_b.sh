#!/bin/bash
# round 4 final B: evidence (PMC, bench lines, rocprofv3 kernel trace + stats) and three
# driver-shaped N=1 lines
set -o pipefail
O=gpurun_out/r04final
mkdir -p $O
bash tools/evidence.sh r04 || exit $?
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$i.json 2> $O/bench_driver_$i.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_driver_$i.json'));print('driver-shaped', d['value'], d['hbm_peak_frac'], d['roofline']['frac'], d['blocking_api']['hbm_peak_frac'], d['blocking_api']['c_caller']['hbm_peak_frac'])"
done
