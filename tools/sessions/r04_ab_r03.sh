#!/bin/bash
# round 4: the round-3 library (tools/ab/r03: its bench.py + ga_amd built from e5fc198) against
# this tree on one box, interleaved: C5 M1 at N=1 and the headline H (no-flag bench)
O=gpurun_out/r04ab
mkdir -p $O
for i in 1 2; do
  for w in C5 H; do
    (cd tools/ab/r03 && timeout -k 10 200 python bench.py --workload $w --no-cpu) > $O/r03_${w}_$i.json 2>/dev/null || exit 1
    timeout -k 10 200 python bench.py --workload $w --no-cpu > $O/r04_${w}_$i.json 2>/dev/null || exit 1
    for t in r03 r04; do
      python -c "import json;d=json.load(open('$O/${t}_${w}_$i.json'));print('$t $w $i', d['value'], d['hbm_peak_frac'], d['ms_per_step'], d.get('roofline',{}).get('kernel_ms_avg'))"
    done
  done
done
