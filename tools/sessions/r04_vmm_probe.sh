#!/bin/bash
# round 4: three processes exchanging VMM blocks by dmabuf descriptor (tools/vmm_probe.hip),
# repeated to get failure rates: same / distinct virtual addresses, blocks released every
# round or kept.  Every failing run's output is kept.
O=gpurun_out/r04vp
mkdir -p $O
N=${N:-15}
for m in ${MODES:-distinctva samevva distinctva_keep samevva_keep}; do
  fails=0; wrong=0; sa=0
  for i in $(seq 1 $N); do
    timeout -k 5 60 ./tools/vmm_probe $m 8 > $O/cur.txt 2>&1
    rc=$?
    w=$(grep -c WRONG $O/cur.txt); s=$(grep -c 'hipMemSetAccess.*invalid' $O/cur.txt)
    wrong=$((wrong + w)); sa=$((sa + s))
    if [ $rc -ne 0 ]; then fails=$((fails + 1)); cp $O/cur.txt $O/${m}_fail_$i.txt; fi
    [ $rc -eq 124 ] || [ $rc -eq 137 ] && { echo "$m run $i timed out"; exit 1; }
  done
  echo "$m: $fails of $N runs failed; WRONG reads $wrong; refused hipMemSetAccess $sa" | tee -a $O/summary.txt
done
