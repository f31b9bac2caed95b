#!/bin/bash
# round 4 session 3: host segments; the virtual-memory segment allocator (vmm.cpp) under
# the multi-rank suite; then the stale-IPC-mapping campaign of r03/s32-s33 (eight ranks on
# one GPU, freed segments going back to the runtime, lease off) -- IPC segments with the
# handle table (every stale mapping reported with the handle bytes it opened and the handle
# of the allocation it reached) against vmm segments.
set -o pipefail
O=${OUT:-gpurun_out/r04s03}
mkdir -p $O
export PYTHONUNBUFFERED=1
[ -n "$SKIP_HOSTSEG" ] || timeout -k 10 300 python -u -m pytest tests/test_multiproc.py -q -k "host_segments" --timeout 200 --timeout-method thread > $O/hostseg.log 2>&1; echo "hostseg rc=$?"; tail -3 $O/hostseg.log
rc=0
[ -n "$SKIP_VMMTEST" ] || { timeout -k 10 600 python -u -m pytest tests/test_multiproc.py -q -k "vmm_segments" --timeout 170 --timeout-method thread > $O/vmm.log 2>&1; rc=$?; echo "vmm rc=$rc"; tail -3 $O/vmm.log; }
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ $rc -eq 0 ] || [ -z "$STOP_ON_VMM_FAIL" ] || exit $rc
REPS=${REPS:-10}
for alloc in ${ALLOCS:-ipc vmm}; do
  for i in $(seq 1 $REPS); do
    if [ -n "$DEFAULTS" ]; then cfg=""; else cfg="COMEX_AMD_SEGMENT_CACHE_MB=0 COMEX_AMD_ONE_PASS_LEASE_US=0"; fi
    env COMEX_AMD_SEGMENT_ALLOC=$alloc $cfg BENCH_CHECK_LOOPS=2 timeout -k 10 150 \
      python bench.py --gpus 8 --steps 2 --warmup 1 --warmup-ms 0 --no-cpu --ga-dims 16384 --c5-steps 2 \
      > $O/${alloc}_$i.json 2> $O/${alloc}_$i.err
    rc=$?
    ref=$(grep -c "hipIpcGetMemHandle of a" $O/${alloc}_$i.err)
    st=$(grep -c "not its tags" $O/${alloc}_$i.err)
    sa=$(grep -c "hipMemSetAccess.*refused" $O/${alloc}_$i.err)
    mm=$(python -c "import json;d=json.load(open('$O/${alloc}_$i.json'));c=d['c5'];print(sum(v['mismatches'] for v in c['exchange_check_loops'].values())+sum(v['result']!='exact' for v in c['exchange_check'].values()))" 2>/dev/null || echo "?")
    echo "${alloc}_$i ${DEFAULTS:+defaults }rc $rc refusals $ref access_refused $sa stale $st mismatches $mm" | tee -a $O/summary.txt
    [ $rc -eq 0 ] || exit $rc
  done
done
