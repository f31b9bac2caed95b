# round-5 GPU check: the whole GPU suite, then the cost of the whole-block tag check
set -o pipefail
out=gpurun_out/${R05_TAG:-r05s1}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread > $out/gpu_suite.log 2>&1
rc=$?
tail -5 $out/gpu_suite.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for alloc in ipc vmm; do
  COMEX_AMD_DEBUG=1 COMEX_AMD_SEGMENT_ALLOC=$alloc timeout -k 10 120 python3 -u tools/malloc_repro.py 1 8 > $out/tagcost_$alloc.log 2>&1 || exit 3
  grep -E "tags|OK" $out/tagcost_$alloc.log | head -12
done
exit $rc
