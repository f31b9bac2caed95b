# round-5: the rest of the ARMCI / comex / message surface under test
set -o pipefail
out=gpurun_out/r05armci
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_multiproc.py -m gpu -v -k "armci_message_groups or ga_layer" --timeout 200 --timeout-method thread -p no:cacheprovider > $out/armci.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|assert|rank . rc" $out/armci.log | head -30 | cut -c1-600
exit $rc
