# round-5: random strided descriptors between two ranks on every route
set -o pipefail
out=gpurun_out/r05rdesc
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_multiproc.py -m gpu -v -k "random_remote_descriptors" --timeout 200 --timeout-method thread -p no:cacheprovider > $out/rdesc.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|assert" $out/rdesc.log | head -40 | cut -c1-500
exit $rc
