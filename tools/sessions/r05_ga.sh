# round-5: the GA layer tests with irregular distributions
set -o pipefail
out=gpurun_out/r05ga
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_multiproc.py -m gpu -v -k "ga_layer" --timeout 200 --timeout-method thread -p no:cacheprovider > $out/ga.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|assert" $out/ga.log | head -30 | cut -c1-500
exit $rc
