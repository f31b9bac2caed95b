# round-5: the whole GPU suite with the random-descriptor, irregular-GA and ARMCI-surface tests
set -o pipefail
out=gpurun_out/r05suite2
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > $out/gpu_suite.log 2>&1
rc=$?
tail -3 $out/gpu_suite.log
grep -E "FAILED|ERROR" $out/gpu_suite.log | head -20
exit $rc
