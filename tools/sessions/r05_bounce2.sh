# round-5: shared-page pageable patches (bounce union and registered union), host operand tests
set -o pipefail
out=gpurun_out/r05bounce2
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_semantics.py tests/test_legacy_acc.py -m gpu -v -k "pageable or host" --timeout 120 --timeout-method thread -p no:cacheprovider > $out/t.log 2>&1
rc=$?
tail -2 $out/t.log; grep FAILED $out/t.log | head; grep -E "^E " $out/t.log | head -20
exit $rc
