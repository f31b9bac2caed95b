# round-5: io-vector tests after moving the GPU-ordering threshold to 2048 pairs
set -o pipefail
out=gpurun_out/r05iovtests
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_multiproc.py -m gpu -v -k "accv or getv or putv or io_vector or scatter or gather or stress or random_remote" --timeout 200 --timeout-method thread -p no:cacheprovider > $out/iov.log 2>&1
rc=$?
tail -2 $out/iov.log
grep -E "FAILED" $out/iov.log | head
exit $rc
