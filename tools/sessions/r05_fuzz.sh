# round-5: seeded random strided descriptors against the oracle (tests/test_gpu_fuzz.py)
set -o pipefail
out=gpurun_out/r05fuzz
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider > $out/fuzz.log 2>&1
rc=$?
tail -40 $out/fuzz.log | cut -c1-600
exit $rc
