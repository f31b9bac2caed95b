# round-5: multi-process GPU test durations with the one-stream rule and with two streams forced
set -o pipefail
out=gpurun_out/r05streams2
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_multiproc.py -m gpu -q --durations=12 --timeout 200 --timeout-method thread -p no:cacheprovider > $out/mp_rule.log 2>&1 || { tail -20 $out/mp_rule.log; exit 11; }
grep -A14 "slowest" $out/mp_rule.log | cut -c1-150
COMEX_AMD_STREAMS=2 timeout -k 10 600 python -u -m pytest tests/test_multiproc.py -m gpu -q --durations=12 --timeout 200 --timeout-method thread -p no:cacheprovider > $out/mp_two.log 2>&1 || { tail -20 $out/mp_two.log; exit 12; }
grep -A14 "slowest" $out/mp_two.log | cut -c1-150
