# round-5: small pageable spans through a pinned bounce buffer -- the whole GPU suite, then
# the small-call latencies again
set -o pipefail
out=gpurun_out/r05bounce
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > $out/gpu_suite.log 2>&1
rc=$?
tail -2 $out/gpu_suite.log
grep -E "FAILED|ERROR" $out/gpu_suite.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/latency_probe.py > $out/latency.jsonl 2> $out/latency.err || { tail -10 $out/latency.err; exit 11; }
cat $out/latency.jsonl
