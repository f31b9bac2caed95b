# round-5: non-blocking calls from small pageable sources through the per-thread pinned ring,
# and the completion flag for any source when the destination is HBM: the GPU suite, the
# small-call probe from C and the Python latency probe
set -euo pipefail
out=gpurun_out/${R05_TAG:-r05ring}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/small_call_probe 1024 > $out/small_calls.jsonl 2> $out/small_calls.err
cat $out/small_calls.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider > $out/gpu_suite.log 2>&1 || { grep -E "FAILED|Error|error" $out/gpu_suite.log | head -20; tail -3 $out/gpu_suite.log; exit 1; }
tail -1 $out/gpu_suite.log
timeout -k 10 120 python -u tools/latency_probe.py > $out/latency.jsonl 2> $out/latency.err
cat $out/latency.jsonl
