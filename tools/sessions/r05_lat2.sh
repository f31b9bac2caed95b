# round-5: small-call latency after polling the completion event before blocking
set -o pipefail
out=gpurun_out/r05lat2
mkdir -p $out
timeout -k 10 300 python3 tools/latency_probe.py > $out/latency.jsonl 2> $out/latency.err || { tail -10 $out/latency.err; exit 11; }
cat $out/latency.jsonl
