# round-5: streaming accumulate rate against the allocation (hipMalloc vs contiguous), 1..8 GiB
set -o pipefail
out=gpurun_out/r05alloc
mkdir -p $out
timeout -k 10 300 ./tools/alloc_probe > $out/alloc_probe.jsonl 2> $out/alloc_probe.err || { tail -5 $out/alloc_probe.err; exit 11; }
cat $out/alloc_probe.jsonl
