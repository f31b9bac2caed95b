# round-5: stamps of a small blocking call with two ranks on one GPU (both busy / other idle)
set -o pipefail
out=gpurun_out/r05lat5
mkdir -p $out
LAT_STAMPS=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29581 tools/latency_probe.py > $out/default.jsonl 2> $out/default.err || { tail -5 $out/default.err; exit 11; }
grep -E "stamps|accs_dev_64\"" $out/default.jsonl
LAT_STAMPS=1 COMEX_AMD_STREAMS=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29582 tools/latency_probe.py > $out/streams1.jsonl 2> $out/streams1.err || { tail -5 $out/streams1.err; exit 12; }
grep -E "stamps|accs_dev_64\"" $out/streams1.jsonl
