# round-5: small-call latency to a remote owner (2 ranks on one GPU, and with every peer
# treated as another GPU)
set -o pipefail
out=gpurun_out/r05lat3
mkdir -p $out
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 tools/latency_probe.py > $out/remote.jsonl 2> $out/remote.err || { tail -20 $out/remote.err; exit 11; }
grep remote $out/remote.jsonl
COMEX_AMD_PEER_LOADS=all timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29562 tools/latency_probe.py > $out/remote_proxy.jsonl 2> $out/remote_proxy.err || { tail -20 $out/remote_proxy.err; exit 12; }
grep remote $out/remote_proxy.jsonl
