# round-5: why local small calls take ~55 us with two ranks on one GPU (15 us with every
# peer treated as another GPU): as is, with the one-pass route off, and one rank only busy
set -o pipefail
out=gpurun_out/r05lat4
mkdir -p $out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29570 + RANDOM % 100)) tools/latency_probe.py > $out/$tag.jsonl 2> $out/$tag.err || { tail -5 $out/$tag.err; return 1; }
  echo "$tag: $(grep -E '"accs_dev_64"|"NGA_Acc_16x16"' $out/$tag.jsonl | tr '\n' ' ')"
}
run default X=1 || exit 11
run onepass_off COMEX_AMD_ONE_PASS=0 || exit 12
run proxy COMEX_AMD_PEER_LOADS=all || exit 13
run streams1 COMEX_AMD_STREAMS=1 || exit 14
