# round-5: the slow completion flag with two ranks on one GPU: other rank idle; a pull stream forced
set -o pipefail
out=gpurun_out/r05lat6
mkdir -p $out
run() {
  local tag=$1; shift
  env LAT_STAMPS=1 "$@" timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 100)) tools/latency_probe.py > $out/$tag.jsonl 2> $out/$tag.err || { tail -5 $out/$tag.err; return 1; }
  echo "$tag: $(grep -E 'stamps|"accs_dev_64"' $out/$tag.jsonl | tr '\n' ' ')"
}
run rank0_only LAT_ONLY_RANK0=1 || exit 11
run pull1 COMEX_AMD_PULL_STREAMS=1 || exit 12
run streams3 COMEX_AMD_STREAMS=3 || exit 13
run hwq8 GPU_MAX_HW_QUEUES=8 || exit 14
