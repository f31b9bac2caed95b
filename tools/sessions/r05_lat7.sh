# round-5: ranks sharing one GPU -- small-call latency and the headline's aggregate rate with
# 1, 2 and 3 library streams per process, 2 and 4 ranks
set -o pipefail
out=gpurun_out/r05lat7
mkdir -p $out
for n in 2 4; do
  for s in 1 2 3; do
    COMEX_AMD_STREAMS=$s LAT_STAMPS=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29700 + 10 * n + s)) tools/latency_probe.py > $out/lat_n${n}_s$s.jsonl 2> $out/lat_n${n}_s$s.err || { tail -5 $out/lat_n${n}_s$s.err; exit 11; }
    echo "n=$n streams=$s: $(grep -E '"accs_dev_64"|"accs_dev_65536"|"NGA_Acc_16x16"' $out/lat_n${n}_s$s.jsonl | tr '\n' ' ')"
    timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29800 + 10 * n + s)) bench.py --gpus $n --steps 200 --warmup 10 --no-cpu --no-extras --streams $s > $out/bench_n${n}_s$s.json 2> $out/bench_n${n}_s$s.err || { tail -5 $out/bench_n${n}_s$s.err; exit 12; }
    python3 -c "import json;d=json.load(open('$out/bench_n${n}_s$s.json'));print('  bench n=$n streams=$s', d['value'], d['ms_per_step'])"
  done
done
