# round-5: re-measure on the current tree the figures DESIGN still quoted from rounds 1-4
# (strided put/get, element types, the packed pipeline and route to self, column sums,
# io-vector / GA scatter rates)
set -o pipefail
out=gpurun_out/r05refresh
mkdir -p $out
for x in put get; do
  for w in H C3 C4; do
    timeout -k 10 120 python3 bench.py --xfer $x --workload $w --steps 200 --warmup 20 --no-cpu --no-host \
      > $out/${x}_$w.json 2> $out/${x}_$w.err || exit 11
    cat $out/${x}_$w.json
  done
done
for op in 37 38 39 40 41 42; do
  timeout -k 10 150 python3 tools/shape_sweep.py --op $op --rows 128,1024,16384 > $out/types_$op.jsonl 2> $out/types_$op.err || exit 12
  cat $out/types_$op.jsonl
done
timeout -k 10 120 python3 bench.py --pipeline --steps 100 --warmup 10 --no-cpu --no-host > $out/pipeline_H.json 2> $out/pipeline_H.err || exit 13
cat $out/pipeline_H.json
timeout -k 10 120 python3 bench.py --self-packed --steps 100 --warmup 10 --no-cpu --no-host > $out/self_packed_H.json 2> $out/self_packed_H.err || exit 14
cat $out/self_packed_H.json
timeout -k 10 120 python3 tools/cols_rate.py 37 38 39 40 41 42 > $out/cols_rate.jsonl 2> $out/cols_rate.err || exit 15
cat $out/cols_rate.jsonl
timeout -k 10 300 python3 tools/scatter_bench.py --pairs 16384,65536,262144,1048576 > $out/scatter_accv.jsonl 2> $out/scatter_accv.err || exit 16
cat $out/scatter_accv.jsonl
timeout -k 10 300 python3 tools/scatter_bench.py --ga > $out/scatter_ga.jsonl 2> $out/scatter_ga.err || exit 17
cat $out/scatter_ga.jsonl
