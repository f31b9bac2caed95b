# round-5: kernel trace of small io-vector calls (16 Ki and 64 Ki single-f64 pairs)
set -o pipefail
out=gpurun_out/r05ivt
mkdir -p $out
export TMPDIR=/tmp
for n in 16384 65536; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p$n -o iov -- python3 tools/scatter_bench.py --pairs $n --no-cpu --steps 200 > $out/bench_$n.jsonl 2> $out/bench_$n.err || exit 11
  find $out/p$n -name '*kernel_stats.csv' -exec cp {} $out/stats_$n.csv \;
  find $out/p$n -name '*kernel_trace.csv' -exec cp {} $out/trace_$n.csv \;
  cat $out/stats_$n.csv
done
