# round-5: hashed io-vector insert with claim + dup mark -- io-vector tests, kernel trace
# of 16 Ki / 64 Ki calls, whole-call rates
set -o pipefail
out=gpurun_out/${R05_TAG:-r05iov2}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_semantics.py -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider -k "accv or putv or getv or vector or iov" > $out/tests_local.log 2>&1 || { tail -30 $out/tests_local.log; exit 11; }
tail -1 $out/tests_local.log
timeout -k 10 400 python -u -m pytest tests/test_multiproc.py -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider -k "vector or scatter or toggles" > $out/tests_mp.log 2>&1 || { tail -30 $out/tests_mp.log; exit 12; }
tail -1 $out/tests_mp.log
for n in 16384 65536; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p$n -o iov -- python3 tools/scatter_bench.py --pairs $n --no-cpu --steps 200 > $out/trace_bench_$n.jsonl 2> $out/trace_bench_$n.err || exit 13
  find $out/p$n -name '*kernel_stats.csv' -exec cp {} $out/stats_$n.csv \;
  cut -c1-60,200- $out/stats_$n.csv | head -6
done
for i in 1 2; do
  timeout -k 10 120 python3 tools/scatter_bench.py --pairs 16384,65536,262144,1048576 --steps 50 > $out/rates_$i.jsonl 2>&1 || exit 14
done
for f in $out/rates_1.jsonl $out/rates_2.jsonl; do python3 -c "
import json
for l in open('$f'):
    try: d=json.loads(l)
    except Exception: continue
    print(d['pairs'], d['ms_per_call'], d['cpu_reference']['ms_per_call'])"; done
