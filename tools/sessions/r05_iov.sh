# round-5: io-vector contiguous-side fast path -- its parity tests, the multi-rank
# io-vector tests, and comex_accv / NGA_Scatter_acc rates against the previous code
# (ab_alt/), interleaved
set -o pipefail
out=gpurun_out/r05iov
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_semantics.py -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider -k "accv or putv or getv or vector or iov" > $out/tests_local.log 2>&1 || { tail -30 $out/tests_local.log; exit 11; }
tail -1 $out/tests_local.log
timeout -k 10 400 python -u -m pytest tests/test_multiproc.py -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider -k "vector or scatter or toggles" > $out/tests_mp.log 2>&1 || { tail -30 $out/tests_mp.log; exit 12; }
tail -1 $out/tests_mp.log
for i in 1 2; do
  timeout -k 10 120 python3 tools/scatter_bench.py --pairs 16384,65536,262144,1048576 --no-cpu --steps 50 > $out/new_$i.jsonl 2>&1 || exit 13
  timeout -k 10 120 python3 ab_alt/tools/scatter_bench.py --pairs 16384,65536,262144,1048576 --no-cpu --steps 50 > $out/old_$i.jsonl 2>&1 || exit 14
done
timeout -k 10 120 python3 tools/scatter_bench.py --pairs 16384,65536,262144 --steps 50 > $out/new_cpu.jsonl 2>&1 || exit 15
for f in $out/new_1.jsonl $out/old_1.jsonl $out/new_2.jsonl $out/old_2.jsonl $out/new_cpu.jsonl; do echo $f; python3 -c "
import json,sys
for l in open('$f'):
    try: d=json.loads(l)
    except Exception: continue
    print(d.get('pairs'), d.get('ms_per_call'), d.get('cpu_ms_per_call', d.get('cpu_ref_ms_per_call')))"; done
