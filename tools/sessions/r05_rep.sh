# round-5: small scatters with repeated destinations (host hash check -> GPU ordering instead
# of the one-lane serial kernel); io-vector tests
set -o pipefail
out=gpurun_out/r05rep
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_multiproc.py -m gpu -q -k "accv or getv or putv or io_vector or scatter or gather or stress or random_remote or vector" --timeout 200 --timeout-method thread -p no:cacheprovider > $out/iov.log 2>&1 || { tail -30 $out/iov.log; exit 10; }
tail -1 $out/iov.log
timeout -k 10 200 python3 tools/scatter_bench.py --pairs 64,256,1024,2047 --slots 200 --steps 50 > $out/rep.jsonl 2> $out/rep.err || { tail -5 $out/rep.err; exit 11; }
python3 -c "
import json
for l in open('$out/rep.jsonl'):
    d=json.loads(l); print(d['pairs'], d['repeated_destinations'], d['ms_per_call'], d['cpu_reference']['ms_per_call'])
"
timeout -k 10 200 python3 abtree/tools/scatter_bench.py --pairs 64,256,1024,2047 --slots 200 --steps 50 > $out/rep_old.jsonl 2> $out/rep_old.err || { tail -5 $out/rep_old.err; exit 12; }
python3 -c "
import json
for l in open('$out/rep_old.jsonl'):
    d=json.loads(l); print('old', d['pairs'], d['repeated_destinations'], d['ms_per_call'])
"
