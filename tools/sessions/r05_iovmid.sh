# round-5: io-vector calls of 256..8192 pairs (host overlap check below kIovRunsMin, the GPU
# ordered path from it); TAG names the build being measured
set -o pipefail
out=gpurun_out/r05iovmid
mkdir -p $out
timeout -k 10 200 python3 tools/scatter_bench.py --pairs 16,64,256,512,1024,2047,2048,4096,8192 --steps 50 > $out/accv_$TAG.jsonl 2> $out/accv_$TAG.err || { tail -5 $out/accv_$TAG.err; exit 11; }
python3 -c "
import json
for l in open('$out/accv_$TAG.jsonl'):
    d=json.loads(l); print(d['pairs'], d['ms_per_call'], d['cpu_reference']['ms_per_call'])
"
