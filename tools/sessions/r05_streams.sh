# round-5: one library stream per process when ranks share the GPU -- the whole GPU suite,
# 2-rank latency and the N=2 rehearsal
set -o pipefail
out=gpurun_out/r05streams
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > $out/gpu_suite.log 2>&1
rc=$?
tail -2 $out/gpu_suite.log; grep -E "FAILED|ERROR" $out/gpu_suite.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29901 tools/latency_probe.py > $out/lat_n2.jsonl 2> $out/lat_n2.err || { tail -5 $out/lat_n2.err; exit 11; }
grep -E '"accs_dev_64"|"accs_pageable_64"|"NGA_Acc_16x16"|remote_NGA_Acc_16x16' $out/lat_n2.jsonl
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29902 bench.py --gpus 2 --steps 20 --warmup 5 > $out/bench_n2.json 2> $out/bench_n2.err || { tail -5 $out/bench_n2.err; exit 12; }
python3 -c "import json;d=json.load(open('$out/bench_n2.json'));c=d['c5'];print('N2', d['value'], {k:v['result'] for k,v in c['exchange_precheck'].items()}, {k:v['result'] for k,v in c['exchange_check'].items()})"
