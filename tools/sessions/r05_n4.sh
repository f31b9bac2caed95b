# round-5: the driver's N > 1 shape with 4 ranks sharing this box's one GPU (the
# default routes, then every peer treated as another GPU), full 32768^2 C5 extras
set -o pipefail
out=gpurun_out/r05n4
mkdir -p $out
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 4 --steps 20 --warmup 5 > $out/n4.json 2> $out/n4.err || exit 11
python3 -c "import json;d=json.load(open('$out/n4.json'));c=d['c5'];print('N4', d['value'], d['topology'], {k:v['result'] for k,v in c['exchange_precheck'].items()}, {k:v['result'] for k,v in c['exchange_check'].items()}, c['M2']['ms_per_step'], c['M2_src_in_segment']['ms_per_step'])"
COMEX_AMD_PEER_LOADS=all timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29545 bench.py --gpus 4 --steps 20 --warmup 5 > $out/n4_proxy.json 2> $out/n4_proxy.err || exit 12
python3 -c "import json;d=json.load(open('$out/n4_proxy.json'));c=d['c5'];print('N4proxy', d['value'], d['topology'], {k:v['result'] for k,v in c['exchange_precheck'].items()}, {k:v['result'] for k,v in c['exchange_check'].items()}, c['M2']['ms_per_step'], c['M2_src_in_segment']['ms_per_step'], c['M2'].get('routes'))"
