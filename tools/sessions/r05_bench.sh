# round-5 bench checks: the driver's N=1 line (host_inclusive block), the N=2
# rehearsal on one GPU (exchange precheck), the cross-device proxy, and a host-source
# remote accumulate on the proxy
set -o pipefail
out=gpurun_out/${R05_TAG:-r05s2}
mkdir -p $out
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/n1.json 2> $out/n1.err || exit 11
python3 -c "import json;d=json.load(open('$out/n1.json'));print('N1', d['value'], d['hbm_peak_frac'], d['roofline']['frac']); print(json.dumps(d.get('host_inclusive'))[:1500])"
timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 --ga-dims 16384 > $out/n2.json 2> $out/n2.err || exit 12
python3 -c "import json;d=json.load(open('$out/n2.json'));c=d['c5'];print('N2', d['value'], {k:v['result'] for k,v in c['exchange_precheck'].items()}, {k:v['result'] for k,v in c['exchange_check'].items()})"
COMEX_AMD_PEER_LOADS=all timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 --ga-dims 16384 > $out/n2_proxy.json 2> $out/n2_proxy.err || exit 13
python3 -c "import json;d=json.load(open('$out/n2_proxy.json'));c=d['c5'];print('N2proxy', d['value'], {k:v['result'] for k,v in c['exchange_precheck'].items()}, {k:v['result'] for k,v in c['exchange_check'].items()}, c['M2'].get('inter_rank_GBps_per_gpu'))"
COMEX_AMD_PEER_LOADS=all timeout -k 10 240 python3 bench.py --gpus 2 --exchange --host-src --sets 2 --no-extras --steps 20 --warmup 5 > $out/n2_hostsrc_exchange.json 2> $out/n2_hostsrc_exchange.err || exit 14
python3 -c "import json;d=json.load(open('$out/n2_hostsrc_exchange.json'));print('hostsrc exchange', d['value'], d.get('routes'), d['ms_per_step'])"
COMEX_AMD_PEER_LOADS=all timeout -k 10 240 python3 bench.py --gpus 2 --exchange --sets 2 --no-extras --steps 20 --warmup 5 > $out/n2_dev_exchange.json 2> $out/n2_dev_exchange.err || exit 15
python3 -c "import json;d=json.load(open('$out/n2_dev_exchange.json'));print('dev exchange', d['value'], d.get('routes'), d['ms_per_step'])"
