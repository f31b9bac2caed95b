# round-5: GPU suite after the fence/owner-event publication change, and the exchange
# rates on the one-GPU proxy against profiles/r05/s2 (same commands)
set -o pipefail
out=gpurun_out/r05s4
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider > $out/gpu_suite.log 2>&1
rc=$?
tail -2 $out/gpu_suite.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
COMEX_AMD_PEER_LOADS=all timeout -k 10 240 python3 bench.py --gpus 2 --exchange --sets 2 --no-extras --steps 50 --warmup 5 > $out/n2_dev_exchange_$i.json 2> $out/n2_dev_exchange_$i.err || exit 15
python3 -c "import json;d=json.load(open('$out/n2_dev_exchange_$i.json'));print('dev exchange packed', d['value'], d['ms_per_step'])"
COMEX_AMD_PEER_LOADS=all timeout -k 10 240 python3 bench.py --gpus 2 --exchange --src-seg --sets 2 --no-extras --steps 50 --warmup 5 > $out/n2_srcseg_exchange_$i.json 2> $out/n2_srcseg_exchange_$i.err || exit 16
python3 -c "import json;d=json.load(open('$out/n2_srcseg_exchange_$i.json'));print('dev exchange direct-source', d['value'], d['ms_per_step'], d.get('routes'))"
done
COMEX_AMD_PEER_LOADS=all timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 --ga-dims 16384 > $out/n2_proxy.json 2> $out/n2_proxy.err || exit 13
python3 -c "import json;d=json.load(open('$out/n2_proxy.json'));c=d['c5'];print('N2proxy', d['value'], {k:v['result'] for k,v in c['exchange_precheck'].items()}, {k:v['result'] for k,v in c['exchange_check'].items()}, c['M2']['ms_per_step'], c['M2_src_in_segment']['ms_per_step'])"
exit $rc
