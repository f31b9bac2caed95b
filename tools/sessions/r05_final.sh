# round-5 evidence set, one GPU call: the GPU suite, smoke, the driver's N=1 invocation
# three times, tools/evidence.sh (PMC, configs, rocprofv3 kernel traces), and the
# driver's N=2 shape under torch.distributed.run on this box's one GPU
set -euo pipefail
out=gpurun_out/${R05_TAG:-r05final}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider > $out/gpu_suite.log 2>&1
tail -2 $out/gpu_suite.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
for i in 1 2 3; do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver_$i.json 2> $out/bench_driver_$i.err
  python3 -c "import json;d=json.load(open('$out/bench_driver_$i.json'));print('driver', d['value'], d['hbm_peak_frac'], d['roofline']['frac'])"
done
bash tools/evidence.sh r05
cp -r gpurun_out/evidence $out/
timeout -k 10 300 python3 bench.py --workload C5 --no-cpu > $out/bench_C5_n1.json 2> $out/bench_C5_n1.err
python3 -c "import json;d=json.load(open('$out/bench_C5_n1.json'));print('C5 N=1', d['value'], d['hbm_peak_frac'], d['roofline']['frac'])"
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 2 --steps 20 --warmup 5 > $out/bench_n2.json 2> $out/bench_n2.err
python3 -c "import json;d=json.load(open('$out/bench_n2.json'));c=d['c5'];print('N2', d['value'], {k:v['result'] for k,v in c['exchange_precheck'].items()}, {k:v['result'] for k,v in c['exchange_check'].items()})"
