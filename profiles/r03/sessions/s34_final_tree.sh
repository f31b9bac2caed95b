# round 3 session 34: the final tree (segment tags, staging tag check): the GPU suite as the
# driver runs it, smoke, three driver-shaped headline runs, and the driver's N = 8 invocation
# rehearsed with eight ranks on one GPU at the configured GA size
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s34
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -v --timeout 480 --timeout-method thread -m gpu > $O/gpu_suite.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_suite.log | head; tail -1 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
cat $O/smoke.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$i.json 2> $O/bench_driver_$i.err || exit 1
  python -c "import json; d=json.load(open('$O/bench_driver_$i.json')); print('H', d['value'], d['hbm_peak_frac'], d['roofline']['frac'], d['value_region']['total_us'], d['blocking_api']['hbm_peak_frac'], d['cpu_baseline']['value'])"
done
timeout -k 10 600 python -u bench.py --gpus 8 --steps 5 --warmup 1 --no-cpu > $O/bench8_onegpu.json 2> $O/bench8_onegpu.err || { tail -5 $O/bench8_onegpu.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench8_onegpu.json')); c=d['c5']
print('N=8 on one GPU', d['value'], 'M1', c['M1']['ms_per_step'], 'M2', c['M2']['ms_per_step'], 'M2 seg', c['M2_src_in_segment']['ms_per_step'], {k: v['result'] for k, v in c['exchange_check'].items()})"
echo "refusals: $(grep -c hipIpcGetMemHandle $O/bench8_onegpu.err) stale: $(grep -c 'not its tag' $O/bench8_onegpu.err)"
