# round 3 session 14: (1) store-policy A/B on the bare-HIP headline region with controls
# (two copies of the library's nt config), the order rotating every round, 300 rounds, regions
# of K and 2K launches; (2) the whole GPU suite (the interleaved-columns perf floor relaxed:
# 0.707 of peak on the s13 box), smoke, a driver-shaped bench with the CPU baseline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s14
export TMPDIR=/tmp
timeout -k 10 200 ./tools/completion_probe 20 300 2 "0:0,0:4,4:4,0:0,0:1,1:1" > gpurun_out/s14/store_ab.jsonl 2> gpurun_out/s14/sp.err || exit 1
cat gpurun_out/s14/store_ab.jsonl
timeout -k 10 900 python -u -m pytest tests/ -v --timeout 480 --timeout-method thread -m gpu > gpurun_out/s14/gpu_suite.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/s14/gpu_suite.log | head; tail -2 gpurun_out/s14/gpu_suite.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s14/smoke.log 2>&1 || exit 1
cat gpurun_out/s14/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s14/bench.json 2> gpurun_out/s14/bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/s14/bench.json')); print('H', d['value'], d['hbm_peak_frac'], d['roofline']['frac'], d['value_region']['total_us'], d.get('blocking_api'), d['cpu_baseline'])"
