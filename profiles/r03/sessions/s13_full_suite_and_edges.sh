# round 3 session 13 (re-entry after the container was re-created):
# (1) the region's edges: does a store policy that leaves no dirty L2 lines (write-through)
#     shorten the end-of-launch release?  bare-HIP probe, regions of K and 2K launches per
#     policy (slope = per launch, intercept = the two edges); and the HSA runtime's completion
#     signalling without interrupts (HSA_ENABLE_INTERRUPT=0) on the probe and on driver-shaped
#     bench runs, interleaved;
# (2) the whole GPU suite as the driver runs it (new: the library's own radix sort, the bench
#     extras watchdog), smoke, a driver-shaped bench with the CPU baseline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s13
export TMPDIR=/tmp
timeout -k 10 200 ./tools/completion_probe 20 60 2 > gpurun_out/s13/store_policy.jsonl 2> gpurun_out/s13/sp.err || exit 1
cat gpurun_out/s13/store_policy.jsonl
HSA_ENABLE_INTERRUPT=0 timeout -k 10 200 ./tools/completion_probe 20 60 2 > gpurun_out/s13/store_policy_noint.jsonl 2> gpurun_out/s13/sp2.err || exit 1
cat gpurun_out/s13/store_policy_noint.jsonl
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/s13/bench_int_$i.json 2> gpurun_out/s13/bench_int_$i.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/s13/bench_int_$i.json')); print('interrupts', d['hbm_peak_frac'], d['roofline']['frac'], d['value_region']['total_us'])"
  HSA_ENABLE_INTERRUPT=0 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/s13/bench_noint_$i.json 2> gpurun_out/s13/bench_noint_$i.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/s13/bench_noint_$i.json')); print('polling', d['hbm_peak_frac'], d['roofline']['frac'], d['value_region']['total_us'])"
done
timeout -k 10 900 python -u -m pytest tests/ -x -v --timeout 480 --timeout-method thread -m gpu > gpurun_out/s13/gpu_suite.log 2>&1
rc=$?; tail -4 gpurun_out/s13/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s13/smoke.log 2>&1 || exit 1
cat gpurun_out/s13/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s13/bench.json 2> gpurun_out/s13/bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/s13/bench.json')); print('H', d['value'], d['hbm_peak_frac'], d['roofline']['frac'], d['value_region']['total_us'], d.get('blocking_api'))"
