# round 3 session 31: round-end evidence on the final tree (after the one-pass floor/lease, the segment cache) -- the GPU suite as the driver runs
# it, smoke, three driver-shaped headline runs (CPU baseline included), rocprofv3 kernel trace +
# stats of the same command (two library streams, and one), PMC HBM traffic of the headline
# kernel (separate FETCH_SIZE / WRITE_SIZE passes), the other single-GPU configs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s31
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -v --timeout 480 --timeout-method thread -m gpu > $O/gpu_suite.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_suite.log | head; tail -1 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
cat $O/smoke.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$i.json 2> $O/bench_driver_$i.err || exit 1
  python -c "import json; d=json.load(open('$O/bench_driver_$i.json')); print('H', d['value'], d['hbm_peak_frac'], d['roofline']['frac'], d['roofline']['kernel_ms_avg'], d['value_region']['total_us'], d['blocking_api']['hbm_peak_frac'], d['cpu_baseline']['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_prof_2streams.json 2> $O/bench_prof_2streams.err || exit 1
find $O/prof2 -name '*kernel_stats.csv' -exec cp {} $O/rocprof_stats_2streams.csv \;
find $O/prof2 -name '*kernel_trace.csv' -exec cp {} $O/rocprof_trace_2streams.csv \;
python3 tools/kernel_union.py $O/rocprof_trace_2streams.csv --json $O/kernel_union_2streams.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --tune streams=1 > $O/bench_prof_1stream.json 2> $O/bench_prof_1stream.err || exit 1
find $O/prof1 -name '*kernel_stats.csv' -exec cp {} $O/rocprof_stats_1stream.csv \;
head -3 $O/rocprof_stats_1stream.csv
timeout -k 10 400 python3 tools/pmc_traffic.py --workload H --tag r03_final > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
tail -3 $O/pmc.log
cp profiles/pmc_latest.json profiles/pmc_r03*.json $O/ 2>/dev/null
for w in C2 C3 C4 H8200; do
  timeout -k 10 300 python bench.py --gpus 1 --workload $w --steps 100 --warmup 5 --no-cpu > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
  python -c "import json; d=json.load(open('$O/bench_$w.json')); print('$w', d['hbm_peak_frac'], d['roofline']['frac'])"
done
rm -rf $O/prof1 $O/prof2
