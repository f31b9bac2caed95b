# round 3 session 39: the final binary -- the GPU suite exactly as the driver runs it, and smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s39
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q --timeout 480 --timeout-method thread -m gpu > gpurun_out/s39/gpu_suite.log 2>&1
rc=$?; tail -2 gpurun_out/s39/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s39/smoke.log 2>&1 || exit 1
cat gpurun_out/s39/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/s39/bench_default.json 2> gpurun_out/s39/bench_default.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/s39/bench_default.json')); print('bench (no flags)', d['value'], d['hbm_peak_frac'], d['roofline']['frac'], d['steps'], d['cpu_baseline']['value'])"
