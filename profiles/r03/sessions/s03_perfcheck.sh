# round 3 session 03: is the headline kernel slower after the kernel-set trim, or is it the box?
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s03
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_semantics.py -k "interleaved or ordered_kernel_large" > gpurun_out/s03/tests.log 2>&1
rc=$?; grep -E "GB/s|passed|failed" gpurun_out/s03/tests.log
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s03/bench_$i.json 2> gpurun_out/s03/bench_$i.err || exit 1
  python - <<PY
import json; d = json.load(open("gpurun_out/s03/bench_$i.json"))
print("bench", $i, d["value"], d["hbm_peak_frac"], d["roofline"]["frac"], d["value_region"])
PY
done
exit $rc
