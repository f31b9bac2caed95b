# round 3 session 12: the hashed io-vector path (parity tests, then the small-n scatter A/B
# against the radix path), and the bare-HIP region of the headline shape interleaved with
# driver-shaped bench runs (tools/completion_probe, mode 1)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s12
export TMPDIR=/tmp
P="python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 400 $P tests/test_gpu_parity.py -k "accv or iov or getv or putv" > gpurun_out/s12/iov_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/s12/iov_tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for h in 1 0; do
    COMEX_AMD_IOV_HASH=$h timeout -k 10 200 python -u tools/scatter_bench.py --pairs 16384,65536,262144,1048576 --steps 40 > gpurun_out/s12/scatter_h${h}_$i.jsonl 2> gpurun_out/s12/scatter_h${h}_$i.err || exit 1
    python -c "
import json
for l in open('gpurun_out/s12/scatter_h${h}_$i.jsonl'):
    d = json.loads(l)
    if 'pairs' in d: print('hash=$h', d['pairs'], d['ms_per_call'], d.get('cpu_reference', {}).get('ms_per_call'))"
  done
done
for i in 1 2 3; do
  timeout -k 10 120 ./tools/completion_probe 20 200 1 >> gpurun_out/s12/bare_region_H.jsonl 2>> gpurun_out/s12/bare.err || exit 1
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/s12/bench_$i.json 2> gpurun_out/s12/bench_$i.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/s12/bench_$i.json')); print('bench', d['hbm_peak_frac'], d['roofline']['frac'], d['value_region']['total_us'])"
done
cat gpurun_out/s12/bare_region_H.jsonl
BENCH_DIAG_REGIONS=40 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/s12/bench_diag40.json 2> gpurun_out/s12/bench_diag40.err || exit 1
python - <<'PY'
import json, statistics
d = json.load(open("gpurun_out/s12/bench_diag40.json"))
t = sorted(r["total_us"] for r in d["diag_regions"])
print("library regions (40 more, same process): min %.1f median %.1f max %.1f us" % (t[0], statistics.median(t), t[-1]))
PY
