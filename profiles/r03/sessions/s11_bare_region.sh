# round 3 session 11: the bare-HIP region of the headline shape (tools/completion_probe,
# no library: 20 launches of a minimal 2-D axpy kernel, two streams, host clock to both
# synchronizations) interleaved with driver-shaped bench runs on the same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s11
for i in 1 2 3; do
  timeout -k 10 120 ./tools/completion_probe 20 200 1 >> gpurun_out/s11/bare_region_H.jsonl 2>> gpurun_out/s11/bare.err || exit 1
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/s11/bench_$i.json 2> gpurun_out/s11/bench_$i.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/s11/bench_$i.json')); print('bench', d['hbm_peak_frac'], d['roofline']['frac'], d['value_region']['total_us'])"
done
BENCH_DIAG_REGIONS=40 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/s11/bench_diag40.json 2> gpurun_out/s11/bench_diag40.err || exit 1
cat gpurun_out/s11/bare_region_H.jsonl
python - <<'PY'
import json, statistics
d = json.load(open("gpurun_out/s11/bench_diag40.json"))
t = sorted(r["total_us"] for r in d["diag_regions"])
print("library regions (40 more, same process): min %.1f median %.1f max %.1f us" % (t[0], statistics.median(t), t[-1]))
PY
