# round 3 session 15: write-through (sc1) stores in the streaming kernels (store_wt=1, the new
# default) against nt stores (store_wt=0): parity of the kernel families under both, then
# driver-shaped headline runs interleaved, the other configs (C2, C3, C4, H8200) with both,
# and the row-length sweep (flat kernel) with both
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s15
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_semantics.py > gpurun_out/s15/kernel_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s15/kernel_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for wt in 1 0; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --tune store_wt=$wt > gpurun_out/s15/bench_wt${wt}_$i.json 2> gpurun_out/s15/bench_wt${wt}_$i.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/s15/bench_wt${wt}_$i.json')); print('H wt=$wt', d['hbm_peak_frac'], d['roofline']['frac'], d['value_region']['total_us'])"
  done
done
for w in C2 C3 C4 H8200; do
  for wt in 1 0; do
    timeout -k 10 300 python bench.py --gpus 1 --workload $w --steps 100 --warmup 5 --no-cpu --tune store_wt=$wt > gpurun_out/s15/bench_${w}_wt$wt.json 2> gpurun_out/s15/bench_${w}_wt$wt.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/s15/bench_${w}_wt$wt.json')); print('$w wt=$wt', d['hbm_peak_frac'], d['roofline']['frac'])"
  done
done
for wt in 1 0; do
  timeout -k 10 300 python -u tools/shape_sweep.py --rows 64,128,256,512,1024,4096,16384 --tune store_wt=$wt > gpurun_out/s15/shape_wt$wt.jsonl 2> gpurun_out/s15/shape_wt$wt.err || exit 1
done
paste -d' ' <(python -c "
import json
for l in open('gpurun_out/s15/shape_wt1.jsonl'):
    d=json.loads(l); print('row', d.get('row_bytes'), 'wt1', d['frac_8TBps'], d['kernel']['kind'])") <(python -c "
import json
for l in open('gpurun_out/s15/shape_wt0.jsonl'):
    d=json.loads(l); print('wt0', d['frac_8TBps'], d['kernel']['kind'])")
