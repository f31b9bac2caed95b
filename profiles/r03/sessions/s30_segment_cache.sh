# round 3 session 30: freed segments kept with their IPC export for the next comex_malloc of
# the same size (no hipFree / hipMalloc / export churn at recycled addresses): the multi-rank
# suite (new: test_segment_cache_reuse), then the 8-rank one-GPU bench rehearsal with the
# exchange check repeated, counting export refusals
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s30
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_multiproc.py > gpurun_out/s30/multiproc.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/s30/multiproc.log | head; tail -1 gpurun_out/s30/multiproc.log; [ $rc -eq 0 ] || exit $rc
for dims in 16384 32768; do
  BENCH_CHECK_LOOPS=6 timeout -k 10 600 python -u bench.py --gpus 8 --steps 3 --warmup 1 --warmup-ms 0 --no-cpu --ga-dims $dims --c5-steps 2 > gpurun_out/s30/bench8_$dims.json 2> gpurun_out/s30/bench8_$dims.err || { tail -5 gpurun_out/s30/bench8_$dims.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/s30/bench8_$dims.json'))['c5']
print('$dims', 'M2', d['M2']['ms_per_step'], 'M2 seg', d['M2_src_in_segment']['ms_per_step'], {k: v['result'] for k, v in d['exchange_check'].items()}, {k: (v['mismatches'], v['loops']) for k, v in d['exchange_check_loops'].items()})"
  echo "refusals: $(grep -c hipIpcGetMemHandle gpurun_out/s30/bench8_$dims.err)"
done
