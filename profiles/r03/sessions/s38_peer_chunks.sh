# round 3 session 38: two chunks per staging sub-ring for owners on another GPU (pack of k+1
# overlapping the pull of k): correctness of the forced cross-device paths, and the 2-rank
# exchange through the packed route with every peer treated as another GPU, 1 vs 2 chunks
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s38
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_multiproc.py -k "forced or stress" > gpurun_out/s38/forced.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/s38/forced.log | head; tail -1 gpurun_out/s38/forced.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for c in 1 2 4; do
    env -u RANK -u WORLD_SIZE -u LOCAL_RANK COMEX_AMD_PEER_LOADS=all COMEX_AMD_PEER_CHUNKS=$c timeout -k 10 300 python -u bench.py --gpus 2 --exchange --steps 60 --warmup 5 --no-cpu --no-extras --workload C3 > gpurun_out/s38/ex_c${c}_$i.json 2> gpurun_out/s38/ex_c${c}_$i.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/s38/ex_c${c}_$i.json')); print('chunks $c', d['value'], d['ms_per_step'], d.get('routes'))"
  done
done
