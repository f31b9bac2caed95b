# round 3 session 07: asynchronous one-pass (deferred lock release): tests, then the 2-rank exchange
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s07
P="python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 900 $P tests/test_multiproc.py -k "one_pass or c5 or c1 or stress or ga_layer or self_after or bench_two" > gpurun_out/s07/mp.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/s07/mp.log | tail -8; [ $rc -eq 0 ] || exit $rc
for mode in onepass packed; do
  op=1; [ $mode = packed ] && op=0
  env -u RANK -u WORLD_SIZE -u LOCAL_RANK COMEX_AMD_ONE_PASS=$op timeout -k 10 300 python -u bench.py --gpus 2 --exchange --steps 100 --warmup 5 --no-cpu --no-extras > gpurun_out/s07/exchange2_$mode.json 2> gpurun_out/s07/exchange2_$mode.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/s07/exchange2_$mode.json')); print('$mode', d['value'], 'GiB/s =', round(d['value']*2**30/8e12, 4), 'of one GPU')"
done
env -u RANK -u WORLD_SIZE -u LOCAL_RANK timeout -k 10 300 python -u bench.py --gpus 2 --exchange --api blocking --steps 100 --warmup 5 --no-cpu --no-extras > gpurun_out/s07/exchange2_onepass_blocking.json 2> gpurun_out/s07/exchange2_onepass_blocking.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/s07/exchange2_onepass_blocking.json')); print('onepass blocking', d['value'], round(d['value']*2**30/8e12, 4))"
