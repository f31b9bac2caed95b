# round-5: device code as one module + flag page at init -- suite, the driver's N=1
# invocation twice (blocking_api at 20 steps), and the first comex_malloc's tag time
set -o pipefail
out=gpurun_out/r05s5
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider > $out/gpu_suite.log 2>&1
rc=$?
tail -2 $out/gpu_suite.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver_$i.json 2> $out/bench_driver_$i.err || exit 11
  python3 -c "import json;d=json.load(open('$out/bench_driver_$i.json'));b=d['blocking_api'];print('driver', d['value'], d['hbm_peak_frac'], d['roofline']['frac'], 'blocking', b['hbm_peak_frac'], b['c_caller']['hbm_peak_frac'])"
done
COMEX_AMD_DEBUG=1 timeout -k 10 120 python3 -u tools/malloc_repro.py 1 8 > $out/tagcost_ipc.log 2>&1 || exit 12
grep -E "tags" $out/tagcost_ipc.log | head -8
exit $rc
