# round-5: the maps pass parsed by hand in 64 KiB pieces; GA gather/scatter locating owners twice
set -o pipefail
out=gpurun_out/r05scatter4
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "accv or getv" --timeout 120 --timeout-method thread -p no:cacheprovider > $out/iov_tests.log 2>&1 || { tail -30 $out/iov_tests.log; exit 10; }
tail -3 $out/iov_tests.log
timeout -k 10 200 python3 tools/scatter_bench.py --src host --pairs 65536,1048576,4194304 --no-cpu > $out/accv_host.jsonl 2> $out/accv_host.err || exit 11
cat $out/accv_host.jsonl
timeout -k 10 200 python3 tools/scatter_bench.py --ga --pairs 65536,1048576,4194304 > $out/ga.jsonl 2> $out/ga.err || exit 12
cat $out/ga.jsonl
COMEX_AMD_DEBUG=3 timeout -k 10 200 python3 tools/scatter_bench.py --ga --pairs 4194304 --steps 3 > $out/ga_trace.jsonl 2> $out/ga_trace.err || exit 13
COMEX_AMD_DEBUG=3 timeout -k 10 200 python3 tools/scatter_bench.py --src host --pairs 1048576 --steps 3 --no-cpu > $out/accv_trace.jsonl 2> $out/accv_trace.err || exit 14
grep 'iov ' $out/ga_trace.err | tail -24
echo ---
grep 'iov ' $out/accv_trace.err | tail -12
