# round-5: where a GA scatter-accumulate of 1 Mi elements from host `v` spends its time
# (NGA_Scatter_acc_flat 10 ms against NGA_Gather_flat 3 ms in profiles/r05/refresh)
set -o pipefail
out=gpurun_out/r05scatter
mkdir -p $out
timeout -k 10 200 python3 tools/scatter_bench.py --src host --pairs 65536,1048576,4194304 --no-cpu > $out/accv_host.jsonl 2> $out/accv_host.err || exit 11
cat $out/accv_host.jsonl
timeout -k 10 200 python3 tools/scatter_bench.py --ga --pairs 65536,1048576,4194304 > $out/ga.jsonl 2> $out/ga.err || exit 12
cat $out/ga.jsonl
COMEX_AMD_DEBUG=3 timeout -k 10 200 python3 tools/scatter_bench.py --ga --pairs 1048576 --steps 3 > $out/ga_trace.jsonl 2> $out/ga_trace.err || exit 13
COMEX_AMD_DEBUG=3 timeout -k 10 200 python3 tools/scatter_bench.py --src host --pairs 1048576 --steps 3 --no-cpu > $out/accv_trace.jsonl 2> $out/accv_trace.err || exit 14
grep 'iov ' $out/ga_trace.err | tail -40
echo ---
grep 'iov ' $out/accv_trace.err | tail -20
