# round 3 session 09: IPC export probe with the file-descriptor scenarios, a kernel trace of
# the 64 Ki-pair io-vector call, stamped + one-stream profiled headline runs (region edges,
# dispatch tail), the whole multi-rank suite on the current tree
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s09
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ipc_export_probe.py 16 > gpurun_out/s09/ipc_probe.jsonl 2> gpurun_out/s09/ipc_probe.err
rc=$?; cat gpurun_out/s09/ipc_probe.jsonl | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/s09/prof_scatter -o run -- python3 tools/scatter_bench.py --pairs 65536 --steps 200 --no-cpu > gpurun_out/s09/scatter_prof.jsonl 2> gpurun_out/s09/scatter_prof.err || exit 1
cat gpurun_out/s09/scatter_prof.jsonl
BENCH_STAMPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s09/prof_stamps -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/s09/prof_stamps_bench.json 2> gpurun_out/s09/prof_stamps.err || exit 1
python tools/region_edges.py gpurun_out/s09/prof_stamps/run_results.db gpurun_out/s09/prof_stamps_bench.json > gpurun_out/s09/region_edges_stamps.json || exit 1
cat gpurun_out/s09/region_edges_stamps.json | grep -v "^  [0-9]"
BENCH_STAMPS=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/s09/stamps_unprofiled.json 2> gpurun_out/s09/stamps_unprofiled.err || exit 1
COMEX_AMD_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s09/prof_1stream -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/s09/prof_1stream_bench.json 2> gpurun_out/s09/prof_1stream.err || exit 1
python tools/dispatch_tail.py gpurun_out/s09/prof_1stream/run_results.db 8 > gpurun_out/s09/dispatch_tail_1stream.json || exit 1
head -40 gpurun_out/s09/dispatch_tail_1stream.json
P="python -u -m pytest -v --timeout 480 --timeout-method thread -m gpu"
timeout -k 10 900 $P tests/test_multiproc.py > gpurun_out/s09/mp.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/s09/mp.log | tail -8; exit $rc
