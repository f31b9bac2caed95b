# round 3 session 33: comex_malloc now tags every new segment and every peer checks its fresh
# IPC mapping reads the tags (a stale mapping -> the block is replaced, collectively).  The
# whole GPU suite, then the s32 failing configuration again (segment cache off, one-pass lease
# off, 30 eight-rank runs): refusals, stale mappings caught, mismatches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s33
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -v --timeout 480 --timeout-method thread -m gpu > gpurun_out/s33/gpu_suite.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/s33/gpu_suite.log | head; tail -1 gpurun_out/s33/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
run() {  # name env...
  local name=$1; shift
  env BENCH_CHECK_LOOPS=2 "$@" timeout -k 10 300 python -u bench.py --gpus 8 --steps 2 --warmup 1 --warmup-ms 0 --no-cpu --ga-dims 16384 --c5-steps 2 > gpurun_out/s33/$name.json 2> gpurun_out/s33/$name.err || { tail -5 gpurun_out/s33/$name.err; return 1; }
  python - "$name" <<'PY'
import json, sys
name = sys.argv[1]
d = json.load(open(f"gpurun_out/s33/{name}.json"))["c5"]
mm = sum(v["result"] != "exact" for v in d["exchange_check"].values()) + sum(v["mismatches"] for v in d["exchange_check_loops"].values())
err = open(f"gpurun_out/s33/{name}.err").read()
print(name, "refusals", err.count("hipIpcGetMemHandle"), "stale mappings caught", err.count("not its tags"), "mismatches", mm)
PY
}
for i in $(seq 1 30); do run off_$i COMEX_AMD_SEGMENT_CACHE_MB=0 COMEX_AMD_ONE_PASS_LEASE_US=0 || exit 1; done
