# round 3 session 32: is the single exchange-check MISMATCH of s27 tied to the IPC export
# refusals?  30 eight-rank one-GPU rehearsals (16384^2, exchange check x3 per route) with the
# segment cache off and the one-pass lease off (the s27 conditions), then 30 with the defaults;
# count refusals and mismatches per run
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s32
export TMPDIR=/tmp
run() {  # name env...
  local name=$1; shift
  env BENCH_CHECK_LOOPS=2 "$@" timeout -k 10 300 python -u bench.py --gpus 8 --steps 2 --warmup 1 --warmup-ms 0 --no-cpu --ga-dims 16384 --c5-steps 2 > gpurun_out/s32/$name.json 2> gpurun_out/s32/$name.err || { tail -5 gpurun_out/s32/$name.err; return 1; }
  python - "$name" <<'PY'
import json, sys
name = sys.argv[1]
d = json.load(open(f"gpurun_out/s32/{name}.json"))["c5"]
mm = sum(v["result"] != "exact" for v in d["exchange_check"].values()) + sum(v["mismatches"] for v in d["exchange_check_loops"].values())
first = [v for v in d["exchange_check"].values() if v["result"] != "exact"] + [v["first_mismatch"] for v in d["exchange_check_loops"].values() if v["first_mismatch"]]
ref = open(f"gpurun_out/s32/{name}.err").read().count("hipIpcGetMemHandle")
print(name, "refusals", ref, "mismatches", mm, (first[0].get("a_rank_with_wrong_elements"), first[0].get("its_wrong_elements"), first[0].get("its_first_wrong_value")) if first else "")
PY
}
for i in $(seq 1 30); do run off_$i COMEX_AMD_SEGMENT_CACHE_MB=0 COMEX_AMD_ONE_PASS_LEASE_US=0 || exit 1; done
for i in $(seq 1 30); do run on_$i || exit 1; done
