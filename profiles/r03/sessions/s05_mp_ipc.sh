# round 3 session 05: the multi-rank suite after the memory-lock deadlock fix, then six
# two-rank C5 bench runs (the round-2 IPC refusal scenario) with the address history on
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s05
P="python -u -m pytest -v --timeout 480 --timeout-method thread -m gpu"
timeout -k 10 1200 $P tests/test_multiproc.py > gpurun_out/s05/mp.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/s05/mp.log | tail -8; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2 3 4 5 6; do
  env -u RANK -u WORLD_SIZE -u LOCAL_RANK timeout -k 10 240 python -u bench.py --gpus 2 --steps 4 --warmup 1 --warmup-ms 0 --no-cpu \
     --ga-dims 16384 --c5-steps 2 > gpurun_out/s05/c5_2ranks_$i.json 2> gpurun_out/s05/c5_2ranks_$i.err || exit 1
  grep -c "hipIpcGetMemHandle" gpurun_out/s05/c5_2ranks_$i.err || true
  python - <<PY
import json; d = json.load(open("gpurun_out/s05/c5_2ranks_$i.json"))
c = d["c5"]; print("run $i", {k: c["exchange_check"][k]["result"] for k in c["exchange_check"]}, c["M2"]["ms_per_step"], c["M2_src_in_segment"]["ms_per_step"], c["M2"].get("routes"))
PY
done
exit $rc
