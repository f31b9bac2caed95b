# run one multi-process worker mode by hand (N ranks on this box), output per
# rank to gpurun_out/mp_<mode>_<rank>.log.  The ranks must share their parent
# (the built-in bootstrap names its shm segment after the parent pid), so the
# time limit wraps this whole script: timeout -k 10 S bash tools/mp_debug.sh MODE N
MODE=${1:-remote}
N=${2:-2}
PORT=$((29600 + RANDOM % 300))
mkdir -p gpurun_out
pids=()
for r in $(seq 0 $((N-1))); do
  RANK=$r WORLD_SIZE=$N LOCAL_RANK=$r MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT COMEX_AMD_JOBID=dbg$PORT COMEX_AMD_STAGING_MB=16 COMEX_AMD_DEBUG=${DBG:-0} \
    python3 -u tests/mp_worker.py $MODE > gpurun_out/mp_${MODE}_$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
exit $rc
