# round 3 session 28: the C5 exchange check MISMATCH seen once with 8 ranks on one GPU and the
# one-pass lease off (s27): repeat the 8-rank 16384^2 bench rehearsal with lease 0 and 400
# (the default) and with the one-pass route off, and report whose block is wrong and what it reads
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s28
export TMPDIR=/tmp
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --gpus 8 --steps 3 --warmup 1 --warmup-ms 0 --no-cpu --ga-dims 16384 --c5-steps 2 > gpurun_out/s28/$name.json 2> gpurun_out/s28/$name.err || { tail -5 gpurun_out/s28/$name.err; return 1; }
  python -c "
import json; d=json.load(open('gpurun_out/s28/$name.json'))['c5']['exchange_check']
print('$name', {k: (v['result'], v.get('a_rank_with_wrong_elements'), v.get('its_wrong_elements'), v.get('its_first_wrong_value')) for k, v in d.items()})"
  grep -c "hipIpcGetMemHandle" gpurun_out/s28/$name.err || true
}
for i in 1 2 3; do
  run lease0_$i COMEX_AMD_ONE_PASS_LEASE_US=0 || exit 1
  run lease400_$i COMEX_AMD_ONE_PASS_LEASE_US=400 || exit 1
done
run onepass_off COMEX_AMD_ONE_PASS=0 || exit 1
run lease0_noretry COMEX_AMD_ONE_PASS_LEASE_US=0 COMEX_AMD_IPC_RETRY=1 || exit 1
