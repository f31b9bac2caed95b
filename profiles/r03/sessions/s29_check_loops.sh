# round 3 session 29: the exchange check repeated (BENCH_CHECK_LOOPS) with 8 ranks on one GPU,
# to reproduce the single MISMATCH of s27: one-pass lease 0 and 400, 8192^2 (fast) and 16384^2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s29
export TMPDIR=/tmp
run() {  # name dims loops env...
  local name=$1 dims=$2 loops=$3; shift 3
  env BENCH_CHECK_LOOPS=$loops "$@" timeout -k 10 500 python -u bench.py --gpus 8 --steps 3 --warmup 1 --warmup-ms 0 --no-cpu --ga-dims $dims --c5-steps 2 > gpurun_out/s29/$name.json 2> gpurun_out/s29/$name.err || { tail -5 gpurun_out/s29/$name.err; return 1; }
  python -c "
import json; d=json.load(open('gpurun_out/s29/$name.json'))['c5']
print('$name', {k: (v['mismatches'], v['loops'], v['first_mismatch'] and {x: v['first_mismatch'].get(x) for x in ('a_rank_with_wrong_elements', 'its_wrong_elements', 'its_first_wrong_value', 'routes_rank')}) for k, v in d['exchange_check_loops'].items()})"
  echo "refusals: $(grep -c hipIpcGetMemHandle gpurun_out/s29/$name.err)"
}
run l0_8k 8192 25 COMEX_AMD_ONE_PASS_LEASE_US=0 || exit 1
run l400_8k 8192 25 || exit 1
run l0_16k 16384 12 COMEX_AMD_ONE_PASS_LEASE_US=0 || exit 1
run l400_16k 16384 12 || exit 1
