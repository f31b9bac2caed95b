#!/bin/bash
# round 4 session 1: GPU suite + column-kernel rates + system-scope load proxy (one GPU)
set -o pipefail
O=gpurun_out/r04s01
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest tests/test_gpu_semantics.py -q -s -k "large_overlapping or column_ordered" --timeout 150 --timeout-method thread > $O/cols.log 2>&1 || { echo "cols failed"; tail -30 $O/cols.log; }
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?
tail -5 $O/gpu_suite.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
# system-scope loads on the one-GPU proxy (every peer treated as another GPU), 2-rank exchange of H
for m in direct_sys packed_sys direct_plain packed_plain; do
  case $m in
    direct_sys) env="COMEX_AMD_PEER_LOADS=all"; a="--src-seg";;
    packed_sys) env="COMEX_AMD_PEER_LOADS=all"; a="";;
    direct_plain) env="COMEX_AMD_PEER_LOADS=off COMEX_AMD_ONE_PASS=0"; a="--src-seg";;
    packed_plain) env="COMEX_AMD_PEER_LOADS=off COMEX_AMD_ONE_PASS=0"; a="";;
  esac
  env $env timeout -k 10 120 python bench.py --gpus 2 --exchange $a --steps 300 --no-cpu --no-extras > $O/$m.json 2> $O/$m.err || { echo "$m failed"; tail -20 $O/$m.err; exit 1; }
  python -c "import json,sys;d=json.load(open('$O/$m.json'));print('$m',d['value'],d['hbm_peak_frac'],d['ms_per_step'],d.get('routes'))"
done
