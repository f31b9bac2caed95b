#!/bin/bash
# round 4 session 2: column kernel rates, C5 full size on the cross-device routes,
# system-scope 2-D kernels on the one-GPU proxy, the driver's N=8 line rehearsed on one GPU
set -o pipefail
O=gpurun_out/r04s02
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest tests/test_gpu_semantics.py -q -s -k "large_overlapping or column_ordered" --timeout 150 --timeout-method thread > $O/cols.log 2>&1; echo "cols rc=$?"; grep -E "column-ordered kernel|passed|failed" $O/cols.log
timeout -k 10 600 python -u -m pytest tests/test_multiproc.py -q -k "c5_full_size or cross_device or owner_host" --timeout 500 --timeout-method thread > $O/c5.log 2>&1; rc=$?; echo "c5 rc=$rc"; tail -3 $O/c5.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
grep -h "C5 M2 exact\|C5 M1 exact" gpurun_out/progress/c5full.log | tail -20
for m in direct_sys packed_sys; do
  case $m in
    direct_sys) a="--src-seg";;
    packed_sys) a="";;
  esac
  COMEX_AMD_PEER_LOADS=all timeout -k 10 120 python bench.py --gpus 2 --exchange $a --steps 300 --no-cpu --no-extras > $O/$m.json 2> $O/$m.err || { echo "$m failed"; tail -20 $O/$m.err; exit 1; }
  python -c "import json,sys;d=json.load(open('$O/$m.json'));print('$m',d['value'],d['hbm_peak_frac'],d['ms_per_step'],d.get('routes'))"
done
timeout -k 10 300 python bench.py --gpus 8 --steps 20 --warmup 5 > $O/n8.json 2> $O/n8.err; echo "n8 rc=$?"
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04s02/n8.json"))
print({k: d.get(k) for k in ("value", "hbm_peak_frac", "topology", "cpu_baseline_note")})
for k, v in d.get("c5", {}).items():
    print(k, json.dumps(v)[:600])
PY
# blocking API: completion flag (default) vs the runtime's sync, interleaved
for i in 1 2; do
  for w in flag sync; do
    COMEX_AMD_BLOCKING_WAIT=$w timeout -k 10 120 python bench.py --steps 100 --warmup 5 --no-cpu > $O/blk_${w}_$i.json 2> $O/blk_${w}_$i.err || { echo "blk $w failed"; tail $O/blk_${w}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$O/blk_${w}_$i.json'));print('blocking $w', d['value'], d['hbm_peak_frac'], d['blocking_api'])"
  done
done
