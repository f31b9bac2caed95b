#!/bin/bash
# round 4 session 6: the vmm segment allocator (private VA window, descriptors over
# sockets) under its own tests, the whole multi-rank suite with it as the allocator, the
# eight-rank campaign of s03 with it, and a driver-shaped N=1 bench line (blocking_api
# through the prototype-free ctypes call)
set -o pipefail
O=gpurun_out/r04s06
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_multiproc.py -q -k "vmm_segments" --timeout 170 --timeout-method thread > $O/vmm.log 2>&1; rc=$?; echo "vmm rc=$rc"; tail -n 3 $O/vmm.log
[ $rc -eq 0 ] || exit $rc
COMEX_AMD_SEGMENT_ALLOC=vmm timeout -k 10 900 python -u -m pytest tests/test_multiproc.py -q -x --timeout 300 --timeout-method thread > $O/mp_vmm.log 2>&1; rc=$?; echo "multiproc under vmm rc=$rc"; tail -n 3 $O/mp_vmm.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err; rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('$O/bench_n1.json'));print(d['value'], d['roofline']['frac'], d.get('blocking_api'))"
# HBM segments from hipMemCreate vs hipMalloc under the HBM-bound kernel: C5 M1 at N=1 (one 8 GiB block)
for alloc in ipc vmm ipc vmm; do
  COMEX_AMD_SEGMENT_ALLOC=$alloc timeout -k 10 200 python bench.py --workload C5 --steps 20 --warmup 3 --no-cpu > $O/c5_$alloc.json 2> $O/c5_$alloc.err || { echo "c5 $alloc failed"; tail -5 $O/c5_$alloc.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c5_$alloc.json'));print('C5 N=1 $alloc', d['value'], d['hbm_peak_frac'])"
done
OUT=$O SKIP_HOSTSEG=1 SKIP_VMMTEST=1 ALLOCS=vmm REPS=${REPS:-8} bash tools/sessions/r04_s03.sh
