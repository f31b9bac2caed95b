#!/bin/bash
# round 4 session 4: the role-split LDS column kernel (rates + the column geometries)
set -o pipefail
O=gpurun_out/r04s04
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest tests/test_gpu_semantics.py tests/test_gpu_parity.py -q -s -k "large_overlapping or column_ordered or integer_column or golden or knob" --timeout 150 --timeout-method thread > $O/cols.log 2>&1; echo "cols rc=$?"; grep -E "column-ordered kernel|passed|failed" $O/cols.log | tail -8
