#!/bin/bash
# round 4 final A: the whole GPU suite on the final tree (the driver's command shape)
set -o pipefail
O=gpurun_out/r04final
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?
echo "gpu suite rc=$rc"; tail -n 4 $O/gpu_suite.log
exit $rc
