# round-5: HBM fetch granularity of partial-line access (tools/granule_probe.hip), the
# current short-row rates, and the GPU suite after the knob cleanup
set -o pipefail
out=gpurun_out/r05s3
mkdir -p $out
timeout -k 10 120 ./tools/granule_probe 10 > $out/granule_probe.jsonl 2> $out/granule_probe.err || exit 11
cat $out/granule_probe.jsonl
timeout -k 10 200 python3 tools/shape_sweep.py --rows 32,64,128,256,512,1024,16384 > $out/shape_sweep.jsonl 2> $out/shape_sweep.err || exit 12
cat $out/shape_sweep.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider > $out/gpu_suite.log 2>&1
tail -2 $out/gpu_suite.log
