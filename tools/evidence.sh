#!/bin/bash
# tools/evidence.sh TAG -- the measurement evidence of one round, on a GPU box:
#   1. PMC HBM traffic of the H kernel (two separate rocprofv3 --pmc passes)
#   2. bench.py default line (N=1, workload H, CPU baseline included)
#   3. bench lines for the other single-GPU configs (C2, C3, C4, H8200)
#   4. rocprofv3 --kernel-trace --stats of the same bench command (no CPU leg, no
#      host-inclusive block: its zero-copy launches of the same kernel read host memory);
#      merged per-launch busy time from the trace (tools/kernel_union.py), and
#      the same profile with one library stream
# Each GPU step has its own time limit; the first failure ends the script.
# Summaries land in gpurun_out/evidence/ (copy into profiles/<TAG>/ afterwards).
set -euo pipefail
TAG=${1:-r01}
OUT=gpurun_out/evidence
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/pmc_traffic.py --workload H --tag "$TAG" > "$OUT/pmc.log" 2>&1
cp profiles/pmc_latest.json "$OUT/pmc_latest.json"
cp profiles/pmc_"$TAG"*.json "$OUT/" 2>/dev/null || true
timeout -k 10 300 python3 bench.py > "$OUT/bench_H.json" 2> "$OUT/bench_H.err"
for w in C2 C3 C4 H8200; do
    timeout -k 10 300 python3 bench.py --workload "$w" --no-cpu --no-host > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
done
# the profiled run last: a bench started right after rocprofv3 once read half speed
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
    python3 bench.py --no-cpu --no-host > "$OUT/bench_H_prof.json" 2> "$OUT/bench_H_prof.err"
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/rocprofv3_kernel_stats_H.csv" \;
find "$OUT/prof" -name '*kernel_trace.csv' -exec cp {} "$OUT/rocprofv3_kernel_trace_H.csv" \;
python3 tools/kernel_union.py "$OUT/rocprofv3_kernel_trace_H.csv" --json "$OUT/kernel_union_H.json"
# the same with one library stream: per-dispatch AverageNs is then the launch time
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof1" -o bench -- \
    python3 bench.py --no-cpu --no-host --tune streams=1 > "$OUT/bench_H_prof_1stream.json" 2> "$OUT/bench_H_prof_1stream.err"
find "$OUT/prof1" -name '*kernel_stats.csv' -exec cp {} "$OUT/rocprofv3_kernel_stats_H_1stream.csv" \;
echo done
