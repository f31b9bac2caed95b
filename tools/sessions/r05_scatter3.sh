# round-5: GA gather/scatter locating owners twice instead of storing owner + offset per element
set -o pipefail
out=gpurun_out/r05scatter3
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_multiproc.py -m gpu -v -k "scatter or gather or ga_" --timeout 170 --timeout-method thread -p no:cacheprovider > $out/ga_tests.log 2>&1 || { tail -30 $out/ga_tests.log; exit 10; }
tail -3 $out/ga_tests.log
timeout -k 10 200 python3 tools/scatter_bench.py --ga --pairs 65536,1048576,4194304 > $out/ga.jsonl 2> $out/ga.err || exit 12
cat $out/ga.jsonl
