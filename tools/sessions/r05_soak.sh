# round-5 soak: the random-descriptor tests under 6 more seed sets, the two-rank random
# exchange under 6 more seeds per route, the random multi-rank programs under 4 more seeds
set -o pipefail
out=gpurun_out/r05soak
mkdir -p $out
for s in 1 2 3 4 5 6; do
  GAAMD_FUZZ_SEED=$s timeout -k 10 300 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/fuzz_$s.log 2>&1 || { tail -30 $out/fuzz_$s.log; exit 11; }
  echo "fuzz seed $s: $(tail -1 $out/fuzz_$s.log)"
done
for s in 11 12 13 14 15 16; do
  RDESC_SEED=$s RDESC_CASES=300 timeout -k 10 600 python -u -m pytest tests/test_multiproc.py -m gpu -q -k random_remote_descriptors --timeout 250 --timeout-method thread -p no:cacheprovider > $out/rdesc_$s.log 2>&1 || { tail -30 $out/rdesc_$s.log; exit 12; }
  echo "rdesc seed $s: $(tail -1 $out/rdesc_$s.log)"
done
for s in 21 22 23 24; do
  STRESS_SEED=$s timeout -k 10 600 python -u -m pytest tests/test_multiproc.py -m gpu -q -k "stress_random_programs and not one_pass" --timeout 250 --timeout-method thread -p no:cacheprovider > $out/stress_$s.log 2>&1 || { tail -30 $out/stress_$s.log; exit 13; }
  echo "stress seed $s: $(tail -1 $out/stress_$s.log)"
done
