# round-5 soak on the final tree (after the small-call, io-vector and stream changes): new seeds,
# the random-descriptor tests, the two-rank random exchange and the random multi-rank programs
set -o pipefail
out=gpurun_out/r05soak2
mkdir -p $out
for s in 7 8 9 10 11 12; do
  GAAMD_FUZZ_SEED=$s timeout -k 10 300 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/fuzz_$s.log 2>&1 || { tail -30 $out/fuzz_$s.log; exit 11; }
  echo "fuzz seed $s: $(tail -1 $out/fuzz_$s.log)"
done
for s in 31 32 33 34 35 36; do
  RDESC_SEED=$s RDESC_CASES=300 timeout -k 10 600 python -u -m pytest tests/test_multiproc.py -m gpu -q -k random_remote_descriptors --timeout 250 --timeout-method thread -p no:cacheprovider > $out/rdesc_$s.log 2>&1 || { tail -30 $out/rdesc_$s.log; exit 12; }
  echo "rdesc seed $s: $(tail -1 $out/rdesc_$s.log)"
done
for s in 41 42 43 44; do
  STRESS_SEED=$s timeout -k 10 600 python -u -m pytest tests/test_multiproc.py -m gpu -q -k "stress_random_programs and not one_pass" --timeout 250 --timeout-method thread -p no:cacheprovider > $out/stress_$s.log 2>&1 || { tail -30 $out/stress_$s.log; exit 13; }
  echo "stress seed $s: $(tail -1 $out/stress_$s.log)"
done
